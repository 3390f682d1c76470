"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY — see loam_oracle.h).

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
PARITY UNPINNED: the reference has no golden vectors and cannot be built here.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

c_i32 = ctypes.c_int32
c_f = ctypes.c_float
c_d = ctypes.c_double
vp = ctypes.c_void_p


class LMStats(ctypes.Structure):
    _fields_ = [("iterations", c_i32), ("successful", c_i32), ("invalid", c_i32),
                ("termination", c_i32), ("initial_cost", c_d), ("final_cost", c_d)]


class MapStats(ctypes.Structure):
    _fields_ = [("optimized", c_i32), ("corner_stack", c_i32), ("surf_stack", c_i32),
                ("corner_map", c_i32), ("surf_map", c_i32), ("corner_num", c_i32 * 2),
                ("surf_num", c_i32 * 2), ("lm", LMStats * 2), ("center", c_i32 * 3),
                ("valid_num", c_i32), ("ms_total", c_d), ("ms_opt", c_d)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libloam_oracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        sig = {
            "oracle_voxel_grid": (c_i32, [vp, c_i32, c_f, vp]),
            "oracle_set_voxel_order": (c_i32, [c_i32]),
            "oracle_std_sort_perm": (c_i32, [vp, c_i32, vp]),
            "oracle_knn": (c_i32, [vp, c_i32, vp, c_i32, c_i32, vp, vp]),
            "oracle_edge_from_nbrs": (c_i32, [vp, vp, vp]),
            "oracle_plane_from_nbrs": (c_i32, [vp, vp, vp]),
            "oracle_lm_solve": (c_i32, [vp, c_i32, vp, c_i32, ctypes.POINTER(LMStats)]),
            "oracle_lm_normal_eq": (c_i32, [vp, c_i32, vp, vp, vp, vp]),
            "oracle_scanreg_create": (vp, [c_i32, c_d]),
            "oracle_scanreg_destroy": (None, [vp]),
            "oracle_scanreg_input": (c_i32, [vp, vp, c_i32, c_i32]),
            "oracle_scanreg_count": (c_i32, [vp, c_i32]),
            "oracle_scanreg_copy": (c_i32, [vp, c_i32, vp]),
            "oracle_scanreg_curvature": (c_i32, [vp, vp, vp]),
            "oracle_scanreg_ms": (c_d, [vp]),
            "oracle_odom_create": (vp, [c_i32]),
            "oracle_odom_destroy": (None, [vp]),
            "oracle_odom_input": (c_i32, [vp, vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32]),
            "oracle_odom_solve": (c_i32, [vp]),
            "oracle_odom_set_prior": (c_i32, [vp, vp, vp]),
            "oracle_odom_output": (c_i32, [vp, vp, vp, vp, vp]),
            "oracle_odom_count": (c_i32, [vp, c_i32]),
            "oracle_odom_copy": (c_i32, [vp, c_i32, vp]),
            "oracle_odom_stats": (c_i32, [vp, vp, ctypes.POINTER(LMStats)]),
            "oracle_odom_ms": (c_d, [vp]),
            "oracle_map_create": (vp, [c_f, c_f]),
            "oracle_map_destroy": (None, [vp]),
            "oracle_map_input": (c_i32, [vp, vp, c_i32, vp, c_i32, vp, c_i32, vp, vp, c_i32]),
            "oracle_map_solve": (c_i32, [vp]),
            "oracle_map_pose": (c_i32, [vp, vp, vp]),
            "oracle_map_get_stats": (c_i32, [vp, ctypes.POINTER(MapStats)]),
            "oracle_map_get_state": (c_i32, [vp, vp, vp, vp]),
            "oracle_map_set_state": (c_i32, [vp, vp, vp, vp]),
            "oracle_map_cube_count": (c_i32, [vp, c_i32, c_i32]),
            "oracle_map_cube_copy": (c_i32, [vp, c_i32, c_i32, vp]),
            "oracle_map_cube_set": (c_i32, [vp, c_i32, c_i32, vp, c_i32]),
            "oracle_map_factor_count": (c_i32, [vp, c_i32]),
            "oracle_map_factors": (c_i32, [vp, c_i32, vp]),
            "oracle_map_round_pose": (c_i32, [vp, c_i32, vp]),
            "oracle_vo_solve": (c_i32, [vp, c_i32, vp, c_i32, ctypes.POINTER(LMStats)]),
            "oracle_vo_normal_eq": (c_i32, [vp, c_i32, vp, vp, vp, vp]),
            "oracle_depth_create": (vp, [vp, vp, vp, c_i32, c_i32, c_i32]),
            "oracle_depth_destroy": (None, [vp]),
            "oracle_depth_process": (c_i32, [vp, vp, c_i32, c_i32]),
            "oracle_depth_count": (c_i32, [vp, c_i32]),
            "oracle_depth_copy": (None, [vp, c_i32, vp]),
            "oracle_depth_buckets": (None, [vp, vp, vp, vp, vp]),
            "oracle_depth_query": (c_d, [vp, vp, c_i32, c_i32, vp]),
            "oracle_depth_ms": (c_d, [vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _f32x4(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim == 1:
        a = a.reshape(-1, 4)
    assert a.shape[1] == 4
    return a


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def voxel_grid(pts, leaf):
    pts = _f32x4(pts)
    out = np.empty_like(pts)
    n = lib().oracle_voxel_grid(_ptr(pts), len(pts), leaf, _ptr(out))
    return out[:n].copy()


def set_voxel_order(order):
    """0: PCL's std::sort order (default), 1: input order; returns the previous setting"""
    return int(lib().oracle_set_voxel_order(int(order)))


class voxel_order:
    """context manager: every oracle VoxelGrid inside uses `order` (0 PCL, 1 input order)"""

    def __init__(self, order):
        self.order = order

    def __enter__(self):
        self.old = set_voxel_order(self.order)
        return self

    def __exit__(self, *exc):
        set_voxel_order(self.old)


def std_sort_perm(keys):
    """the permutation libstdc++ std::sort gives (keys[i], i) compared by key only (u32)"""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.empty(len(k), dtype=np.int32)
    if len(k):
        lib().oracle_std_sort_perm(_ptr(k), len(k), _ptr(perm))
    return perm


def knn(pts, queries, k):
    pts = _f32x4(pts)
    q = _f32x4(queries)
    idx = np.empty((len(q), k), dtype=np.int32)
    d2 = np.empty((len(q), k), dtype=np.float32)
    lib().oracle_knn(_ptr(pts), len(pts), _ptr(q), len(q), k, _ptr(idx), _ptr(d2))
    return idx, d2


def edge_from_nbrs(nbr):
    nbr = _f32x4(nbr)
    a = np.empty(3)
    b = np.empty(3)
    ok = lib().oracle_edge_from_nbrs(_ptr(nbr), _ptr(a), _ptr(b))
    return bool(ok), a, b


def plane_from_nbrs(nbr):
    nbr = _f32x4(nbr)
    n = np.empty(3)
    d = np.empty(1)
    ok = lib().oracle_plane_from_nbrs(_ptr(nbr), _ptr(n), _ptr(d))
    return bool(ok), n, float(d[0])


def lm_solve(factors, x, max_iter=4):
    f = np.ascontiguousarray(factors, dtype=np.float64).reshape(-1, 10)
    x = np.array(x, dtype=np.float64).copy()
    st = LMStats()
    lib().oracle_lm_solve(_ptr(f), len(f), _ptr(x), max_iter, ctypes.byref(st))
    return x, st


def vo_solve(factors, x6, max_iter=100):
    """visual-odometry LM (angles_0to1, t_0to1); factors: (n, 10) type 4 / 5 records"""
    f = np.ascontiguousarray(factors, dtype=np.float64).reshape(-1, 10)
    x = np.array(x6, dtype=np.float64).copy()
    st = LMStats()
    lib().oracle_vo_solve(_ptr(f), len(f), _ptr(x), max_iter, ctypes.byref(st))
    return x, st


def vo_normal_eq(factors, x6):
    f = np.ascontiguousarray(factors, dtype=np.float64).reshape(-1, 10)
    x = np.ascontiguousarray(x6, dtype=np.float64)
    cost = np.empty(1)
    jtj = np.empty(36)
    jtr = np.empty(6)
    m = lib().oracle_vo_normal_eq(_ptr(f), len(f), _ptr(x), _ptr(cost), _ptr(jtj), _ptr(jtr))
    return float(cost[0]), jtj.reshape(6, 6), jtr, m


def lm_normal_eq(factors, x):
    f = np.ascontiguousarray(factors, dtype=np.float64).reshape(-1, 10)
    x = np.ascontiguousarray(x, dtype=np.float64)
    cost = np.empty(1)
    jtj = np.empty(36)
    jtr = np.empty(6)
    m = lib().oracle_lm_normal_eq(_ptr(f), len(f), _ptr(x), _ptr(cost), _ptr(jtj), _ptr(jtr))
    return float(cost[0]), jtj.reshape(6, 6), jtr, m


class ScanRegistration:
    """Oracle ScanRegistration (scan_registration.cpp:144-513)."""
    CLOUDS = ("laserCloud", "cornerPointsSharp", "cornerPointsLessSharp", "surfPointsFlat",
              "surfPointsLessFlat")

    def __init__(self, n_scans=64, minimum_range=5.0):
        self.h = lib().oracle_scanreg_create(n_scans, minimum_range)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_scanreg_destroy(self.h)
            self.h = None

    def input(self, xyz):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        lib().oracle_scanreg_input(self.h, _ptr(xyz), len(xyz), xyz.shape[1])

    def cloud(self, which):
        n = lib().oracle_scanreg_count(self.h, which)
        out = np.empty((n, 4), dtype=np.float32)
        lib().oracle_scanreg_copy(self.h, which, _ptr(out))
        return out

    def output(self):
        return tuple(self.cloud(i) for i in range(5))

    def curvature(self):
        n = lib().oracle_scanreg_count(self.h, 0)
        c = np.empty(n, dtype=np.float32)
        lab = np.empty(n, dtype=np.int32)
        lib().oracle_scanreg_curvature(self.h, _ptr(c), _ptr(lab))
        return c, lab

    @property
    def ms(self):
        return lib().oracle_scanreg_ms(self.h)


class LaserOdometry:
    """Oracle LaserOdometry (laser_odometry.cpp:137-679)."""

    def __init__(self, mapping_skip_frame=1):
        self.h = lib().oracle_odom_create(mapping_skip_frame)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_odom_destroy(self.h)
            self.h = None

    def input(self, full, sharp, less_sharp, flat, less_flat):
        cl = [_f32x4(c) for c in (full, sharp, less_sharp, flat, less_flat)]
        args = []
        for c in cl:
            args += [_ptr(c), len(c)]
        lib().oracle_odom_input(self.h, *args)

    def solve(self):
        lib().oracle_odom_solve(self.h)

    def set_prior(self, q=None, t=None):
        """VO prior (!detach_VO_LO): every outer round starts from it; None clears"""
        if q is None:
            lib().oracle_odom_set_prior(self.h, None, None)
            return
        self._prior = (np.ascontiguousarray(q, dtype=np.float64), np.ascontiguousarray(t, dtype=np.float64))
        lib().oracle_odom_set_prior(self.h, _ptr(self._prior[0]), _ptr(self._prior[1]))

    def output(self):
        q = np.empty(4); t = np.empty(3); qlc = np.empty(4); tlc = np.empty(3)
        skip = lib().oracle_odom_output(self.h, _ptr(q), _ptr(t), _ptr(qlc), _ptr(tlc))
        return q, t, qlc, tlc, bool(skip)

    def cloud(self, which):
        n = lib().oracle_odom_count(self.h, which)
        out = np.empty((n, 4), dtype=np.float32)
        lib().oracle_odom_copy(self.h, which, _ptr(out))
        return out

    def stats(self):
        corr = np.empty(4, dtype=np.int32)
        lm = (LMStats * 2)()
        lib().oracle_odom_stats(self.h, _ptr(corr), lm)
        return corr, [lm[0], lm[1]]

    @property
    def ms(self):
        return lib().oracle_odom_ms(self.h)


class LaserMapping:
    """Oracle LaserMapping (laser_mapping.cpp:147-814)."""
    N_CUBES = 21 * 21 * 11

    def __init__(self, line_res=0.4, plane_res=0.8):
        self.h = lib().oracle_map_create(line_res, plane_res)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_map_destroy(self.h)
            self.h = None

    def input(self, corner, surf, full, q_wodom, t_wodom, skip=False):
        c, s = _f32x4(corner), _f32x4(surf)
        f = _f32x4(full) if full is not None else np.zeros((0, 4), np.float32)
        q = np.ascontiguousarray(q_wodom, dtype=np.float64)
        t = np.ascontiguousarray(t_wodom, dtype=np.float64)
        lib().oracle_map_input(self.h, _ptr(c), len(c), _ptr(s), len(s), _ptr(f), len(f),
                               _ptr(q), _ptr(t), int(skip))

    def solve(self):
        lib().oracle_map_solve(self.h)

    def pose(self):
        q = np.empty(4); t = np.empty(3)
        lib().oracle_map_pose(self.h, _ptr(q), _ptr(t))
        return q, t

    def stats(self):
        st = MapStats()
        lib().oracle_map_get_stats(self.h, ctypes.byref(st))
        return st

    def get_state(self):
        cen = np.empty(3, dtype=np.int32); q = np.empty(4); t = np.empty(3)
        lib().oracle_map_get_state(self.h, _ptr(cen), _ptr(q), _ptr(t))
        return cen, q, t

    def set_state(self, cen, q, t):
        cen = np.ascontiguousarray(cen, dtype=np.int32)
        q = np.ascontiguousarray(q, dtype=np.float64)
        t = np.ascontiguousarray(t, dtype=np.float64)
        lib().oracle_map_set_state(self.h, _ptr(cen), _ptr(q), _ptr(t))

    def cube(self, which, cube):
        n = lib().oracle_map_cube_count(self.h, which, cube)
        out = np.empty((n, 4), dtype=np.float32)
        if n:
            lib().oracle_map_cube_copy(self.h, which, cube, _ptr(out))
        return out

    def set_cube(self, which, cube, pts):
        pts = _f32x4(pts)
        lib().oracle_map_cube_set(self.h, which, cube, _ptr(pts), len(pts))

    def cubes(self, which):
        """dict cube -> points for all non-empty cubes"""
        out = {}
        for c in range(self.N_CUBES):
            if lib().oracle_map_cube_count(self.h, which, c) > 0:
                out[c] = self.cube(which, c)
        return out

    def factors(self, rnd):
        n = lib().oracle_map_factor_count(self.h, rnd)
        out = np.empty((n, 10))
        if n:
            lib().oracle_map_factors(self.h, rnd, _ptr(out))
        return out

    def round_pose(self, rnd):
        x = np.empty(7)
        lib().oracle_map_round_pose(self.h, rnd, _ptr(x))
        return x


class PointCloudUtil:
    """Oracle depth association (visual_odometry point_cloud_util.cpp:183-487)."""

    def __init__(self, cam_T_velo, rect0_T_cam, P_rect0, grid=5, img_w=1242, img_h=375):
        self._m = [np.ascontiguousarray(cam_T_velo, dtype=np.float32).reshape(16),
                   np.ascontiguousarray(rect0_T_cam, dtype=np.float32).reshape(16),
                   np.ascontiguousarray(P_rect0, dtype=np.float32).reshape(12)]
        self.h = lib().oracle_depth_create(_ptr(self._m[0]), _ptr(self._m[1]), _ptr(self._m[2]), grid, img_w, img_h)
        self.grid = grid
        self.new_w = int(np.ceil(np.float32(img_w) / np.float32(grid)))
        self.new_h = int(np.ceil(np.float32(img_h) / np.float32(grid)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_depth_destroy(self.h)
            self.h = None

    def process(self, xyz):
        """projectPointCloud + downsamplePointCloud (visual_odometry.cpp:201-214)"""
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        return lib().oracle_depth_process(self.h, _ptr(xyz), len(xyz), xyz.shape[1])

    def cloud(self, which):
        """0: point_cloud_2d, 1: point_cloud_2d_dnsp, (n, 3) float32"""
        n = lib().oracle_depth_count(self.h, which)
        out = np.empty((n, 3), dtype=np.float32)
        if n:
            lib().oracle_depth_copy(self.h, which, _ptr(out))
        return out

    def buckets(self):
        n = self.new_w * self.new_h
        bx, by, bd = (np.empty(n, dtype=np.float32) for _ in range(3))
        bc = np.empty(n, dtype=np.int32)
        lib().oracle_depth_buckets(self.h, _ptr(bx), _ptr(by), _ptr(bd), _ptr(bc))
        return bx, by, bd, bc

    def query(self, xy, radius=2):
        xy = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
        out = np.empty(len(xy), dtype=np.float32)
        ms = lib().oracle_depth_query(self.h, _ptr(xy), len(xy), radius, _ptr(out)) if len(xy) else 0.0
        self.query_ms = ms
        return out

    @property
    def ms(self):
        return lib().oracle_depth_ms(self.h)
