"""LaserMapping on MI355X — host mirror of the reference interface.

Mirrors ``vloam::LaserMapping`` (src/lidar_odometry_mapping/include/lidar_odometry_mapping/
laser_mapping.h:85-100): ``init`` / ``reset`` / ``input`` / ``solveMapping`` / ``output``,
same argument meaning (clouds are (n, 4) float32 x, y, z, intensity = pcl::PointXYZI;
quaternions xyzw like ``parameters[0..3]``).  The ROS publishers are not part of the core:
``output`` returns what ``publish`` would send (laser_mapping.cpp:816-911).

``BatchMapper`` exposes the batched form: n independent streams per handle, one set of
kernel launches per ``solve`` for all of them.
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, f32x4, lib, ptr

N_CUBES = 21 * 21 * 11


class BatchMapper:
    """n_streams independent LaserMapping streams.  With ``comm`` (loam_amd.comm.Comm) every
    stream is sharded over the comm's ranks: this object is one rank's share, every rank
    feeds identical inputs and calls ``solve`` together (include/loam_core.h)."""

    def __init__(self, n_streams=1, device=0, params=None, comm=None, **param_overrides):
        self.params = params if params is not None else _core.default_params(**param_overrides)
        self.n_streams = n_streams
        self.device = device
        self.comm = comm  # kept alive as long as the mapper
        h = ctypes.c_void_p()
        if comm is None:
            check(lib().loam_mapper_create(ctypes.byref(self.params), device, n_streams, ctypes.byref(h)))
        else:
            check(lib().loam_mapper_create_sharded(ctypes.byref(self.params), device, n_streams, comm.h,
                                                   ctypes.byref(h)))
        self.h = h

    def point_owner(self, which, xyz):
        """rank storing map point xyz of map `which` (0 corner, 1 surf) under this sharding"""
        leaf = self.params.mapping_line_resolution if which == 0 else self.params.mapping_plane_resolution
        return shard_owner(xyz, leaf, self.comm.size if self.comm is not None else 1)


    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_mapper_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(lib().loam_mapper_reset(self.h))

    def input(self, stream, corner, surf, q_wodom, t_wodom, skip_frame=False):
        c, s = f32x4(corner), f32x4(surf)
        q = np.ascontiguousarray(q_wodom, dtype=np.float64)
        t = np.ascontiguousarray(t_wodom, dtype=np.float64)
        check(lib().loam_mapper_input(self.h, stream, ptr(c), len(c), ptr(s), len(s),
                                      ptr(q), ptr(t), int(skip_frame)))

    def input_device(self, stream, corner_ptr, n_corner, surf_ptr, n_surf, q_wodom, t_wodom,
                     skip_frame=False):
        q = np.ascontiguousarray(q_wodom, dtype=np.float64)
        t = np.ascontiguousarray(t_wodom, dtype=np.float64)
        check(lib().loam_mapper_input_device(self.h, stream, corner_ptr, n_corner, surf_ptr,
                                             n_surf, ptr(q), ptr(t), int(skip_frame)))

    def input_device_batch(self, streams, corner_ptrs, n_corner, surf_ptrs, n_surf, q_wodom, t_wodom):
        """n streams at once: arrays of stream ids, device pointers (uint64) and sizes"""
        st = np.ascontiguousarray(streams, dtype=np.int32)
        cp = np.ascontiguousarray(corner_ptrs, dtype=np.uint64)
        cn = np.ascontiguousarray(n_corner, dtype=np.int32)
        sp = np.ascontiguousarray(surf_ptrs, dtype=np.uint64)
        sn = np.ascontiguousarray(n_surf, dtype=np.int32)
        q = np.ascontiguousarray(q_wodom, dtype=np.float64).reshape(-1, 4)
        t = np.ascontiguousarray(t_wodom, dtype=np.float64).reshape(-1, 3)
        check(lib().loam_mapper_input_device_batch(self.h, len(st), ptr(st), ptr(cp), ptr(cn), ptr(sp),
                                                   ptr(sn), ptr(q), ptr(t)))

    @staticmethod
    def batch_args(streams, corner_ptrs, n_corner, surf_ptrs, n_surf, q_wodom, t_wodom):
        """input_device_batch's arrays made contiguous once, with their addresses: a tuple for
        input_device_batch_args (frame loops that replay prepared inputs skip the per-call numpy
        conversions; the arrays are kept alive in the tuple)"""
        arrs = (np.ascontiguousarray(streams, dtype=np.int32), np.ascontiguousarray(corner_ptrs, dtype=np.uint64),
                np.ascontiguousarray(n_corner, dtype=np.int32), np.ascontiguousarray(surf_ptrs, dtype=np.uint64),
                np.ascontiguousarray(n_surf, dtype=np.int32),
                np.ascontiguousarray(q_wodom, dtype=np.float64).reshape(-1, 4),
                np.ascontiguousarray(t_wodom, dtype=np.float64).reshape(-1, 3))
        return (len(arrs[0]),) + tuple(ptr(a) for a in arrs) + (arrs,)

    def input_device_batch_args(self, args):
        """input_device_batch from batch_args' tuple"""
        check(lib().loam_mapper_input_device_batch(self.h, *args[:8]))

    def stack(self, stream, which):
        """laserCloudCornerStack (0) / laserCloudSurfStack (1) of the last solve, (n, 4) float32"""
        n = check(lib().loam_mapper_stack_copy(self.h, stream, which, None, 0))
        out = np.empty((n, 4), dtype=np.float32)
        if n:
            check(lib().loam_mapper_stack_copy(self.h, stream, which, ptr(out), n))
        return out

    def lm_path(self):
        """the LM schedule of this handle: 0 two launches per iteration, 1 persistent round, 2 in-process
        group round, 3 persistent round with cross-process IPC peer slots (loam_mapper_lm_path)"""
        return check(lib().loam_mapper_lm_path(self.h))

    def total_iterations(self):
        """sum of the LM iterations of every stream in the last solve"""
        return check(lib().loam_mapper_total_iterations(self.h))

    def stats_all(self):
        out = (_core.MapStats * self.n_streams)()
        check(lib().loam_mapper_stats_all(self.h, out, self.n_streams))
        return list(out)

    def debug_counters(self, reset=False):
        out = np.zeros(96, dtype=np.uint64)  # LOAM_DEBUG_COUNTERS
        check(lib().loam_mapper_debug_counters(self.h, ptr(out), len(out), int(reset)))
        return out

    def solve(self):
        check(lib().loam_mapper_solve(self.h))

    def solve_async(self):
        """enqueue solveMapping for the streams with an input and return (include/loam_core.h).
        With a frame already in flight the new one is queued behind it (on the device for
        graph-path handles): give frame f + 1 and call this before waiting for frame f."""
        check(lib().loam_mapper_solve_async(self.h))

    def wait(self):
        """finish the oldest frame in the queue; pose / stats / get_state then report it"""
        check(lib().loam_mapper_wait(self.h))

    def solve_pose(self):
        """solve() that returns at the frame's pose: the insertion and re-VoxelGrid of the cubes
        finish beside the next frame (include/loam_core.h loam_mapper_solve_pose)"""
        check(lib().loam_mapper_solve_pose(self.h))

    def prefetch(self):
        """queue the stack VoxelGrids of the pending inputs now, beside a frame in flight"""
        check(lib().loam_mapper_prefetch(self.h))

    def set_profiling(self, enable=True):
        check(lib().loam_mapper_set_profiling(self.h, int(enable)))

    def kernel_times(self):
        kt = _core.KernelTimes()
        check(lib().loam_mapper_kernel_times(self.h, ctypes.byref(kt)))
        return {name: dict(ms=kt.ms[i], launches=int(kt.launches[i]), bytes=kt.bytes[i])
                for i, name in enumerate(_core.KFAM)}

    def reset_kernel_times(self):
        check(lib().loam_mapper_reset_kernel_times(self.h))

    def pose(self, stream=0):
        q = np.empty(4)
        t = np.empty(3)
        check(lib().loam_mapper_pose(self.h, stream, ptr(q), ptr(t)))
        return q, t

    def stats(self, stream=0):
        st = _core.MapStats()
        check(lib().loam_mapper_stats(self.h, stream, ctypes.byref(st)))
        return st

    def get_state(self, stream=0):
        cen = np.empty(3, dtype=np.int32)
        q = np.empty(4)
        t = np.empty(3)
        check(lib().loam_mapper_get_state(self.h, stream, ptr(cen), ptr(q), ptr(t)))
        return cen, q, t

    def set_state(self, stream, cen, q_wmap_wodom, t_wmap_wodom):
        cen = np.ascontiguousarray(cen, dtype=np.int32)
        q = np.ascontiguousarray(q_wmap_wodom, dtype=np.float64)
        t = np.ascontiguousarray(t_wmap_wodom, dtype=np.float64)
        check(lib().loam_mapper_set_state(self.h, stream, ptr(cen), ptr(q), ptr(t)))

    def cube(self, stream, which, cube):
        n = check(lib().loam_mapper_cube_count(self.h, stream, which, cube))
        out = np.empty((n, 4), dtype=np.float32)
        if n:
            check(lib().loam_mapper_cube_copy(self.h, stream, which, cube, ptr(out)))
        return out

    def set_cube(self, stream, which, cube, pts):
        pts = f32x4(pts)
        check(lib().loam_mapper_cube_set(self.h, stream, which, cube, ptr(pts), len(pts)))

    def map_cloud(self, stream=0):
        """laserCloudMap of the /laser_cloud_map publisher (laser_mapping.cpp:884-899)"""
        n = check(lib().loam_mapper_map_copy(self.h, stream, None, 0))
        out = np.empty((n, 4), dtype=np.float32)
        if n:
            check(lib().loam_mapper_map_copy(self.h, stream, ptr(out), n))
        return out

    def register_cloud(self, stream, cloud):
        """laserCloudFullRes in the map frame with the current pose (laser_mapping.cpp:901-905)"""
        c = f32x4(cloud)
        out = np.empty_like(c)
        check(lib().loam_mapper_register_cloud(self.h, stream, ptr(c), len(c), ptr(out)))
        return out

    def cubes(self, stream, which):
        out = {}
        for c in range(N_CUBES):
            if check(lib().loam_mapper_cube_count(self.h, stream, which, c)) > 0:
                out[c] = self.cube(stream, which, c)
        return out


class LaserMapping:
    """Single-stream drop-in with the reference method names."""

    def __init__(self, device=0, **param_overrides):
        self._m = BatchMapper(1, device, **param_overrides)
        self._skip = False

    def init(self):
        self._m.reset()

    def reset(self):  # laser_mapping.cpp:132-136 — per-frame submap counters only
        pass

    def input(self, laserCloudCornerLast, laserCloudSurfLast, laserCloudFullRes, q_wodom_curr,
              t_wodom_curr, skip_frame=False):
        self._skip = bool(skip_frame)
        self._m.input(0, laserCloudCornerLast, laserCloudSurfLast, q_wodom_curr, t_wodom_curr,
                      skip_frame)

    def solveMapping(self):
        self._m.solve()

    def output(self):
        return self._m.pose(0)

    def stats(self):
        return self._m.stats(0)

    @property
    def batch(self):
        return self._m


def shard_owner(xyz, leaf, nrank):
    """owner rank of a map point (4 m voxel-aligned blocks, include/loam_core.h)"""
    p = np.ascontiguousarray(np.asarray(xyz, dtype=np.float32)[:3])
    return check(lib().loam_shard_owner(ptr(p), float(leaf), int(nrank)))
