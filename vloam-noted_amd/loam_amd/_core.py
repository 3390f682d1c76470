"""ctypes binding of libloam_core.so (include/loam_core.h).

The product path: every call goes to the HIP kernels through the C-ABI.  There is no CPU
fallback — if the library or a gfx950 device is missing, calls raise ``LoamError``.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LOAM_CORE_LIB: an alternative build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("LOAM_CORE_LIB") or os.path.join(_HERE, "_lib", "libloam_core.so")

c_i32 = ctypes.c_int32
c_f = ctypes.c_float
c_d = ctypes.c_double
vp = ctypes.c_void_p

LOAM_OK = 0
ERRORS = {-1: "LOAM_ERR_ARG", -2: "LOAM_ERR_HIP", -3: "LOAM_ERR_CAPACITY", -4: "LOAM_ERR_STATE",
          -5: "LOAM_ERR_NODEVICE", -6: "LOAM_ERR_SYNC", -7: "LOAM_ERR_EARLIER"}


class LoamError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"{ERRORS.get(rc, rc)}: {msg}")
        self.rc = rc


class Params(ctypes.Structure):
    _fields_ = [("scan_line", c_i32), ("minimum_range", c_d), ("mapping_skip_frame", c_i32),
                ("map_pub_number", c_i32), ("mapping_line_resolution", c_d),
                ("mapping_plane_resolution", c_d), ("detach_vo_lo", c_i32),
                ("verbose_level", c_i32), ("max_input_points", c_i32),
                ("max_map_points", c_i32), ("max_submap_points", c_i32), ("exact_voxel_order", c_i32)]


class LMStats(ctypes.Structure):
    _fields_ = [("iterations", c_i32), ("successful", c_i32), ("invalid", c_i32),
                ("termination", c_i32), ("initial_cost", c_d), ("final_cost", c_d)]


class MapStats(ctypes.Structure):
    _fields_ = [("optimized", c_i32), ("corner_stack", c_i32), ("surf_stack", c_i32),
                ("corner_map", c_i32), ("surf_map", c_i32), ("corner_num", c_i32 * 2),
                ("surf_num", c_i32 * 2), ("lm", LMStats * 2), ("center", c_i32 * 3),
                ("valid_num", c_i32), ("ms_total", c_d), ("ms_opt", c_d), ("queued", c_i32),
                ("rerun", c_i32)]


class OdomStats(ctypes.Structure):
    _fields_ = [("corner_num", c_i32 * 2), ("surf_num", c_i32 * 2), ("lm", LMStats * 2),
                ("n_corner_last", c_i32), ("n_surf_last", c_i32), ("ms", c_d)]


class DepthParams(ctypes.Structure):
    _fields_ = [("cam_T_velo", c_f * 16), ("rect0_T_cam", c_f * 16), ("P_rect0", c_f * 12),
                ("grid", c_i32), ("img_width", c_i32), ("img_height", c_i32), ("max_points", c_i32)]


KFAM = ("stack_voxelgrid", "submap_hash_build", "correspondence", "lm_pass", "insert",
        "cube_revoxel", "other")


class KernelTimes(ctypes.Structure):
    _fields_ = [("ms", c_d * 8), ("launches", ctypes.c_int64 * 8), ("bytes", c_d * 8)]


# name -> (restype, argtypes); must cover every function declared in include/loam_core.h
SIGNATURES = {
    "loam_params_default": (None, [ctypes.POINTER(Params)]),
    "loam_last_error": (ctypes.c_char_p, []),
    "loam_version": (c_i32, []),
    "loam_scanreg_create": (c_i32, [ctypes.POINTER(Params), c_i32, ctypes.POINTER(vp)]),
    "loam_scanreg_destroy": (c_i32, [vp]),
    "loam_scanreg_input": (c_i32, [vp, vp, c_i32, c_i32]),
    "loam_scanreg_input_device": (c_i32, [vp, vp, c_i32, c_i32]),
    "loam_scanreg_host_buffer": (c_i32, [vp, ctypes.POINTER(vp), ctypes.POINTER(c_i32)]),
    "loam_scanreg_input_async": (c_i32, [vp, vp, c_i32, c_i32]),
    "loam_scanreg_wait": (c_i32, [vp]),
    "loam_scanreg_counts": (c_i32, [vp, vp]),
    "loam_scanreg_copy": (c_i32, [vp, c_i32, vp, c_i32]),
    "loam_scanreg_device_ptr": (c_i32, [vp, c_i32, ctypes.POINTER(vp)]),
    "loam_scanreg_curvature": (c_i32, [vp, vp, vp, c_i32]),
    "loam_scanreg_ms": (c_d, [vp]),
    "loam_scanreg_debug_counters": (c_i32, [vp, vp, c_i32, c_i32]),
    "loam_scanreg_create_batch": (c_i32, [ctypes.POINTER(Params), c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_scanreg_input_batch": (c_i32, [vp, c_i32, vp, vp, c_i32, c_i32]),
    "loam_scanreg_frame_counts": (c_i32, [vp, c_i32, vp]),
    "loam_scanreg_frame_device_ptr": (c_i32, [vp, c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_scanreg_frame_copy": (c_i32, [vp, c_i32, c_i32, vp, c_i32]),
    "loam_odometry_create": (c_i32, [ctypes.POINTER(Params), c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_odometry_destroy": (c_i32, [vp]),
    "loam_odometry_reset": (c_i32, [vp]),
    "loam_odometry_input": (c_i32, [vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32]),
    "loam_odometry_input_device": (c_i32, [vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32, vp, c_i32]),
    "loam_odometry_solve": (c_i32, [vp]),
    "loam_odometry_set_prior": (c_i32, [vp, c_i32, vp, vp]),
    "loam_odometry_output": (c_i32, [vp, c_i32, vp, vp, vp, vp, ctypes.POINTER(c_i32)]),
    "loam_odometry_last_cloud": (c_i32, [vp, c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_odometry_copy_last": (c_i32, [vp, c_i32, c_i32, vp, c_i32]),
    "loam_odometry_stats": (c_i32, [vp, c_i32, ctypes.POINTER(OdomStats)]),
    "loam_mapper_create": (c_i32, [ctypes.POINTER(Params), c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_mapper_destroy": (c_i32, [vp]),
    "loam_mapper_reset": (c_i32, [vp]),
    "loam_mapper_input": (c_i32, [vp, c_i32, vp, c_i32, vp, c_i32, vp, vp, c_i32]),
    "loam_mapper_input_device": (c_i32, [vp, c_i32, vp, c_i32, vp, c_i32, vp, vp, c_i32]),
    "loam_mapper_input_device_batch": (c_i32, [vp, c_i32, vp, vp, vp, vp, vp, vp, vp]),
    "loam_mapper_stats_all": (c_i32, [vp, vp, c_i32]),
    "loam_mapper_total_iterations": (ctypes.c_int64, [vp]),
    "loam_mapper_lm_path": (c_i32, [vp]),
    "loam_mapper_solve": (c_i32, [vp]),
    "loam_mapper_solve_async": (c_i32, [vp]),
    "loam_mapper_wait": (c_i32, [vp]),
    "loam_mapper_solve_pose": (c_i32, [vp]),
    "loam_mapper_prefetch": (c_i32, [vp]),
    "loam_mapper_debug_counters": (c_i32, [vp, vp, c_i32, c_i32]),
    "loam_mapper_pose": (c_i32, [vp, c_i32, vp, vp]),
    "loam_mapper_set_profiling": (c_i32, [vp, c_i32]),
    "loam_mapper_kernel_times": (c_i32, [vp, ctypes.POINTER(KernelTimes)]),
    "loam_mapper_reset_kernel_times": (c_i32, [vp]),
    "loam_mapper_stats": (c_i32, [vp, c_i32, ctypes.POINTER(MapStats)]),
    "loam_mapper_get_state": (c_i32, [vp, c_i32, vp, vp, vp]),
    "loam_mapper_set_state": (c_i32, [vp, c_i32, vp, vp, vp]),
    "loam_mapper_cube_count": (c_i32, [vp, c_i32, c_i32, c_i32]),
    "loam_mapper_cube_copy": (c_i32, [vp, c_i32, c_i32, c_i32, vp]),
    "loam_mapper_stack_copy": (c_i32, [vp, c_i32, c_i32, vp, c_i32]),
    "loam_mapper_cube_set": (c_i32, [vp, c_i32, c_i32, c_i32, vp, c_i32]),
    "loam_mapper_map_copy": (c_i32, [vp, c_i32, vp, ctypes.c_int64]),
    "loam_mapper_register_cloud": (c_i32, [vp, c_i32, vp, c_i32, vp]),
    "loam_mapper_register_cloud_device": (c_i32, [vp, c_i32, vp, c_i32, vp]),
    "loam_comm_create": (c_i32, [c_i32, c_i32, vp, ctypes.POINTER(vp)]),
    "loam_comm_rccl_unique_id": (c_i32, [vp]),
    "loam_comm_create_rccl": (c_i32, [c_i32, c_i32, vp, c_i32, ctypes.POINTER(vp)]),
    "loam_comm_create_local": (c_i32, [c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_comm_destroy": (c_i32, [vp]),
    "loam_comm_allreduce_sum": (c_i32, [vp, vp, ctypes.c_int64, c_i32, vp]),
    "loam_comm_allgather": (c_i32, [vp, vp, vp, ctypes.c_int64, vp]),
    "loam_mapper_create_sharded": (c_i32, [ctypes.POINTER(Params), c_i32, c_i32, vp, ctypes.POINTER(vp)]),
    "loam_shard_owner": (c_i32, [vp, c_f, c_i32]),
    "loam_depth_params_default": (None, [ctypes.POINTER(DepthParams)]),
    "loam_depth_create": (c_i32, [ctypes.POINTER(DepthParams), c_i32, c_i32, ctypes.POINTER(vp)]),
    "loam_depth_destroy": (c_i32, [vp]),
    "loam_depth_input": (c_i32, [vp, c_i32, vp, c_i32, c_i32]),
    "loam_depth_input_device": (c_i32, [vp, c_i32, vp, c_i32, c_i32]),
    "loam_depth_process": (c_i32, [vp]),
    "loam_depth_counts": (c_i32, [vp, c_i32, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]),
    "loam_depth_copy": (c_i32, [vp, c_i32, c_i32, vp, c_i32]),
    "loam_depth_buckets": (c_i32, [vp, c_i32, vp, vp, vp, vp]),
    "loam_depth_query": (c_i32, [vp, c_i32, vp, vp, c_i32, vp]),
    "loam_depth_query_device": (c_i32, [vp, c_i32, vp, vp, c_i32, vp]),
    "loam_depth_ms": (c_d, [vp]),
    "loam_vo_solve": (c_i32, [c_i32, c_i32, vp, vp, vp, c_i32, vp]),
    "loam_lm_solve": (c_i32, [c_i32, vp, c_i32, vp, c_i32, ctypes.POINTER(LMStats)]),
    "loam_lm_normal_equations": (c_i32, [c_i32, vp, c_i32, vp, vp, vp, vp]),
    "loam_voxel_grid": (c_i32, [c_i32, vp, c_i32, c_f, vp, ctypes.POINTER(c_i32)]),
    "loam_voxel_grid_pcl": (c_i32, [c_i32, vp, c_i32, c_f, vp, ctypes.POINTER(c_i32)]),
    "loam_sort_perm": (c_i32, [c_i32, vp, c_i32, c_i32, vp]),
    "loam_voxel_merge": (c_i32, [c_i32, vp, c_i32, vp, c_i32, c_f, vp, ctypes.POINTER(c_i32),
                                 ctypes.POINTER(c_i32)]),
    "loam_knn_radius": (c_i32, [c_i32, vp, c_i32, vp, c_i32, c_i32, c_f, vp, vp]),
}

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise LoamError(-5, f"{LIB_PATH} not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("LOAM_CORE_LIB") and not hasattr(L, name):
                continue  # an A/B build of an older tree: entry points added since stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc):
    if rc < 0:
        raise LoamError(rc, lib().loam_last_error().decode())
    return rc


def default_params(**kw):
    p = Params()
    lib().loam_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def f32x4(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim == 1:
        a = a.reshape(-1, 4)
    if a.shape[1] != 4:
        raise ValueError("points must be (n, 4) float32: x, y, z, intensity")
    return a


def ptr(a):
    return a.ctypes.data if a is not None and a.size else None
