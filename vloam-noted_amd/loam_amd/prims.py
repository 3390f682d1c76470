"""Standalone HIP primitives behind the mapping stage (C-ABI, include/loam_core.h).

Same argument meaning as the pieces of the reference they replace:
  voxel_grid   pcl::VoxelGrid<PointXYZI>::filter (laser_mapping.cpp:492-500, :795-808), a voxel's
               points summed in input order (the mapper's kernels)
  voxel_grid_pcl  the same with PCL's summation order (scan_registration.cpp:497-501's kernel)
  sort_perm    std::sort's permutation under a key-only comparator (stdsort.h)
  knn_radius   pcl::KdTreeFLANN::nearestKSearch restricted to d2 < radius2 (:554, :633)
  lm_solve     ceres::Solve with the reference's options (:709-717) on factor records
  lm_normal_equations  cost, J^T J, J^T r at x (Huber-corrected, local 6-dof)
Every call runs on the GPU; there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, f32x4, lib, ptr


def voxel_grid(pts, leaf, device=0):
    pts = f32x4(pts)
    out = np.empty_like(pts)
    n = _core.c_i32()
    check(lib().loam_voxel_grid(device, ptr(pts), len(pts), float(leaf), ptr(out), ctypes.byref(n)))
    return out[: n.value].copy()


def voxel_grid_pcl(pts, leaf, device=0):
    """VoxelGrid with PCL's own within-voxel summation order (std::sort permutation)"""
    pts = f32x4(pts)
    out = np.empty_like(pts)
    n = _core.c_i32()
    check(lib().loam_voxel_grid_pcl(device, ptr(pts), len(pts), float(leaf), ptr(out), ctypes.byref(n)))
    return out[: n.value].copy()


def sort_perm(keys, n_waves=16, device=0):
    """the libstdc++ std::sort permutation of (keys[i], i) compared by key, computed on the GPU"""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.empty(len(k), dtype=np.int32)
    check(lib().loam_sort_perm(device, ptr(k), len(k), int(n_waves), ptr(perm)))
    return perm


def voxel_merge(fixed, added, leaf, device=0):
    """VoxelGrid of fixed ++ added, `fixed` being a VoxelGrid fixed point; returns (out, merged)"""
    c, a = f32x4(fixed), f32x4(added)
    out = np.empty((len(c) + len(a), 4), dtype=np.float32)
    n, m = _core.c_i32(), _core.c_i32()
    check(lib().loam_voxel_merge(device, ptr(c), len(c), ptr(a), len(a), float(leaf), ptr(out),
                                 ctypes.byref(n), ctypes.byref(m)))
    return out[: n.value].copy(), bool(m.value)


def knn_radius(pts, queries, k=5, radius2=1.0, device=0):
    pts, q = f32x4(pts), f32x4(queries)
    idx = np.empty((len(q), k), dtype=np.int32)
    d2 = np.empty((len(q), k), dtype=np.float32)
    check(lib().loam_knn_radius(device, ptr(pts), len(pts), ptr(q), len(q), k, float(radius2),
                                ptr(idx), ptr(d2)))
    return idx, d2


def _factors(f):
    f = np.ascontiguousarray(f, dtype=np.float64)
    return f.reshape(-1, 10)


def lm_solve(factors, x, max_iterations=4, device=0):
    f = _factors(factors)
    x = np.array(x, dtype=np.float64).copy()
    st = _core.LMStats()
    check(lib().loam_lm_solve(device, ptr(f), len(f), ptr(x), max_iterations, ctypes.byref(st)))
    return x, st


def lm_normal_equations(factors, x, device=0):
    f = _factors(factors)
    x = np.ascontiguousarray(x, dtype=np.float64)
    cost = np.empty(1)
    jtj = np.empty(36)
    jtr = np.empty(6)
    check(lib().loam_lm_normal_equations(device, ptr(f), len(f), ptr(x), ptr(cost), ptr(jtj), ptr(jtr)))
    return float(cost[0]), jtj.reshape(6, 6), jtr
