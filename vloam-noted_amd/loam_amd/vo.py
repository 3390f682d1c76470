"""Visual-odometry pose solve on MI355X — host side of VisualOdometry::solveNlsAll
(src/visual_odometry/src/visual_odometry.cpp:304-509).

``vo_factors`` builds the residual blocks of one frame pair the way the reference does
(:346-493): a match whose previous point has a depth (``queryDepth`` > 0) becomes a
CostFunctor32 (3D point in rectified camera 0 -> normalised image point), otherwise a
CostFunctor22 (epipolar).  ``solve`` runs any number of such problems on the device (one
workgroup per problem, every Ceres iteration on the GPU): HuberLoss(0.1), TR-LM, DENSE_QR,
max_num_iterations = 100 (:70-74).
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, lib, ptr

CF32, CF22 = 4, 5


def vo_factors(prev_xy, curr_xy, depth0, P_rect0):
    """factor records (n, 10) of one frame pair.  prev_xy / curr_xy: matched pixel coordinates
    (the reference stores them in ints, :346); depth0: queryDepth of the previous points.
    The 3x3 solves with P_rect0.leftCols(3) (:421-424, colPivHouseholderQr in float) are done
    in float64 and rounded to float32 here: the records match the reference to float rounding,
    not bit for bit."""
    K = np.asarray(P_rect0, dtype=np.float64)[:, :3]
    prev = np.asarray(prev_xy).astype(np.int32).astype(np.float32)
    curr = np.asarray(curr_xy).astype(np.int32).astype(np.float32)
    d0 = np.asarray(depth0, dtype=np.float32)
    n = len(prev)
    out = np.zeros((n, 10))
    ones = np.ones(n, np.float32)
    p1 = np.linalg.solve(K, np.stack([curr[:, 0], curr[:, 1], ones]).astype(np.float64)).T.astype(np.float32)
    x1 = p1[:, 0].astype(np.float64) / p1[:, 2].astype(np.float64)
    y1 = p1[:, 1].astype(np.float64) / p1[:, 2].astype(np.float64)
    has = d0 > 0
    h0 = np.stack([prev[:, 0] * d0, prev[:, 1] * d0, d0])
    X0 = np.linalg.solve(K, h0.astype(np.float64)).T.astype(np.float32)
    p0 = np.linalg.solve(K, np.stack([prev[:, 0], prev[:, 1], ones]).astype(np.float64)).T.astype(np.float32)
    out[has, 0] = CF32
    out[has, 1:4] = X0[has]
    out[has, 4] = x1[has]
    out[has, 5] = y1[has]
    nh = ~has
    out[nh, 0] = CF22
    out[nh, 4] = p0[nh, 0].astype(np.float64) / p0[nh, 2].astype(np.float64)
    out[nh, 5] = p0[nh, 1].astype(np.float64) / p0[nh, 2].astype(np.float64)
    out[nh, 7] = x1[nh]
    out[nh, 8] = y1[nh]
    return out


def solve(problems, x0=None, max_iterations=100, device=0):
    """problems: list of (n_i, 10) factor arrays; x0: (P, 6) initial angles_0to1, t_0to1 (zeros
    by default, reset_VO_to_identity).  Returns (x (P, 6), [LMStats])."""
    P = len(problems)
    off = np.zeros(P + 1, dtype=np.int32)
    for i, f in enumerate(problems):
        off[i + 1] = off[i] + len(f)
    F = np.ascontiguousarray(np.concatenate([np.asarray(f, dtype=np.float64).reshape(-1, 10) for f in problems])
                             if P else np.zeros((0, 10)))
    x = np.zeros((P, 6)) if x0 is None else np.array(x0, dtype=np.float64).reshape(P, 6).copy()
    st = (_core.LMStats * max(P, 1))()
    check(lib().loam_vo_solve(device, P, ptr(off), ptr(F), ptr(x), max_iterations, st))
    return x, [st[i] for i in range(P)]
