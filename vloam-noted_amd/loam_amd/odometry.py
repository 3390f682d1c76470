"""LaserOdometry on MI355X — host mirror of vloam::LaserOdometry
(src/lidar_odometry_mapping/include/lidar_odometry_mapping/laser_odometry.h:70-84).

``input(sharp, lessSharp, flat, lessFlat)`` / ``solveLO()`` / ``output()`` with the reference's
meaning: clouds are (n, 4) float32 (x, y, z, intensity = scanID + 0.1 relTime); ``output``
returns q_w_curr, t_w_curr, q_last_curr, t_last_curr and skip_frame
(laser_odometry.cpp:660-679).  ``BatchOdometry`` holds n independent streams per handle.
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, f32x4, lib, ptr


class BatchOdometry:
    def __init__(self, n_streams=1, device=0, params=None, **param_overrides):
        self.params = params if params is not None else _core.default_params(**param_overrides)
        self.n_streams = n_streams
        h = ctypes.c_void_p()
        check(lib().loam_odometry_create(ctypes.byref(self.params), device, n_streams, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_odometry_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(lib().loam_odometry_reset(self.h))

    def input(self, stream, sharp, less_sharp, flat, less_flat):
        cl = [f32x4(c) for c in (sharp, less_sharp, flat, less_flat)]
        args = []
        for c in cl:
            args += [ptr(c), len(c)]
        check(lib().loam_odometry_input(self.h, stream, *args))

    def input_device(self, stream, ptrs, counts):
        args = []
        for p, n in zip(ptrs, counts):
            args += [p, n]
        check(lib().loam_odometry_input_device(self.h, stream, *args))

    def set_prior(self, stream, q=None, t=None):
        """VO prior velo_last_VOT_velo_curr for the next solve (detach_vo_lo = 0 only,
        laser_odometry.cpp:237-250); None clears it"""
        if q is None:
            check(lib().loam_odometry_set_prior(self.h, stream, None, None))
            return
        q = np.ascontiguousarray(q, dtype=np.float64)
        t = np.ascontiguousarray(t, dtype=np.float64)
        check(lib().loam_odometry_set_prior(self.h, stream, ptr(q), ptr(t)))

    def solve(self):
        check(lib().loam_odometry_solve(self.h))

    def output(self, stream=0):
        q, t, qlc, tlc = np.empty(4), np.empty(3), np.empty(4), np.empty(3)
        skip = _core.c_i32()
        check(lib().loam_odometry_output(self.h, stream, ptr(q), ptr(t), ptr(qlc), ptr(tlc), ctypes.byref(skip)))
        return q, t, qlc, tlc, bool(skip.value)

    def last_cloud_device(self, stream, which):
        p = ctypes.c_void_p()
        n = check(lib().loam_odometry_last_cloud(self.h, stream, which, ctypes.byref(p)))
        return p.value, n

    def last_cloud(self, stream, which):
        _, n = self.last_cloud_device(stream, which)
        out = np.empty((n, 4), dtype=np.float32)
        if n:
            check(lib().loam_odometry_copy_last(self.h, stream, which, ptr(out), n))
        return out

    def stats(self, stream=0):
        st = _core.OdomStats()
        check(lib().loam_odometry_stats(self.h, stream, ctypes.byref(st)))
        return st


class LaserOdometry:
    """Single-stream drop-in with the reference method names."""

    def __init__(self, device=0, **param_overrides):
        self._o = BatchOdometry(1, device, **param_overrides)

    def init(self):
        self._o.reset()

    def input(self, laserCloud, cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat, surfPointsLessFlat):
        self._o.input(0, cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat, surfPointsLessFlat)

    def solveLO(self):
        self._o.solve()

    def output(self):
        """q_w_curr, t_w_curr, laserCloudCornerLast, laserCloudSurfLast, skip_frame"""
        q, t, _, _, skip = self._o.output(0)
        return q, t, self._o.last_cloud(0, 0), self._o.last_cloud(0, 1), skip

    def stats(self):
        return self._o.stats(0)

    @property
    def batch(self):
        return self._o
