"""ScanRegistration on MI355X — host mirror of vloam::ScanRegistration
(src/lidar_odometry_mapping/include/lidar_odometry_mapping/scan_registration.h:64-81).

``input(cloud)`` takes an (n, >=3) float32 array (pcl::PointXYZ fields first); ``output()``
returns the five clouds of ScanRegistration::output (scan_registration.cpp:566-577) as
(n, 4) float32 arrays (x, y, z, intensity = scanID + 0.1 * relTime).
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, lib, ptr

CLOUDS = ("laserCloud", "cornerPointsSharp", "cornerPointsLessSharp", "surfPointsFlat",
          "surfPointsLessFlat")


class ScanRegistration:
    def __init__(self, device=0, params=None, **param_overrides):
        self.params = params if params is not None else _core.default_params(**param_overrides)
        h = ctypes.c_void_p()
        check(lib().loam_scanreg_create(ctypes.byref(self.params), device, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_scanreg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init(self):
        pass

    def reset(self):
        pass

    def input(self, cloud):
        xyz = np.ascontiguousarray(cloud, dtype=np.float32)
        check(lib().loam_scanreg_input(self.h, ptr(xyz), len(xyz), xyz.shape[1]))

    def input_device(self, d_ptr, n, stride):
        check(lib().loam_scanreg_input_device(self.h, d_ptr, n, stride))

    def host_buffer(self):
        """the handle's page-locked ingest buffer as a (cap, 4) float32 array (write a frame
        there, then input_async(n=...) copies from it without staging)"""
        p = ctypes.c_void_p()
        cap = ctypes.c_int32()
        check(lib().loam_scanreg_host_buffer(self.h, ctypes.byref(p), ctypes.byref(cap)))
        buf = (ctypes.c_float * (4 * cap.value)).from_address(p.value)
        return np.ctypeslib.as_array(buf).reshape(cap.value, 4)

    def input_async(self, cloud=None, n=None):
        """queue one frame (cloud is copied into the pinned buffer first; or n points already
        written there by the caller) and return; wait() or any accessor completes it"""
        check(lib().loam_scanreg_wait(self.h))  # the buffer is free once the last frame is done
        buf = self.host_buffer()
        if cloud is not None:
            c = np.asarray(cloud, dtype=np.float32)
            n = len(c)
            if c.shape[1] == 4:
                buf[:n] = c  # one contiguous copy
            else:
                buf[:n, :3] = c[:, :3]
        check(lib().loam_scanreg_input_async(self.h, buf.ctypes.data, int(n), 4))

    def wait(self):
        check(lib().loam_scanreg_wait(self.h))

    def counts(self):
        c = np.zeros(5, dtype=np.int32)
        check(lib().loam_scanreg_counts(self.h, ptr(c)))
        return c

    def cloud(self, which):
        n = int(self.counts()[which])
        out = np.empty((n, 4), dtype=np.float32)
        check(lib().loam_scanreg_copy(self.h, which, ptr(out), n))
        return out

    def output(self):
        return tuple(self.cloud(i) for i in range(5))

    def device_ptr(self, which):
        p = ctypes.c_void_p()
        n = check(lib().loam_scanreg_device_ptr(self.h, which, ctypes.byref(p)))
        return p.value, n

    def curvature(self):
        n = int(self.counts()[0])
        c = np.empty(n, dtype=np.float32)
        lab = np.empty(n, dtype=np.int32)
        check(lib().loam_scanreg_curvature(self.h, ptr(c), ptr(lab), n))
        return c, lab

    @property
    def ms(self):
        return lib().loam_scanreg_ms(self.h)

    def debug_counters(self, reset=False):
        """ring VoxelGrid phase cycles (include/loam_core.h LOAM_SR_DEBUG_COUNTERS)"""
        out = np.zeros(24, np.uint64)
        check(lib().loam_scanreg_debug_counters(self.h, ptr(out), 24, int(reset)))
        return out


class ScanRegistrationBatch:
    """Up to ``max_frames`` independent scans per launch sequence (loam_scanreg_create_batch):
    ``input_batch(clouds)`` runs them together; ``cloud(frame, which)`` / ``device_ptr(frame,
    which)`` read frame ``frame``'s clouds.  Bit-identical to one ScanRegistration per scan."""

    def __init__(self, max_frames, device=0, params=None, **param_overrides):
        self.params = params if params is not None else _core.default_params(**param_overrides)
        self.max_frames = max_frames
        h = ctypes.c_void_p()
        check(lib().loam_scanreg_create_batch(ctypes.byref(self.params), device, int(max_frames), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_scanreg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def input_batch(self, clouds):
        """clouds: host (n, >= 3) float32 arrays (same stride), one per frame"""
        arrs = [np.ascontiguousarray(c, dtype=np.float32) for c in clouds]
        stride = arrs[0].shape[1] if arrs and arrs[0].ndim == 2 else 4
        ptrs = np.array([a.ctypes.data for a in arrs], dtype=np.uint64)
        ns = np.array([len(a) for a in arrs], dtype=np.int32)
        check(lib().loam_scanreg_input_batch(self.h, len(arrs), ptr(ptrs), ptr(ns), int(stride), 0))

    def input_batch_device(self, ptrs, counts, stride=4):
        """device pointers (integers) and point counts, one per frame"""
        p = np.ascontiguousarray(ptrs, dtype=np.uint64)
        n = np.ascontiguousarray(counts, dtype=np.int32)
        check(lib().loam_scanreg_input_batch(self.h, len(p), ptr(p), ptr(n), int(stride), 1))

    def counts(self, frame):
        c = np.zeros(5, dtype=np.int32)
        check(lib().loam_scanreg_frame_counts(self.h, int(frame), ptr(c)))
        return c

    def cloud(self, frame, which):
        n = int(self.counts(frame)[which])
        out = np.empty((n, 4), dtype=np.float32)
        check(lib().loam_scanreg_frame_copy(self.h, int(frame), int(which), ptr(out), n))
        return out

    def device_ptr(self, frame, which):
        p = ctypes.c_void_p()
        n = check(lib().loam_scanreg_frame_device_ptr(self.h, int(frame), int(which), ctypes.byref(p)))
        return p.value, n

    @property
    def ms(self):
        return lib().loam_scanreg_ms(self.h)
