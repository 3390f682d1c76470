"""Synthetic HDL-64E street frames (ctypes over libloam_synth.so, csrc/synth.cpp).

KITTI bags are not available offline, so tests and bench run on this
generator: 64 rings x ``n_az`` azimuths, ring-major order, range noise N(0, 0.02 m).
"""
import ctypes
import os

import numpy as np

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(__file__), "_lib", "libloam_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (make -C vloam-noted_amd)")
        lib = ctypes.CDLL(path)
        lib.synth_frame.restype = ctypes.c_int32
        lib.synth_frame.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                    ctypes.c_void_p, ctypes.c_void_p]
        lib.synth_frame_ex.restype = ctypes.c_int32
        lib.synth_frame_ex.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                       ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
        lib.synth_pose.restype = None
        lib.synth_pose.argtypes = [ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_void_p, ctypes.c_void_p]
        _LIB = lib
    return _LIB


# edge-case modes (csrc/synth.cpp): azimuth-interleaved order, per-laser azimuth offsets,
# elevations on the ring-rule boundaries, 1 cm coordinate quantization, 16- and 32-laser sensors
COLUMN_MAJOR, LASER_AZ, BOUNDARY, QUANTIZE, VLP16, HDL32 = 1, 2, 4, 8, 16, 32


def frame(seed: int, index: int, n_az: int = 2000, speed: float = 1.0, flags: int = 0):
    """Return (xyz float32 [n, 3] in the sensor frame, ground-truth pose7 = q xyzw + t)."""
    buf = np.empty((64 * n_az, 3), dtype=np.float32)
    pose = np.empty(7, dtype=np.float64)
    n = _lib().synth_frame_ex(seed, index, n_az, speed, flags, buf.ctypes.data, pose.ctypes.data)
    return buf[:n].copy(), pose


def pose(seed: int, index: float, speed: float = 1.0):
    q = np.empty(4, dtype=np.float64)
    t = np.empty(3, dtype=np.float64)
    _lib().synth_pose(seed, float(index), speed, q.ctypes.data, t.ctypes.data)
    return q, t
