"""Visual-odometry depth association on MI355X — host mirror of ``vloam::PointCloudUtil``.

Mirrors src/visual_odometry/include/visual_odometry/point_cloud_util.h:25-75: the point cloud
is projected into the rectified camera 0 image (``projectPointCloud``), bucketed on a 5 px grid
(``downsamplePointCloud``) and queried per image feature (``queryDepth``), as
visual_odometry.cpp:195-214 and :371-372 call them.  ``BatchDepth`` holds n independent
instances on one device (one launch sequence per ``process`` for all of them).
"""
import ctypes

import numpy as np

from . import _core
from ._core import check, lib, ptr

# A KITTI raw 2011_09_26 calibration (calib_velo_to_cam R|T, calib_cam_to_cam R_rect_00,
# P_rect_00): the matrices the reference reads at point_cloud_util.cpp:60-141.  Synthetic
# tests and the bench use it with the HDL-64E scene generator.
_R = np.array([7.533745e-03, -9.999714e-01, -6.166020e-04, 1.480249e-02, 7.280733e-04, -9.998902e-01,
               9.998621e-01, 7.523790e-03, 1.480755e-02]).reshape(3, 3)
_T = np.array([-4.069766e-03, -7.631618e-02, -2.717806e-01])
KITTI_CAM_T_VELO = np.eye(4, dtype=np.float32)
KITTI_CAM_T_VELO[:3, :3] = _R
KITTI_CAM_T_VELO[:3, 3] = _T
KITTI_RECT0_T_CAM = np.eye(4, dtype=np.float32)
KITTI_RECT0_T_CAM[:3, :3] = np.array([9.999239e-01, 9.837760e-03, -7.445048e-03, -9.869795e-03, 9.999421e-01,
                                      -4.278459e-03, 7.402527e-03, 4.351614e-03, 9.999631e-01]).reshape(3, 3)
KITTI_P_RECT0 = np.array([7.215377e+02, 0.0, 6.095593e+02, 0.0, 0.0, 7.215377e+02, 1.728540e+02, 0.0,
                          0.0, 0.0, 1.0, 0.0], dtype=np.float32).reshape(3, 4)


def depth_params(cam_T_velo=KITTI_CAM_T_VELO, rect0_T_cam=KITTI_RECT0_T_CAM, P_rect0=KITTI_P_RECT0, **kw):
    p = _core.DepthParams()
    lib().loam_depth_params_default(ctypes.byref(p))
    for name, m, n in (("cam_T_velo", cam_T_velo, 16), ("rect0_T_cam", rect0_T_cam, 16), ("P_rect0", P_rect0, 12)):
        a = np.ascontiguousarray(m, dtype=np.float32).reshape(n)
        getattr(p, name)[:] = [float(v) for v in a]
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class BatchDepth:
    def __init__(self, n_streams=1, device=0, params=None, **kw):
        self.params = params if params is not None else depth_params(**kw)
        self.n_streams = n_streams
        self.new_w = int(np.ceil(np.float32(self.params.img_width) / np.float32(self.params.grid)))
        self.new_h = int(np.ceil(np.float32(self.params.img_height) / np.float32(self.params.grid)))
        h = ctypes.c_void_p()
        check(lib().loam_depth_create(ctypes.byref(self.params), device, n_streams, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_depth_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def input(self, stream, xyz):
        xyz = np.ascontiguousarray(xyz, dtype=np.float32)
        if xyz.ndim != 2 or xyz.shape[1] < 3:
            raise ValueError("points must be (n, >=3) float32")
        check(lib().loam_depth_input(self.h, stream, ptr(xyz), len(xyz), xyz.shape[1]))

    def input_device(self, stream, d_ptr, n, stride):
        check(lib().loam_depth_input_device(self.h, stream, d_ptr, n, stride))

    def process(self):
        check(lib().loam_depth_process(self.h))

    def counts(self, stream=0):
        a, b = ctypes.c_int32(), ctypes.c_int32()
        check(lib().loam_depth_counts(self.h, stream, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def cloud(self, stream, which):
        """0: point_cloud_2d, 1: point_cloud_2d_dnsp, (n, 3) float32 (u, v, depth)"""
        n = check(lib().loam_depth_copy(self.h, stream, which, None, 0))
        out = np.empty((n, 3), dtype=np.float32)
        if n:
            check(lib().loam_depth_copy(self.h, stream, which, ptr(out), n))
        return out

    def buckets(self, stream=0):
        n = self.new_w * self.new_h
        bx, by, bd = (np.empty(n, dtype=np.float32) for _ in range(3))
        bc = np.empty(n, dtype=np.int32)
        check(lib().loam_depth_buckets(self.h, stream, ptr(bx), ptr(by), ptr(bd), ptr(bc)))
        return bx, by, bd, bc

    def query(self, streams, xy, radius=2):
        xy = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
        st = np.ascontiguousarray(np.broadcast_to(np.asarray(streams, dtype=np.int32), (len(xy),)))
        out = np.empty(len(xy), dtype=np.float32)
        check(lib().loam_depth_query(self.h, len(xy), ptr(st), ptr(xy), radius, ptr(out)))
        return out

    def query_device(self, n, d_streams, d_xy, d_depth, radius=2):
        check(lib().loam_depth_query_device(self.h, n, d_streams, d_xy, radius, d_depth))

    @property
    def ms(self):
        return lib().loam_depth_ms(self.h)


class PointCloudUtil:
    """Single-instance drop-in with the reference method names."""

    def __init__(self, device=0, **kw):
        self._b = BatchDepth(1, device, **kw)
        self.point_cloud_3d_tilde = None

    def projectPointCloud(self):
        # the device runs projection and downsampling as one launch sequence
        self._b.input(0, self.point_cloud_3d_tilde)
        self._b.process()

    def downsamplePointCloud(self):
        pass  # done by projectPointCloud's launch sequence

    @property
    def point_cloud_2d(self):
        return self._b.cloud(0, 0)

    @property
    def point_cloud_2d_dnsp(self):
        return self._b.cloud(0, 1)

    def queryDepth(self, x, y, searching_radius=2):
        return float(self._b.query(0, np.array([[x, y]], dtype=np.float32), searching_radius)[0])
