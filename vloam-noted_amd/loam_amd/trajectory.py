"""KITTI-format trajectory rows of the odometry / mapping poses.

Restates VloamTF::{LO,MO,VO}2Cam0StartFrame (vloam_tf.cpp:84-160) as called by the driver
(vloam_main_node.cpp:192-198): for frame `count` (counted from start_frame, negative: skipped)

    cam0_init_T_cam0_last  = base_T_cam0^-1 * world_T_base_last * base_T_cam0      (:115, :141)
    cam0_init_T_cam0_start = cam0_init_T_cam0_last                    if count == 0 (:117-118)
    cam0_start_T_cam0_last = cam0_init_T_cam0_start^-1 * cam0_init_T_cam0_last      (:120)

then tf2::toMsg (rotation -> quaternion, tf2 Matrix3x3::getRotation), tf2::transformToEigen
(quaternion -> rotation matrix), cast<float>, and one "%f" x 12 row of the top 3 x 4 block
(:122-133).  world_T_base_last is the stage's pose: LaserOdometry's q_w_curr / t_w_curr
(laser_odometry.cpp:619-620) for LO rows, LaserMapping's (laser_mapping.cpp:834-835, or the
high-frequency pose on skipped frames :858-861) for MO rows.  base_T_cam0 is the static
base <- imu <- cam0 extrinsic (vloam_tf.cpp:58).

Host bookkeeping in float64 (tf2 is double precision), no device work.
"""
from __future__ import annotations

import numpy as np


def quat_to_matrix(q) -> np.ndarray:
    """tf2 Matrix3x3::setRotation (x, y, z, w): scaled by 2 / |q|^2, so q need not be unit."""
    x, y, z, w = (float(v) for v in q)
    d = x * x + y * y + z * z + w * w
    s = 2.0 / d
    xs, ys, zs = x * s, y * s, z * s
    wx, wy, wz = w * xs, w * ys, w * zs
    xx, xy, xz = x * xs, x * ys, x * zs
    yy, yz, zz = y * ys, y * zs, z * zs
    return np.array([[1.0 - (yy + zz), xy - wz, xz + wy],
                     [xy + wz, 1.0 - (xx + zz), yz - wx],
                     [xz - wy, yz + wx, 1.0 - (xx + yy)]])


def matrix_to_quat(R) -> np.ndarray:
    """tf2 Matrix3x3::getRotation: trace branch, else the largest diagonal element's branch."""
    R = np.asarray(R, dtype=np.float64)
    trace = R[0, 0] + R[1, 1] + R[2, 2]
    t = [0.0, 0.0, 0.0, 0.0]
    if trace > 0.0:
        s = np.sqrt(trace + 1.0)
        t[3] = s * 0.5
        s = 0.5 / s
        t[0] = (R[2, 1] - R[1, 2]) * s
        t[1] = (R[0, 2] - R[2, 0]) * s
        t[2] = (R[1, 0] - R[0, 1]) * s
    else:
        i = (2 if R[1, 1] < R[2, 2] else 1) if R[0, 0] < R[1, 1] else (2 if R[0, 0] < R[2, 2] else 0)
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        t[i] = s * 0.5
        s = 0.5 / s
        t[3] = (R[k, j] - R[j, k]) * s
        t[j] = (R[j, i] + R[i, j]) * s
        t[k] = (R[k, i] + R[i, k]) * s
    return np.array(t)


def eigen_quat_matrix(q) -> np.ndarray:
    """Eigen QuaternionBase::toRotationMatrix (assumes a unit quaternion, no rescaling)."""
    x, y, z, w = (float(v) for v in q)
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1.0 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1.0 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1.0 - (txx + tyy)]])


def transform(q, t) -> np.ndarray:
    """4 x 4 homogeneous matrix of tf2::Transform(Quaternion(q), Vector3(t))."""
    T = np.eye(4)
    T[:3, :3] = quat_to_matrix(q)
    T[:3, 3] = np.asarray(t, dtype=np.float64)
    return T


def inverse(T) -> np.ndarray:
    """tf2::Transform::inverse: basis^T, -basis^T * origin."""
    out = np.eye(4)
    Rt = T[:3, :3].T
    out[:3, :3] = Rt
    out[:3, 3] = Rt @ -T[:3, 3]
    return out


def row_text(T) -> str:
    """the fprintf of vloam_tf.cpp:126-133 after toMsg / transformToEigen / cast<float>"""
    R = eigen_quat_matrix(matrix_to_quat(T[:3, :3]))
    M = np.empty((3, 4), dtype=np.float32)
    M[:, :3] = R.astype(np.float32)
    M[:, 3] = np.asarray(T[:3, 3], dtype=np.float64).astype(np.float32)
    return " ".join("%f" % float(v) for v in M.reshape(-1)) + "\n"


class KittiTrajectoryWriter:
    """One trajectory file (LO, MO or VO rows).  write(count, q, t) per frame, with count =
    frame - start_frame as the driver passes it (vloam_main_node.cpp:194-198); count < 0 writes
    nothing, count == 0 latches the start frame."""

    def __init__(self, path_or_file=None, base_T_cam0=None):
        self.base_T_cam0 = np.eye(4) if base_T_cam0 is None else np.asarray(base_T_cam0, dtype=np.float64)
        self.cam0_T_base = inverse(self.base_T_cam0)
        self.start = None
        self.rows: list[str] = []
        self._own = isinstance(path_or_file, str)
        self.f = open(path_or_file, "w") if self._own else path_or_file

    def write(self, count: int, q_world_base, t_world_base) -> str | None:
        if count < 0:
            return None
        init_last = self.cam0_T_base @ transform(q_world_base, t_world_base) @ self.base_T_cam0
        if count == 0:
            self.start = init_last
        if self.start is None:
            raise ValueError("KittiTrajectoryWriter: the first written frame must have count 0")
        row = row_text(inverse(self.start) @ init_last)
        self.rows.append(row)
        if self.f is not None:
            self.f.write(row)
        return row

    def close(self):
        if self._own and self.f is not None:
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def parse_rows(text: str) -> np.ndarray:
    """rows of a KITTI trajectory file -> [n, 4, 4] poses"""
    vals = np.array([[float(v) for v in line.split()] for line in text.splitlines() if line.strip()])
    out = np.tile(np.eye(4), (len(vals), 1, 1))
    out[:, :3, :] = vals.reshape(-1, 3, 4)
    return out
