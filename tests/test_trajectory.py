"""KITTI trajectory writer (loam_amd/trajectory.py, vloam_tf.cpp:84-160).

Pinned by the reference's own saved trajectory (tests/golden/kitti_mo1_2011_10_03_0042.txt,
539 MO rows that vloam_tf.cpp:136-160 wrote for KITTI 2011_10_03_drive_0042; copied by
tests/golden/make_kitti_fixture.py): the rows are cam0_start_T_cam0_last, so world poses made
from them through a base_T_cam0 extrinsic must come back out as the same rows, in the same
"%f" x 12 format.  The tf2 / Eigen quaternion helpers are checked against scipy.
"""
import io
import os
import re

import numpy as np
from scipy.spatial.transform import Rotation

from loam_amd import trajectory as T

FIX = os.path.join(os.path.dirname(__file__), "golden", "kitti_mo1_2011_10_03_0042.txt")
ROW = re.compile(r"^(-?\d+\.\d{6} ){11}-?\d+\.\d{6}\n$")


def _extrinsic():
    """a KITTI-like base_T_cam0: camera z forward, x right, y down, plus a small misalignment"""
    R = np.array([[0.0, 0.0, 1.0], [-1.0, 0.0, 0.0], [0.0, -1.0, 0.0]])
    R = Rotation.from_rotvec([0.004, -0.011, 0.007]).as_matrix() @ R
    E = np.eye(4)
    E[:3, :3] = R
    E[:3, 3] = [1.08, -0.32, 1.73]
    return E


def test_quaternion_helpers_match_scipy():
    rng = np.random.default_rng(3)
    for q in Rotation.random(200, random_state=4).as_quat():
        R = T.quat_to_matrix(q * rng.uniform(0.5, 2.0))  # tf2 rescales by 2 / |q|^2
        assert np.abs(R - Rotation.from_quat(q).as_matrix()).max() < 1e-14
        q2 = T.matrix_to_quat(R)
        assert min(np.abs(q2 - q).max(), np.abs(q2 + q).max()) < 1e-14
        assert np.abs(T.eigen_quat_matrix(q2) - R).max() < 1e-14


def test_reference_rows_round_trip():
    text = open(FIX).read()
    rows = text.splitlines(keepends=True)
    poses = T.parse_rows(text)
    assert len(rows) == 539 and np.allclose(poses[0], np.eye(4))
    E = _extrinsic()
    Einv = T.inverse(E)
    buf = io.StringIO()
    w = T.KittiTrajectoryWriter(buf, base_T_cam0=E)
    assert w.write(-1, [0, 0, 0, 1], [0, 0, 0]) is None  # before start_frame: nothing
    for k, P in enumerate(poses):
        W = E @ P @ Einv  # world_T_base of frame k (world = base at frame 0)
        w.write(k, T.matrix_to_quat(W[:3, :3]), W[:3, 3])
    out = buf.getvalue().splitlines(keepends=True)
    assert len(out) == len(rows) and all(ROW.match(r) for r in out)
    got, want = T.parse_rows("".join(out)), poses
    # rotations: the file's 6-decimal rows are orthonormal to ~1e-6; translations to float32
    # resolution at up to 1.1 km
    assert np.abs(got[:, :3, :3] - want[:, :3, :3]).max() < 3e-6
    assert np.abs(got[:, :3, 3] - want[:, :3, 3]).max() < 2e-4
    # field for field the text is mostly identical (the rest differ in the 6th decimal: the
    # file's rotations are re-orthonormalised by the quaternion round trip of :122)
    same = sum(x == y for a, b in zip(out, rows) for x, y in zip(a.split(), b.split()))
    assert same > 0.85 * 12 * len(rows), same
    assert out[0] == rows[0]


def test_start_frame_is_relative():
    """rows are relative to the frame written with count 0 (vloam_tf.cpp:117-120)"""
    rng = np.random.default_rng(5)
    qs = Rotation.random(6, random_state=6).as_quat()
    ts = rng.normal(0, 10, (6, 3))
    w = T.KittiTrajectoryWriter(None)
    rows = [w.write(k, qs[k], ts[k]) for k in range(6)]
    assert rows[0] == "1.000000 0.000000 0.000000 0.000000 0.000000 1.000000 0.000000 0.000000 " \
                      "0.000000 0.000000 1.000000 0.000000\n"
    got = T.parse_rows("".join(rows))
    W0 = T.transform(qs[0], ts[0])
    for k in range(6):
        want = T.inverse(W0) @ T.transform(qs[k], ts[k])
        assert np.abs(got[k] - want).max() < 1e-5
