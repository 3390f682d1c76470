"""GPU: visual-odometry depth association (include/loam_core.h loam_depth_*) against the
oracle restatement of point_cloud_util.cpp:183-487 — bit-exact: point_cloud_2d (input order),
bucket counts and running averages, point_cloud_2d_dnsp (reversed (x, y) order) and queryDepth
results, for single and batched streams, host and device inputs, strided clouds, the committed
fixture and the edge cases (empty cloud, nothing in front, queries off the image)."""
import ctypes
import os

import numpy as np
import pytest

import loam_oracle as O
from loam_amd import synth
from loam_amd.depth import KITTI_CAM_T_VELO, KITTI_P_RECT0, KITTI_RECT0_T_CAM, BatchDepth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "depth.npz")


def oracle(xyz):
    u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    u.process(xyz)
    return u


def queries(seed, n=800):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-10, 1252, n), rng.uniform(-10, 385, n)], axis=1).astype(np.float32)


def check_stream(g, s, u):
    assert np.array_equal(g.cloud(s, 0), u.cloud(0))
    bx, by, bd, bc = g.buckets(s)
    obx, oby, obd, obc = u.buckets()
    assert np.array_equal(bc, obc)
    occ = bc > 0
    for a, b in ((bx, obx), (by, oby), (bd, obd)):
        assert np.array_equal(a[occ], b[occ])
    assert np.array_equal(g.cloud(s, 1), u.cloud(1))
    assert g.counts(s) == (len(u.cloud(0)), len(u.cloud(1)))


@pytest.mark.parametrize("seed,frame,n_az", [(21, 4, 800), (3, 10, 2000)])
def test_single_stream_bit_exact(seed, frame, n_az):
    xyz, _ = synth.frame(seed, frame, n_az)
    g = BatchDepth(1)
    g.input(0, xyz)
    g.process()
    u = oracle(xyz)
    check_stream(g, 0, u)
    q = queries(seed)
    assert np.array_equal(g.query(0, q), u.query(q))


def test_batched_streams_and_strides():
    g = BatchDepth(3)
    us = []
    for s in range(3):
        xyz, _ = synth.frame(5 + s, 2 * s, 1200)
        if s == 1:  # 4 floats per point (pcl::PointXYZ layout)
            xyz = np.concatenate([xyz, np.full((len(xyz), 1), 7.0, np.float32)], axis=1)
        g.input(s, xyz)
        us.append(oracle(xyz[:, :3]))
    g.process()
    for s in range(3):
        check_stream(g, s, us[s])
    q = queries(11, 900)
    st = np.arange(900, dtype=np.int32) % 3
    got = g.query(st, q)
    for s in range(3):
        assert np.array_equal(got[st == s], us[s].query(q[st == s]))


def test_device_input():
    import torch
    xyz, _ = synth.frame(8, 3, 1500)
    g = BatchDepth(1)
    d = torch.from_numpy(np.ascontiguousarray(xyz)).to("cuda:0")
    torch.cuda.synchronize()
    g.input_device(0, d.data_ptr(), len(xyz), 3)
    g.process()
    check_stream(g, 0, oracle(xyz))


def test_fixture():
    gd = np.load(GOLDEN)
    seed, fr, n_az = (int(v) for v in gd["params"])
    xyz, _ = synth.frame(seed, fr, n_az)
    g = BatchDepth(1)
    g.input(0, xyz)
    g.process()
    assert g.counts(0) == (int(gd["n_front"]), len(gd["dnsp"]))
    assert np.array_equal(g.cloud(0, 1), gd["dnsp"])
    assert np.array_equal(g.buckets(0)[3], gd["bucket_count"])
    assert np.array_equal(g.query(0, gd["queries"]), gd["depth"])


def test_edge_cases():
    g = BatchDepth(2)
    g.input(0, np.zeros((0, 3), np.float32))
    g.input(1, np.array([[-10.0, 0.0, 0.0], [-5.0, 1.0, 0.5]], np.float32))  # all behind the camera
    g.process()
    assert g.counts(0) == (0, 0) and g.counts(1) == (0, 0)
    assert np.all(g.query([0, 1], np.array([[600, 180], [10, 10]], np.float32)) == -1)
    # points on bucket edges and just left of the image (truncation toward zero: bucket 0)
    u = oracle(np.zeros((0, 3), np.float32))
    xyz, _ = synth.frame(2, 0, 600)
    g.input(0, xyz)
    g.process()
    check_stream(g, 0, oracle(xyz))
    with pytest.raises(Exception):
        g.query([5], np.array([[1.0, 1.0]], np.float32))  # stream out of range
