"""CPU: the depth-association oracle (oracle/depth_oracle.cpp) against an independent numpy
restatement of src/visual_odometry/src/point_cloud_util.cpp, and the committed fixture.

- projectPointCloud (:183-219): the float32 matrix chain, front test, (u, v) * (1/depth): bit-exact;
- downsamplePointCloud (:256-324): bucket counts / running averages (a Python loop in input
  order) and the reversed (x, y) order of point_cloud_2d_dnsp: bit-exact;
- queryDepth (:381-487): >= 10 occupied buckets, 3 nearest (double distances rounded to float),
  inverse-distance weights: bit-exact, -1 where the reference gives up.
"""
import os

import numpy as np
import pytest

import loam_oracle as O
from loam_amd import synth
from loam_amd.depth import KITTI_CAM_T_VELO, KITTI_P_RECT0, KITTI_RECT0_T_CAM

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "depth.npz")
f32 = np.float32


def np_project(xyz, A, B, C):
    X = np.concatenate([xyz[:, :3].astype(f32), np.ones((len(xyz), 1), f32)], axis=1)

    def mul_t(V, M, rows):
        out = np.empty((len(V), rows), f32)
        for j in range(rows):
            acc = V[:, 0] * f32(M[j, 0])
            for k in range(1, 4):
                acc = (acc + V[:, k] * f32(M[j, k])).astype(f32)
            out[:, j] = acc
        return out

    v3 = mul_t(mul_t(mul_t(X, A, 4), B, 4), C, 3)
    keep = v3[:, 2] > f32(0.1)
    v3 = v3[keep]
    inv = (f32(1.0) / v3[:, 2]).astype(f32)
    return np.stack([v3[:, 0] * inv, v3[:, 1] * inv, v3[:, 2]], axis=1).astype(f32)


def np_downsample(p2d, grid=5, W=249, H=75):
    bx, by, bd = (np.zeros(W * H, f32) for _ in range(3))
    bc = np.zeros(W * H, np.int32)
    g = f32(grid)
    ix = np.trunc(p2d[:, 0] / g).astype(np.int64)
    iy = np.trunc(p2d[:, 1] / g).astype(np.int64)
    for i in range(len(p2d)):
        if not (0 <= ix[i] < W and 0 <= iy[i] < H):
            continue
        b = ix[i] * H + iy[i]
        x, y, d = p2d[i]
        if bc[b] == 0:
            bx[b], by[b], bd[b] = x, y, d
        else:
            c = f32(bc[b])
            bx[b] = f32(bx[b] + f32(f32(x - bx[b]) / c))
            by[b] = f32(by[b] + f32(f32(y - by[b]) / c))
            bd[b] = f32(bd[b] + f32(f32(d - bd[b]) / c))
        bc[b] += 1
    occ = np.nonzero(bc > 0)[0]
    dnsp = np.stack([bx[occ], by[occ], bd[occ]], axis=1)[::-1]
    return bx, by, bd, bc, dnsp


def np_query(b, x, y, radius=2, grid=5, W=249, H=75):
    bx, by, bd, bc = b
    ix, iy = int(np.trunc(f32(x) / f32(grid))), int(np.trunc(f32(y) / f32(grid)))
    nb = []
    for i in range(ix - radius, ix + radius + 1):
        for j in range(iy - radius, iy + radius + 1):
            if 0 <= i < W and 0 <= j < H and bc[i * H + j] > 0:
                k = i * H + j
                dx, dy = float(f32(x) - bx[k]), float(f32(y) - by[k])
                nb.append((f32(np.sqrt(dx * dx + dy * dy)), bd[k]))
    if len(nb) < 10:
        return f32(-1.0)
    nb.sort(key=lambda t: t[0])  # stable
    (d0, z0), (d1, z1), (d2, z2) = nb[:3]
    num = f32(f32(f32(z0 * d1) * d2) + f32(f32(z1 * d0) * d2))
    num = f32(num + f32(f32(z2 * d0) * d1))
    den = f32(f32(f32(f32(0.0001) + f32(d1 * d2)) + f32(d0 * d2)) + f32(d0 * d1))
    return f32(num / den)


@pytest.fixture(scope="module")
def frame():
    xyz, _ = synth.frame(21, 4, 800)
    u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    u.process(xyz)
    return xyz, u


def test_projection_matches_numpy(frame):
    xyz, u = frame
    ref = np_project(xyz, KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    assert np.array_equal(u.cloud(0), ref)


def test_downsample_matches_numpy(frame):
    _, u = frame
    bx, by, bd, bc, dnsp = np_downsample(u.cloud(0))
    obx, oby, obd, obc = u.buckets()
    assert np.array_equal(obc, bc)
    occ = bc > 0
    assert np.array_equal(obx[occ], bx[occ]) and np.array_equal(oby[occ], by[occ]) and np.array_equal(obd[occ], bd[occ])
    assert np.array_equal(u.cloud(1), dnsp)
    assert 0.05 < len(dnsp) / (249 * 75) < 1.0  # a populated grid (the reference notes ~9.5k on KITTI)


def test_query_matches_numpy(frame):
    _, u = frame
    rng = np.random.default_rng(7)
    q = np.stack([rng.uniform(-10, 1252, 300), rng.uniform(-10, 385, 300)], axis=1).astype(f32)
    got = u.query(q)
    b = u.buckets()
    ref = np.array([np_query(b, x, y) for x, y in q], dtype=f32)
    assert np.array_equal(got, ref)
    assert (got > 0).sum() > 50 and (got == -1).sum() > 50


def test_query_edge_cases():
    u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    assert u.process(np.zeros((0, 3), f32)) == 0  # empty cloud
    assert len(u.cloud(0)) == 0 and len(u.cloud(1)) == 0
    assert np.all(u.query(np.array([[600, 180]], f32)) == -1)
    # every point behind the camera (velodyne x < 0)
    behind = np.array([[-10.0, 0.0, 0.0], [-5.0, 1.0, 0.5]], f32)
    assert u.process(behind) == 0 and len(u.cloud(0)) == 0


def test_oracle_reproduces_fixture():
    import hashlib
    g = np.load(GOLDEN)
    seed, fr, n_az = (int(v) for v in g["params"])
    xyz, _ = synth.frame(seed, fr, n_az)
    u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    u.process(xyz)
    assert hashlib.sha256(u.cloud(0).tobytes()).hexdigest() == str(g["p2d_sha"])
    assert np.array_equal(u.cloud(1), g["dnsp"])
    assert np.array_equal(u.buckets()[3], g["bucket_count"])
    assert np.array_equal(u.query(g["queries"]), g["depth"])
