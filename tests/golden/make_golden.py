"""Generate the committed golden fixtures from the CPU oracle (oracle/loam_oracle.cpp).

The reference ships no tests, fixtures or golden vectors and cannot be built here
(SURVEY.md §4, §8c), so these vectors come from the oracle, which tests/test_oracle.py pins
against independent implementations (cKDTree, numpy eigh/lstsq, finite differences, a numpy
Ceres-LM restatement).  CPU tests check the oracle still reproduces them; GPU tests check the
HIP path against them.

    python tests/golden/make_golden.py [case ...]    # rewrites tests/golden/<case>.npz
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "vloam-noted_amd"), os.path.dirname(HERE)]

import ceres_lm_np as NP  # noqa: E402
import loam_oracle as O  # noqa: E402
from loam_amd import synth  # noqa: E402

SCAN = dict(seed=21, frame=4, n_az=800)
MAP = dict(seed=11, n_frames=8, n_az=800)


def cloud_digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def knn_case():
    rng = np.random.default_rng(1)
    pts = np.zeros((3000, 4), np.float32)
    pts[:, :3] = rng.uniform(-4, 4, (3000, 3))
    q = np.zeros((400, 4), np.float32)
    q[:, :3] = rng.uniform(-4, 4, (400, 3))
    idx, d2 = O.knn(pts, q, 5)
    return dict(pts=pts, q=q, idx=idx, d2=d2)


def voxel_case():
    rng = np.random.default_rng(2)
    pts = np.zeros((6000, 4), np.float32)
    pts[:, :3] = rng.normal(0, 3, (6000, 3))
    pts[:, 3] = rng.uniform(0, 64, 6000)
    with O.voxel_order(1):
        out_input = O.voxel_grid(pts, 0.4)
    # out: PCL's summation order (std::sort of (idx, point) by idx); out_input_order: the
    # mapper kernels' input order (voxel.h)
    return dict(pts=pts, leaf=np.float32(0.4), out=O.voxel_grid(pts, 0.4), out_input_order=out_input)


def lm_case():
    rng = np.random.default_rng(3)
    F, xt = NP.make_problem(rng, 50, 150, kind=3)
    x0 = NP.plus(xt, np.array([0.01, -0.02, 0.015, 0.2, -0.1, 0.3]))
    x, st = O.lm_solve(F, x0)
    return dict(factors=F, x0=x0, x=x, stats=np.array([st.iterations, st.successful, st.invalid,
                                                       st.termination]),
                costs=np.array([st.initial_cost, st.final_cost]))


def scanreg_case():
    xyz, _ = synth.frame(SCAN["seed"], SCAN["frame"], SCAN["n_az"])
    sr = O.ScanRegistration()
    sr.input(xyz)
    c = sr.output()
    return dict(params=np.array([SCAN["seed"], SCAN["frame"], SCAN["n_az"]]),
                counts=np.array([len(x) for x in c]), full_sha=np.array(cloud_digest(c[0])),
                sharp=c[1], less_sharp=c[2], flat=c[3], less_flat=c[4])


def mapping_case():
    """free-running oracle pipeline (scan registration -> mapping with the GT odometry prior)"""
    sr, mp = O.ScanRegistration(), O.LaserMapping()
    poses, stats = [], []
    for f in range(MAP["n_frames"]):
        xyz, gt = synth.frame(MAP["seed"], f, MAP["n_az"])
        sr.input(xyz)
        mp.input(sr.cloud(2), sr.cloud(4), None, gt[:4], gt[4:])
        mp.solve()
        q, t = mp.pose()
        st = mp.stats()
        poses.append(np.concatenate([q, t]))
        stats.append([st.optimized, st.corner_stack, st.surf_stack, st.corner_num[0], st.surf_num[0],
                      st.corner_num[1], st.surf_num[1], st.lm[0].iterations, st.lm[1].iterations])
    return dict(params=np.array([MAP["seed"], MAP["n_frames"], MAP["n_az"]]), poses=np.array(poses),
                stats=np.array(stats))


DEPTH = dict(seed=21, frame=4, n_az=800, n_query=600)


def depth_case():
    """visual-odometry depth association (point_cloud_util.cpp:183-487) of a synthetic scan with
    the KITTI calibration of loam_amd.depth"""
    from loam_amd.depth import KITTI_CAM_T_VELO, KITTI_P_RECT0, KITTI_RECT0_T_CAM
    xyz, _ = synth.frame(DEPTH["seed"], DEPTH["frame"], DEPTH["n_az"])
    u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
    u.process(xyz)
    rng = np.random.default_rng(4)
    q = np.stack([rng.uniform(-10, 1252, DEPTH["n_query"]), rng.uniform(-10, 385, DEPTH["n_query"])],
                 axis=1).astype(np.float32)
    bx, by, bd, bc = u.buckets()
    return dict(params=np.array([DEPTH["seed"], DEPTH["frame"], DEPTH["n_az"]]), p2d_sha=np.array(cloud_digest(u.cloud(0))),
                n_front=np.int32(len(u.cloud(0))), dnsp=u.cloud(1), bucket_count=bc, queries=q, depth=u.query(q))


def vo_case():
    """visual-odometry LM (visual_odometry.cpp:304-509) on a synthetic frame pair"""
    from vo_problems import make_problem
    F, xt = make_problem(np.random.default_rng(5))
    x0 = np.zeros(6)
    x, st = O.vo_solve(F, x0, 100)
    return dict(factors=F, x0=x0, x_true=xt, x=x, max_iter=np.int32(100),
                stats=np.array([st.iterations, st.successful, st.invalid, st.termination]),
                costs=np.array([st.initial_cost, st.final_cost]))


CASES = dict(knn=knn_case, voxel=voxel_case, lm=lm_case, scanreg=scanreg_case, mapping=mapping_case,
             depth=depth_case, vo=vo_case)


def main():
    names = sys.argv[1:] or list(CASES)
    for name in names:
        fn = CASES[name]
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **fn())
        print(f"{path}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
