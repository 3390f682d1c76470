"""GPU parity of LaserOdometry::solveLO (laser_odometry.cpp:199-584) against the oracle.

Both consume the same scan-registration features (the oracle's) frame after frame:
  - correspondence counts (integer work: 1-NN, ring-scan second/third points) identical,
  - LM iteration counts identical,
  - q_last_curr / t_last_curr within 1e-6, the accumulated pose within 1e-4 m / 1e-4 rad
    (device 6x6 Cholesky vs oracle DENSE_QR; BASELINE parity bar),
  - laserCloudCornerLast / SurfLast after the swap identical.
"""
import numpy as np
import pytest

import loam_oracle as O
from helpers import quat_angle
from loam_amd import synth
from loam_amd.odometry import BatchOdometry

pytestmark = pytest.mark.gpu


def features(seed, n_frames, n_az=2000, flags=0, with_gt=False, n_scans=64):
    sr = O.ScanRegistration(n_scans=n_scans)
    out, gts = [], []
    for f in range(n_frames):
        xyz, gt = synth.frame(seed, f, n_az, flags=flags)
        sr.input(xyz)
        out.append(sr.output())
        gts.append(gt)
    return (out, gts) if with_gt else out


@pytest.fixture(scope="module")
def seq():
    return features(5, 10)


def run_oracle(frames, priors=None):
    od = O.LaserOdometry()
    res = []
    for k, c in enumerate(frames):
        od.input(*c)
        if priors is not None:
            od.set_prior(*priors[k])
        od.solve()
        q, t, qlc, tlc, skip = od.output()
        corr, lm = od.stats()
        res.append(dict(q=q, t=t, qlc=qlc, tlc=tlc, corr=list(corr), it=[lm[0].iterations, lm[1].iterations],
                        corner=od.cloud(0), surf=od.cloud(1)))
    return res


@pytest.mark.parametrize("persistent", ["1"])
def test_odometry_sequence(seq, monkeypatch, persistent):
    monkeypatch.setenv("LOAM_LM_PERSISTENT", persistent)
    ref = run_oracle(seq)
    od = BatchOdometry(1)
    worst_t = worst_r = 0.0
    for k, c in enumerate(seq):
        od.input(0, c[1], c[2], c[3], c[4])
        od.solve()
        q, t, qlc, tlc, skip = od.output(0)
        st = od.stats(0)
        r = ref[k]
        assert not skip
        if k > 0:
            assert [st.corner_num[0], st.surf_num[0], st.corner_num[1], st.surf_num[1]] == r["corr"], k
            assert [st.lm[0].iterations, st.lm[1].iterations] == r["it"], k
            assert np.abs(tlc - r["tlc"]).max() < 1e-6 and quat_angle(qlc, r["qlc"]) < 1e-6, k
        worst_t = max(worst_t, float(np.linalg.norm(t - r["t"])))
        worst_r = max(worst_r, quat_angle(q, r["q"]))
        assert np.array_equal(od.last_cloud(0, 0), r["corner"])
        assert np.array_equal(od.last_cloud(0, 1), r["surf"])
    assert worst_t < 1e-4 and worst_r < 1e-4, (worst_t, worst_r)


def test_odometry_batched_streams(seq):
    """streams offset along the same sequence, one launch sequence per solve"""
    ref = run_oracle(seq)
    B = 4
    od = BatchOdometry(B)
    for k in range(len(seq) - B + 1):
        for s in range(B):
            c = seq[k + s] if k + s < len(seq) else seq[-1]
            od.input(s, c[1], c[2], c[3], c[4])
        od.solve()
    # stream 0 consumed frames 0..n-B: compare with the oracle after the same frames
    q, t, _, _, _ = od.output(0)
    r = ref[len(seq) - B]
    assert np.linalg.norm(t - r["t"]) < 1e-4 and quat_angle(q, r["q"]) < 1e-4


def test_odometry_empty_and_first_frame():
    od = BatchOdometry(1)
    z = np.zeros((0, 4), np.float32)
    od.input(0, z, z, z, z)
    od.solve()
    q, t, qlc, tlc, skip = od.output(0)
    assert np.allclose(q, [0, 0, 0, 1]) and np.allclose(t, 0)
    od.input(0, z, z, z, z)
    od.solve()  # inited, no correspondences: LM leaves the pose
    q, t, _, _, _ = od.output(0)
    assert np.allclose(q, [0, 0, 0, 1]) and np.allclose(t, 0)


def test_odometry_more_streams_than_cus(seq):
    """300 streams (one LM workgroup each, more than the GPU holds at once): the LM shares are
    claimed by whichever workgroups run (lm.h), so no residency is needed; every stream matches
    the oracle"""
    ref = run_oracle(seq[:3])
    B = 300
    od = BatchOdometry(B, max_input_points=32768)
    for c in seq[:3]:
        for s in range(B):
            od.input(s, c[1], c[2], c[3], c[4])
        od.solve()
    r = ref[-1]
    for s in range(B):
        q, t, _, _, _ = od.output(s)
        st = od.stats(s)
        assert np.linalg.norm(t - r["t"]) < 1e-4 and quat_angle(q, r["q"]) < 1e-4, s
        assert [st.lm[0].iterations, st.lm[1].iterations] == r["it"], s
    od.close()


def _check_sequence(frames, priors=None, **params):
    """GPU odometry frame by frame against the oracle: counts and iterations identical, poses
    within the BASELINE bar"""
    ref = run_oracle(frames, priors)
    od = BatchOdometry(1, **params)
    for k, c in enumerate(frames):
        od.input(0, c[1], c[2], c[3], c[4])
        if priors is not None:
            od.set_prior(0, *priors[k])
        od.solve()
        q, t, qlc, tlc, _ = od.output(0)
        st = od.stats(0)
        r = ref[k]
        if k > 0:
            assert [st.corner_num[0], st.surf_num[0], st.corner_num[1], st.surf_num[1]] == r["corr"], k
            assert [st.lm[0].iterations, st.lm[1].iterations] == r["it"], k
            assert np.abs(tlc - r["tlc"]).max() < 1e-6 and quat_angle(qlc, r["qlc"]) < 1e-6, k
        assert np.linalg.norm(t - r["t"]) < 1e-4 and quat_angle(q, r["q"]) < 1e-4, k
        assert np.array_equal(od.last_cloud(0, 0), r["corner"])
        assert np.array_equal(od.last_cloud(0, 1), r["surf"])
    od.close()


@pytest.mark.parametrize("flags", [synth.COLUMN_MAJOR | synth.LASER_AZ, synth.QUANTIZE,
                                   synth.BOUNDARY | synth.COLUMN_MAJOR | synth.LASER_AZ | synth.QUANTIZE])
def test_odometry_edge_case_sequence(flags):
    """azimuth-interleaved input with per-laser offsets: int(intensity) is not monotone along
    the last clouds (scanID - 1 before the halfPassed latch), so the reference's ring scans
    (laser_odometry.cpp:309-355, :407-456) visit points by their `continue` / `break` tests,
    which the kernel restates literally"""
    frames = features(7, 6, flags=flags)
    if flags & synth.COLUMN_MAJOR:
        last = frames[2][2]  # a lessSharp cloud (next frame's laserCloudCornerLast)
        assert (np.diff(last[:, 3].astype(np.int32)) < 0).sum() > 5
    _check_sequence(frames)


@pytest.mark.parametrize("lasers", [16, 32])
def test_odometry_16_and_32_lines(lasers):
    """VLP-16 / HDL-32E clouds (N_SCANS 16 / 32): sparser rings, the same scan-to-scan path"""
    frames = features(6, 5, flags=synth.VLP16 if lasers == 16 else synth.HDL32, n_scans=lasers)
    _check_sequence(frames)


def _relative_priors(gts, seed=0):
    """velo_last_VOT_velo_curr: the ground-truth frame-to-frame motion with VO-like noise"""
    from scipy.spatial.transform import Rotation as R
    rng = np.random.default_rng(seed)
    out = [(np.array([0, 0, 0, 1.0]), np.zeros(3))]
    for k in range(1, len(gts)):
        ql, tl, qc, tc = gts[k - 1][:4], gts[k - 1][4:], gts[k][:4], gts[k][4:]
        rl = R.from_quat(ql)
        rel = (rl.inv() * R.from_quat(qc)) * R.from_rotvec(rng.normal(0, 0.002, 3))
        t = rl.inv().apply(tc - tl) + rng.normal(0, 0.02, 3)
        out.append((rel.as_quat(), t))
    return out


def test_odometry_vo_prior():
    """coupled mode (detach_VO_LO = false, laser_odometry.cpp:237-250): every outer round starts
    from the VO prior"""
    frames, gts = features(9, 6, with_gt=True)
    priors = _relative_priors(gts)
    _check_sequence(frames, priors, detach_vo_lo=0)
    # the prior moves the result: the detached solve of the same frames differs
    det = run_oracle(frames)
    cpl = run_oracle(frames, priors)
    assert max(np.abs(a["tlc"] - b["tlc"]).max() for a, b in zip(det[1:], cpl[1:])) > 1e-9


def test_odometry_prior_contract():
    from loam_amd._core import LoamError
    frames = features(9, 2)
    od = BatchOdometry(1, detach_vo_lo=0)
    c = frames[0]
    od.input(0, c[1], c[2], c[3], c[4])
    od.solve()  # first frame: no optimisation, no prior needed
    od.input(0, c[1], c[2], c[3], c[4])
    with pytest.raises(LoamError) as e:
        od.solve()  # coupled mode without the frame's prior
    assert e.value.rc == -4
    od.close()
    det = BatchOdometry(1)
    with pytest.raises(LoamError) as e:
        det.set_prior(0, [0, 0, 0, 1.0], [0, 0, 0.0])
    assert e.value.rc == -4
    det.close()
