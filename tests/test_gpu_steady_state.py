"""GPU parity in the regime the bench times (BASELINE configs[3]): full-density frames
(64 x 2000), steady-state maps (the 5x5x3-cube window saturated after ~150 m) and the window
recentering of laser_mapping.cpp:252-444.

One oracle pipeline run (scan registration -> odometry -> mapping, seed 11, 392 frames) feeds:
  - teacher-forced frames 155 and 160: the oracle's map state before the frame loaded into the
    device mapper, same inputs -> pose within 1e-4 m / 1e-4 rad, stack / submap /
    correspondence counts and LM iterations identical, the updated map within 1e-5 m;
  - the first recentering frame after 380 (grid shift, wrapped slabs cleared), teacher-forced;
  - 24 steady-state frames (150, 160, .., 380) teacher-forced at once through one B = 24 handle,
    stream s holding the oracle's state before frame 150 + 10 s (every stream at a different
    frame of the drive), in both VoxelGrid orders: the per-scan bar of the input-order default
    checked on many frames, not two;
  - a free-running GPU pipeline (HIP scan registration -> HIP odometry -> HIP mapping on the raw
    scans) over 300 frames against the oracle trajectory, in both VoxelGrid summation orders:
    exact_voxel_order = 1 against the oracle in PCL's order, the default input order against the
    oracle in input order (oracle_set_voxel_order) -- every per-scan pose within 1e-4.
The teacher-forced frames load the PCL-order oracle's state; with the input-order mapper its
stacks and cubes differ within the summation-order bound and the pose bar holds.
"""
import numpy as np
import pytest

from helpers import load_state, quat_angle, run_sequence
from loam_amd.mapping import BatchMapper

pytestmark = pytest.mark.gpu

SEED, N_AZ = 11, 2000
STEADY = (155, 160)
RECENTER = tuple(range(380, 392))
BATCH = tuple(range(150, 390, 10))  # 24 frames, one stream each


@pytest.fixture(scope="module")
def seq():
    return run_sequence(seed=SEED, n_frames=RECENTER[-1] + 1, n_az=N_AZ, snapshot_frames=STEADY + RECENTER + BATCH)


def _check(m, rec, s=0):
    q, t = m.pose(s)
    qr, tr = rec["pose"]
    st, sr = m.stats(s), rec["stats"]
    assert np.linalg.norm(t - tr) < 1e-4 and quat_angle(q, qr) < 1e-4, (np.linalg.norm(t - tr), quat_angle(q, qr))
    assert st.optimized == sr.optimized
    assert (st.corner_stack, st.surf_stack, st.corner_map, st.surf_map) == \
        (sr.corner_stack, sr.surf_stack, sr.corner_map, sr.surf_map)
    assert list(st.corner_num) == list(sr.corner_num) and list(st.surf_num) == list(sr.surf_num)
    assert [st.lm[0].iterations, st.lm[1].iterations] == [sr.lm[0].iterations, sr.lm[1].iterations]
    assert list(st.center) == list(sr.center)


def _check_map(m, after, s=0):
    for which, key in ((0, "corner"), (1, "surf")):
        got, ref = m.cubes(s, which), after[key]
        assert sorted(got) == sorted(ref)
        for c in ref:
            assert got[c].shape == ref[c].shape, (key, c)
            assert np.all(np.abs(got[c][:, :3] - ref[c][:, :3]) <= 1e-5 + 4e-7 * np.abs(ref[c][:, :3]))


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("fi", STEADY)
def test_steady_state_teacher_forced(seq, fi, exact):
    rec = seq[fi]
    assert rec["stats"].corner_map > 20000 and rec["stats"].surf_map > 10000  # saturated window
    m = BatchMapper(1, exact_voxel_order=exact)
    load_state(m, 0, rec["before"])
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    _check(m, rec)
    _check_map(m, rec["after"])
    m.close()


@pytest.mark.parametrize("exact", [1, 0])
def test_teacher_forced_batch_of_frames(seq, exact):
    """24 saturated-window frames teacher-forced in one solve of a 24-stream handle: stream s gets
    the oracle's map state before frame BATCH[s] and that frame's inputs, so every stream is at a
    different place of the drive (different cubes, window centre, map density).  Per stream: pose
    within 1e-4 m / 1e-4 rad of the oracle's, stack / submap / correspondence /
    LM iteration counts identical, the updated map within 1e-5 m (every 4th stream)"""
    B = len(BATCH)
    m = BatchMapper(B, exact_voxel_order=exact)
    for s, fi in enumerate(BATCH):
        rec = seq[fi]
        assert rec["stats"].corner_map > 20000 and rec["stats"].surf_map > 10000  # saturated window
        load_state(m, s, rec["before"])
        m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    worst = [0.0, 0.0]
    for s, fi in enumerate(BATCH):
        _check(m, seq[fi], s)
        q, t = m.pose(s)
        qr, tr = seq[fi]["pose"]
        worst = [max(worst[0], float(np.linalg.norm(t - tr))), max(worst[1], quat_angle(q, qr))]
        if s % 4 == 0:
            _check_map(m, seq[fi]["after"], s)
    print(f"teacher-forced {B} frames (exact_voxel_order={exact}): max |dt| {worst[0]:.3e} m, "
          f"max dtheta {worst[1]:.3e} rad")
    m.close()


def test_full_density_recentering(seq):
    shifted = [f for f in RECENTER if not np.array_equal(seq[f]["before"]["cen"], seq[f]["after"]["cen"])]
    assert shifted, "no recentering in the probed frames"
    rec = seq[shifted[0]]
    m = BatchMapper(1)
    load_state(m, 0, rec["before"])
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    _check(m, rec)
    cen, _, _ = m.get_state(0)
    assert np.array_equal(cen, rec["after"]["cen"])
    _check_map(m, rec["after"])
    m.close()


def _oracle_input_order_poses(seq, n):
    """the oracle mapper in input order (the default mode's summation order) on the features and
    priors of the PCL-order run (scan registration and odometry do not depend on the mapper)"""
    import loam_oracle as O
    with O.voxel_order(1):
        m = O.LaserMapping()
        out = []
        for rec in seq[:n]:
            m.input(rec["corner"], rec["surf"], None, rec["q_wodom"], rec["t_wodom"])
            m.solve()
            out.append((m.pose(), m.stats()))
    return out


@pytest.mark.parametrize("exact", [1, 0])
def test_free_running_300_frames(seq, exact):
    """the whole GPU chain on the raw scans, free-running, against the oracle chain in the same
    VoxelGrid summation order: PCL's (exact_voxel_order = 1) or input order (0, the library
    default).  Every per-scan pose within 1e-4 m / 1e-4 rad, correspondence counts and LM
    iterations equal every frame"""
    from loam_amd import synth
    from loam_amd.odometry import BatchOdometry
    from loam_amd.scanreg import ScanRegistration
    n = 300
    ref = [(r["pose"], r["stats"]) for r in seq[:n]] if exact else _oracle_input_order_poses(seq, n)
    sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1, exact_voxel_order=exact)
    dt, dr, counts_bad = [], [], []
    for f in range(n):
        xyz, _ = synth.frame(SEED, f, N_AZ)
        sr.input(xyz)
        ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
        od.input_device(0, ptrs, counts)
        od.solve()
        q, t, _, _, _ = od.output(0)
        (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
        mp.input_device(0, pc, nc, ps, ns, q, t)
        mp.solve()
        qm, tm = mp.pose(0)
        (qr, tr), sr_ = ref[f]
        st = mp.stats(0)
        if (list(st.corner_num), list(st.surf_num), st.lm[0].iterations, st.lm[1].iterations) != \
                (list(sr_.corner_num), list(sr_.surf_num), sr_.lm[0].iterations, sr_.lm[1].iterations):
            counts_bad.append(f)
        dt.append(float(np.linalg.norm(tm - tr)))
        dr.append(quat_angle(qm, qr))
    dt, dr = np.array(dt), np.array(dr)
    print(f"free-running {n} frames (exact_voxel_order={exact}): trans rms {np.sqrt(np.mean(dt ** 2)):.3e} "
          f"max {dt.max():.3e} m, rot rms {np.sqrt(np.mean(dr ** 2)):.3e} max {dr.max():.3e} rad")
    assert counts_bad == []
    assert dt.max() < 1e-4 and dr.max() < 1e-4
    for h in (sr, od, mp):
        h.close()
