"""GPU parity of LaserMapping::solveMapping (laser_mapping.cpp:212-814) against the oracle.

Teacher-forced: the oracle's map state (cubes, cube-grid centre, wmap_T_wodom) before a
frame is loaded into the device mapper, both process the same inputs, then
  - per-scan pose within 1e-4 m / 1e-4 rad (BASELINE.json parity bar; measured ~1e-9),
  - stack / submap sizes and correspondence counts identical (integer work),
  - the map after the update: same cubes, same point counts, points within 1e-5 m.
Free-running: the device mapper consumes the oracle odometry stream for many frames and
stays within 1e-3 m / 1e-3 rad of the oracle trajectory.  The oracle's VoxelGrids sum a voxel's
points in PCL's order, the mapper's kernels in input order: stacks and cube
contents then differ within the float summation-order bound, which these tolerances cover.
Steady-state maps (frame >= 150), recentering at full density and a 300-frame trajectory:
tests/test_gpu_steady_state.py.
"""
import numpy as np
import pytest

from helpers import assert_centroids_within_order_bound, load_state, quat_angle, run_sequence
from loam_amd.mapping import BatchMapper

pytestmark = pytest.mark.gpu

SNAP = (3, 7, 11)


@pytest.fixture(scope="module")
def seq():
    return run_sequence(seed=11, n_frames=12, snapshot_frames=SNAP)


def _check_frame(m, stream, rec):
    q, t = m.pose(stream)
    qr, tr = rec["pose"]
    assert np.linalg.norm(t - tr) < 1e-4, (t, tr)
    assert quat_angle(q, qr) < 1e-4
    st, sr = m.stats(stream), rec["stats"]
    assert st.optimized == sr.optimized
    assert (st.corner_stack, st.surf_stack) == (sr.corner_stack, sr.surf_stack)
    assert (st.corner_map, st.surf_map) == (sr.corner_map, sr.surf_map)
    assert list(st.center) == list(sr.center) and st.valid_num == sr.valid_num
    assert list(st.corner_num) == list(sr.corner_num)
    assert list(st.surf_num) == list(sr.surf_num)
    for r in range(2):
        assert st.lm[r].iterations == sr.lm[r].iterations
    return np.linalg.norm(t - tr), quat_angle(q, qr)


def _check_map(m, stream, after):
    for which, key in ((0, "corner"), (1, "surf")):
        ref = after[key]
        got = m.cubes(stream, which)
        assert sorted(got) == sorted(ref)
        for c in ref:
            a, b = got[c], ref[c]
            assert a.shape == b.shape, (key, c, a.shape, b.shape)
            # a few ulps of the coordinate (the insertion pose differs by ~1e-9: device Cholesky
            # vs DENSE_QR; at 400 m an ulp is 3e-5 m)
            assert np.all(np.abs(a[:, :3] - b[:, :3]) <= 1e-5 + 4e-7 * np.abs(b[:, :3]))


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("fi", SNAP)
def test_teacher_forced_frame(seq, fi, exact):
    rec = seq[fi]
    m = BatchMapper(1, exact_voxel_order=exact)
    load_state(m, 0, rec["before"])
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    _check_frame(m, 0, rec)
    _check_map(m, 0, rec["after"])


def test_batched_streams(seq):
    """three independent streams in one handle, one launch sequence"""
    m = BatchMapper(3)
    for s, fi in enumerate(SNAP):
        load_state(m, s, seq[fi]["before"])
        m.input(s, seq[fi]["corner"], seq[fi]["surf"], seq[fi]["q_wodom"], seq[fi]["t_wodom"])
    m.solve()
    for s, fi in enumerate(SNAP):
        _check_frame(m, s, seq[fi])


def test_free_running(seq):
    m = BatchMapper(1)
    worst_t = worst_r = 0.0
    for rec in seq:
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        q, t = m.pose(0)
        qr, tr = rec["pose"]
        worst_t = max(worst_t, float(np.linalg.norm(t - tr)))
        worst_r = max(worst_r, quat_angle(q, qr))
    assert worst_t < 1e-3 and worst_r < 1e-3, (worst_t, worst_r)


def test_skip_frame_pose(seq):
    """skip_frame: only the high-frequency pose q_wmap_wodom * q_wodom (laser_mapping.cpp:197-201)"""
    m = BatchMapper(1)
    rec = seq[0]
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"], skip_frame=True)
    m.solve()
    q, t = m.pose(0)
    assert np.allclose(q, rec["q_wodom"]) and np.allclose(t, rec["t_wodom"])


@pytest.mark.parametrize("persistent", ["1", "0"])
def test_lm_paths_many_streams(seq, monkeypatch, persistent):
    """both LM implementations (one persistent launch per round / eval + step kernels per pass)
    on 24 streams: each stream is one of the snapshot frames"""
    monkeypatch.setenv("LOAM_LM_PERSISTENT", persistent)
    m = BatchMapper(24)
    for s in range(24):
        fi = SNAP[s % len(SNAP)]
        load_state(m, s, seq[fi]["before"])
        m.input(s, seq[fi]["corner"], seq[fi]["surf"], seq[fi]["q_wodom"], seq[fi]["t_wodom"])
    m.solve()
    for s in range(24):
        _check_frame(m, s, seq[SNAP[s % len(SNAP)]])
    m.close()


@pytest.mark.parametrize("g", ["1", "4", "32"])
def test_lm_workgroups_override(seq, monkeypatch, g):
    """LOAM_LM_G (workgroups per stream of the persistent LM round, read at create): the
    leader's share plus g - 1 claimed shares, reduced in share order, at 1, 4 and 32"""
    monkeypatch.setenv("LOAM_LM_G", g)
    for fi in SNAP[:2]:
        rec = seq[fi]
        m = BatchMapper(1)
        load_state(m, 0, rec["before"])
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        _check_frame(m, 0, rec)
        m.close()


def test_many_streams_exact_order(seq):
    """24 streams in PCL's summation order: the re-VoxelGrid items of all streams go through
    k_insert_bucket's size-class lists (k_revox dispatches them largest first); every stream's
    pose, counts and updated map against the oracle"""
    m = BatchMapper(24, exact_voxel_order=1)
    for s in range(24):
        fi = SNAP[s % len(SNAP)]
        load_state(m, s, seq[fi]["before"])
        m.input(s, seq[fi]["corner"], seq[fi]["surf"], seq[fi]["q_wodom"], seq[fi]["t_wodom"])
    m.solve()
    for s in range(24):
        rec = seq[SNAP[s % len(SNAP)]]
        _check_frame(m, s, rec)
        _check_map(m, s, rec["after"])
    m.close()


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("n_corner,n_surf", [(3000, 9000), (20000, 70000), (6000, 36000)])
def test_stack_voxelgrid_bit_exact(n_corner, n_surf, exact):
    """CornerStack / SurfStack (laser_mapping.cpp:492-500) bit for bit against the oracle
    VoxelGrid: exact_voxel_order = 1 in PCL's order; 0 in input order (single-pass and grouped,
    > VX_UCAP voxels, paths) and within the summation-order bound of PCL's"""
    import loam_oracle as O
    rng = np.random.default_rng(n_surf)

    def cloud(n):  # street-like: a dense ground band plus walls, sensor frame
        g = np.c_[rng.uniform(-60, 60, (n // 2, 2)), rng.normal(-1.7, 0.05, n // 2)]
        w = np.c_[rng.uniform(-60, 60, n - n // 2), rng.choice([-8.0, 8.0], n - n // 2)
                  + rng.normal(0, 0.05, n - n // 2), rng.uniform(-1.7, 12, n - n // 2)]
        xyz = np.concatenate([g, w])[rng.permutation(n)]
        return np.c_[xyz, rng.uniform(0, 64, n)].astype(np.float32)

    corner, surf = cloud(n_corner), cloud(n_surf)
    m = BatchMapper(1, exact_voxel_order=exact)
    m.input(0, corner, surf, np.array([0, 0, 0, 1.0]), np.zeros(3))
    m.solve()
    for which, (c, leaf) in enumerate([(corner, 0.4), (surf, 0.8)]):
        got = m.stack(0, which)
        pcl = O.voxel_grid(c, leaf)
        if exact:
            assert np.array_equal(got.view(np.uint32), pcl.view(np.uint32))
            continue
        with O.voxel_order(1):  # the fast mode sums a voxel's points in input order
            ref = O.voxel_grid(c, leaf)
        assert got.shape == ref.shape
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        assert_centroids_within_order_bound(c, leaf, got, pcl)


def _to_map_np(pose, pts):
    """pointAssociateToMap (laser_mapping.cpp:154-164) with Eigen's _transformVector order"""
    x, y, z, w = (float(v) for v in pose[0])
    t = pose[1]
    out = np.empty_like(pts)
    for i, p in enumerate(pts.astype(np.float64)):
        vx, vy, vz = p[0], p[1], p[2]
        ux, uy, uz = y * vz - z * vy, z * vx - x * vz, x * vy - y * vx
        ux, uy, uz = ux + ux, uy + uy, uz + uz
        cx, cy, cz = y * uz - z * uy, z * ux - x * uz, x * uy - y * ux
        r = ((vx + w * ux) + cx, (vy + w * uy) + cy, (vz + w * uz) + cz)
        out[i, :3] = [np.float32(r[k] + t[k]) for k in range(3)]
        out[i, 3] = pts[i, 3]
    return out


def test_publish_outputs(seq):
    """/laser_cloud_map gather (laser_mapping.cpp:884-899) and the registered full-res cloud
    (:901-911) after a teacher-forced frame"""
    rec = seq[7]
    m = BatchMapper(1)
    load_state(m, 0, rec["before"])
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    got = m.map_cloud(0)
    corner, surf = m.cubes(0, 0), m.cubes(0, 1)
    parts = []
    for c in range(21 * 21 * 11):
        for cubes in (corner, surf):
            if c in cubes:
                parts.append(cubes[c])
    ref = np.concatenate(parts)
    assert np.array_equal(got, ref)
    oref = []
    for c in range(21 * 21 * 11):
        for key in ("corner", "surf"):
            if c in rec["after"][key]:
                oref.append(rec["after"][key][c])
    oref = np.concatenate(oref)
    assert got.shape == oref.shape and np.max(np.abs(got[:, :3] - oref[:, :3])) < 1e-5
    cloud = np.concatenate([rec["corner"], rec["surf"]])[:3000]
    reg = m.register_cloud(0, cloud)
    assert np.array_equal(reg, _to_map_np(m.pose(0), cloud))
    assert len(m.register_cloud(0, np.zeros((0, 4), np.float32))) == 0


def test_recentering_frame():
    """a frame whose pose crosses the cube-grid recentering threshold (laser_mapping.cpp:252-444:
    the grid shifts by one cube, wrapped slabs cleared), teacher-forced from the oracle state:
    pose, counts, grid centre and the shifted map"""
    frames = (384, 385, 386, 387, 388)
    seq = run_sequence(seed=11, n_frames=frames[-1] + 1, n_az=600, snapshot_frames=frames)
    shifted = [f for f in frames if not np.array_equal(seq[f]["before"]["cen"], seq[f]["after"]["cen"])]
    assert shifted, "no recentering in the probed frames"
    rec = seq[shifted[0]]
    m = BatchMapper(1)
    load_state(m, 0, rec["before"])
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    _check_frame(m, 0, rec)
    cen, _, _ = m.get_state(0)
    assert np.array_equal(cen, rec["after"]["cen"])
    _check_map(m, 0, rec["after"])
    # and the frame after it, free-running on the device
    nxt = seq[shifted[0] + 1] if shifted[0] + 1 < len(seq) else None
    if nxt is not None:
        m.input(0, nxt["corner"], nxt["surf"], nxt["q_wodom"], nxt["t_wodom"])
        m.solve()
        q, t = m.pose(0)
        assert np.linalg.norm(t - nxt["pose"][1]) < 1e-4 and quat_angle(q, nxt["pose"][0]) < 1e-4


@pytest.mark.parametrize("n_streams", [1, 8])
def test_arena_compaction_is_transparent(seq, n_streams):
    """a small arena compacts several times (queued at the start of the next frame, decided on
    the device per (stream, map)); poses, statistics and maps stay bit-identical to a mapper
    whose arena never fills.  One stream runs the graph path (a frame with a compaction due
    leaves it), eight streams the batched path."""
    small = dict(max_input_points=32768, max_submap_points=16384, max_map_points=131072)
    big = dict(max_input_points=32768, max_submap_points=16384)
    ms, mb = BatchMapper(n_streams, **small), BatchMapper(n_streams, **big)
    ms.debug_counters(reset=True)
    for k, rec in enumerate(seq):
        for m in (ms, mb):
            for s in range(n_streams):
                r = seq[(k + s) % len(seq)] if n_streams > 1 else rec
                m.input(s, r["corner"], r["surf"], r["q_wodom"], r["t_wodom"])
            m.solve()
        for s in range(n_streams):
            (qs, ts), (qb, tb) = ms.pose(s), mb.pose(s)
            assert np.array_equal(qs, qb) and np.array_equal(ts, tb), (k, s)
            a, b = ms.stats(s), mb.stats(s)
            assert (a.corner_map, a.surf_map, list(a.corner_num), list(a.surf_num)) == \
                (b.corner_map, b.surf_map, list(b.corner_num), list(b.surf_num))
    assert ms.debug_counters()[41] >= n_streams  # compactions happened
    assert mb.debug_counters()[41] == 0
    for s in range(n_streams):
        for which in range(2):
            cs, cb = ms.cubes(s, which), mb.cubes(s, which)
            assert sorted(cs) == sorted(cb)
            for c in cb:
                assert np.array_equal(cs[c], cb[c])
    ms.close()
    mb.close()


def test_concurrent_handles_share_the_gpu(seq):
    """two 64-stream handles, each sizing its persistent LM grid for the whole GPU, solve at the
    same time from two host threads: the LM shares are claimed by whichever workgroups run
    (lm.h), so neither waits on workgroups the other keeps off the GPU; poses are bit-identical
    to one handle running alone"""
    import threading
    B, n = 64, 6
    caps = dict(max_input_points=32768, max_submap_points=16384, max_map_points=262144)

    def feed(m, k):
        for s in range(B):
            r = seq[(k + s) % len(seq)]
            m.input(s, r["corner"], r["surf"], r["q_wodom"], r["t_wodom"])

    ref = BatchMapper(B, **caps)
    want = []
    for k in range(n):
        feed(ref, k)
        ref.solve()
        want.append([ref.pose(s) for s in range(B)])
    ref.close()
    ms = [BatchMapper(B, **caps) for _ in range(2)]
    got = [[None] * n for _ in ms]
    errs = []

    def run(i):
        try:
            for k in range(n):
                feed(ms[i], k)
                ms[i].solve()
                got[i][k] = [ms[i].pose(s) for s in range(B)]
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    for i in range(2):
        for k in range(n):
            for s in range(B):
                (q, t), (qr, tr) = got[i][k][s], want[k][s]
                assert np.array_equal(q, qr) and np.array_equal(t, tr), (i, k, s)
        ms[i].close()


def test_graph_path_bit_identical(seq):
    """handles of <= 4 streams run each frame as one hipGraph; with profiling on (per-launch
    events) the same sequence runs as individual launches: poses, statistics and maps
    bit-identical"""
    runs = []
    for prof in (False, True):
        m = BatchMapper(4, max_input_points=32768, max_submap_points=16384, max_map_points=262144)
        m.set_profiling(prof)
        poses, stats = [], []
        for k in range(8):
            for s in range(4):
                r = seq[(k + s) % len(seq)]
                m.input(s, r["corner"], r["surf"], r["q_wodom"], r["t_wodom"])
            m.solve()
            poses.append([m.pose(s) for s in range(4)])
            stats.append([(m.stats(s).corner_map, m.stats(s).surf_map, tuple(m.stats(s).corner_num),
                           tuple(m.stats(s).surf_num)) for s in range(4)])
        runs.append((poses, stats, [[m.cubes(s, w) for w in range(2)] for s in range(4)]))
        m.close()
    (pa, sa, ma), (pb, sb, mb) = runs
    assert sa == sb
    for k in range(len(pa)):
        for s in range(4):
            assert np.array_equal(pa[k][s][0], pb[k][s][0]) and np.array_equal(pa[k][s][1], pb[k][s][1]), (k, s)
    for s in range(4):
        for w in range(2):
            assert sorted(ma[s][w]) == sorted(mb[s][w])
            for c in ma[s][w]:
                assert np.array_equal(ma[s][w][c], mb[s][w][c])


def _cube_of(v, cen):
    """laser_mapping.cpp:747-756: int((v + 25) / 50) + cen, one less when v + 25 < 0"""
    c = int((np.float32(v) + np.float32(25.0)) / np.float32(50.0)) + int(cen)
    return c - 1 if np.float32(v) + np.float32(25.0) < 0 else c


def edge_state(rec, axis_bounds=((0, -75.0), (1, -75.0), (0, -125.0), (1, -125.0))):
    """the frame's map with every point within 0.5 m of the busiest plane v = B (B + 25 a negative
    multiple of 50) moved onto it and re-filed by the reference's cube rule: cells at v = B hold
    points in two cubes (the cube above at local 0, the cube below at local 50 for v == B)"""
    from scipy.spatial.transform import Rotation as R
    import loam_oracle as O
    before = rec["before"]
    x0 = rec["round_pose"][0]
    qs = np.concatenate([O.voxel_grid(rec["corner"], 0.4), O.voxel_grid(rec["surf"], 0.8)])[:, :3]
    qm = R.from_quat(x0[:4]).apply(qs.astype(np.float64)) + x0[4:]
    axis, b = max(axis_bounds, key=lambda ab: int((np.abs(qm[:, ab[0]] - ab[1]) < 1.0).sum()))
    cen = before["cen"]
    out = dict(cen=cen, q=before["q"], t=before["t"])
    moved = 0
    for key in ("corner", "surf"):
        cubes = {}
        for c, pts in before[key].items():
            for p in pts:
                p = p.copy()
                ijk = [c % 21, (c // 21) % 21, c // 441]
                if abs(float(p[axis]) - b) < 0.5:
                    p[axis] = np.float32(b)
                    ijk[axis] = _cube_of(p[axis], cen[axis])
                    moved += 1
                cubes.setdefault(ijk[0] + 21 * ijk[1] + 441 * ijk[2], []).append(p)
        out[key] = {c: np.array(v, np.float32) for c, v in cubes.items()}
    near = int((np.abs(qm[:, axis] - b) < 1.0).sum())
    return out, moved, near


def test_cube_edge_filing():
    """queries next to a plane v = B where B + 25 is a negative multiple of 50: map points with
    v == B exactly sit in the cube below at local coordinate 50 (laser_mapping.cpp:747-756) while
    the rest of the cell is in the cube above; k_knn scans both.  Against the oracle from the
    same modified state: identical counts and iterations, pose within 1e-4"""
    import loam_oracle as O
    seq = run_sequence(seed=23, n_frames=3, snapshot_frames=(2,))
    rec = seq[2]
    state, moved, near = edge_state(rec)
    assert moved > 20 and near > 40, (moved, near)
    ref = O.LaserMapping()
    ref.set_state(state["cen"], state["q"], state["t"])
    for which, key in ((0, "corner"), (1, "surf")):
        for c, pts in state[key].items():
            ref.set_cube(which, c, pts)
    ref.input(rec["corner"], rec["surf"], None, rec["q_wodom"], rec["t_wodom"])
    ref.solve()
    want = dict(pose=ref.pose(), stats=ref.stats())
    for exact in (1, 0):
        m = BatchMapper(1, exact_voxel_order=exact)
        load_state(m, 0, state)
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        _check_frame(m, 0, want)
        m.close()


@pytest.mark.parametrize("n_streams,exact", [(1, 0), (1, 1), (6, 0)])
def test_async_solve_with_prefetched_stacks(seq, n_streams, exact):
    """loam_mapper_solve_async / _prefetch / _wait (include/loam_core.h): frame f + 1's input is
    given and its stack VoxelGrid queued while frame f is in flight (double-buffered stacks);
    every pose and count equals the blocking loam_mapper_solve, bit for bit.  One stream takes
    the hipGraph path, six the kernel-by-kernel path; host inputs copy on the stack stream"""
    def row(m, s):
        st = m.stats(s)
        q, t = m.pose(s)
        return (q.tobytes(), t.tobytes(), st.corner_stack, st.surf_stack, tuple(st.corner_num), tuple(st.surf_num),
                st.lm[0].iterations, st.lm[1].iterations)

    def feed(m, f):
        for s in range(n_streams):
            rec = seq[f + s]  # stream s runs the sequence s frames ahead
            m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])

    n = len(seq) - n_streams + 1
    ref = BatchMapper(n_streams, exact_voxel_order=exact)
    want = []
    for f in range(n):
        feed(ref, f)
        ref.solve()
        want.append([row(ref, s) for s in range(n_streams)])
    ref.close()
    m = BatchMapper(n_streams, exact_voxel_order=exact)
    got = []
    feed(m, 0)
    m.solve_async()
    for f in range(1, n + 1):
        if f < n:
            feed(m, f)  # while frame f - 1 is in flight
            m.prefetch()
        m.wait()
        got.append([row(m, s) for s in range(n_streams)])
        if f < n:
            m.solve_async()
    m.close()
    assert got == want


@pytest.mark.parametrize("n_streams,exact,defer_every", [(1, 0, 0), (1, 1, 0), (2, 0, 0), (1, 0, 3), (2, 0, 2)])
def test_chained_solve_matches_blocking(seq, n_streams, exact, defer_every, monkeypatch):
    """frames queued behind the one in flight (loam_mapper_solve_async on a graph-path handle,
    include/loam_core.h): frame f + 1 is enqueued before frame f is waited for, its stream records
    prepared on the device (k_frame_prep: transformUpdate, initial guess, window); every pose and
    count equals the blocking loam_mapper_solve, bit for bit.  defer_every > 0 forces the
    deferral path (LOAM_DEFER_EVERY: queued frames whose frame number is a multiple are left to
    the host, which runs them again with their own inputs and stacks)"""
    def row(m, s):
        st = m.stats(s)
        q, t = m.pose(s)
        return (q.tobytes(), t.tobytes(), st.corner_stack, st.surf_stack, tuple(st.corner_num), tuple(st.surf_num),
                st.lm[0].iterations, st.lm[1].iterations, tuple(st.center), st.valid_num)

    def feed(m, f):
        for s in range(n_streams):
            rec = seq[f + s]
            m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])

    n = len(seq) - n_streams + 1
    ref = BatchMapper(n_streams, exact_voxel_order=exact)
    want = []
    for f in range(n):
        feed(ref, f)
        ref.solve()
        want.append([row(ref, s) for s in range(n_streams)])
    ref.close()
    if defer_every:
        monkeypatch.setenv("LOAM_DEFER_EVERY", str(defer_every))
    m = BatchMapper(n_streams, exact_voxel_order=exact)
    monkeypatch.delenv("LOAM_DEFER_EVERY", raising=False)
    got, queued, rerun = [], 0, 0
    feed(m, 0)
    m.solve_async()
    for f in range(1, n + 1):
        if f < n:
            feed(m, f)
            m.solve_async()  # queued behind frame f - 1
        m.wait()             # frame f - 1
        got.append([row(m, s) for s in range(n_streams)])
        queued += m.stats(0).queued
        rerun += m.stats(0).rerun
    m.close()
    assert got == want
    if defer_every:
        assert queued > 0 and rerun > 0, (queued, rerun)
    else:
        assert queued >= n - 2, queued  # every frame but the first ran queued behind another


@pytest.mark.parametrize("n_streams,exact,defer_every", [(1, 0, 0), (1, 1, 0), (3, 0, 0), (1, 0, 3), (6, 0, 0)])
def test_solve_pose_matches_blocking(seq, n_streams, exact, defer_every, monkeypatch):
    """loam_mapper_solve_pose (include/loam_core.h): each call returns at the frame's poses, its
    map update finishing beside the next frame; poses, counts and iterations after every frame,
    then every cube of the final maps, equal the blocking loam_mapper_solve bit for bit.
    defer_every > 0: frames the device defers are finished whole (run again on the host path);
    6 streams: the handle does not run frames as a graph, every frame is finished whole."""
    def row(m, s):
        st = m.stats(s)
        q, t = m.pose(s)
        return (q.tobytes(), t.tobytes(), st.corner_stack, st.surf_stack, tuple(st.corner_num), tuple(st.surf_num),
                st.lm[0].iterations, st.lm[1].iterations, tuple(st.center), st.valid_num, m.total_iterations())

    def feed(m, f):
        for s in range(n_streams):
            rec = seq[f + s]
            m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])

    def maps(m):
        return [[m.cubes(s, w) for w in (0, 1)] for s in range(n_streams)]

    n = len(seq) - n_streams + 1
    ref = BatchMapper(n_streams, exact_voxel_order=exact)
    want = []
    for f in range(n):
        feed(ref, f)
        ref.solve()
        want.append([row(ref, s) for s in range(n_streams)])
    want_maps = maps(ref)
    ref.close()
    if defer_every:
        monkeypatch.setenv("LOAM_DEFER_EVERY", str(defer_every))
    m = BatchMapper(n_streams, exact_voxel_order=exact)
    monkeypatch.delenv("LOAM_DEFER_EVERY", raising=False)
    got = []
    for f in range(n):
        feed(m, f)
        m.solve_pose()
        got.append([row(m, s) for s in range(n_streams)])
    got_maps = maps(m)  # (finishes the last frame's map update first)
    m.close()
    assert got == want
    for gs, ws in zip(got_maps, want_maps):
        for gc, wc in zip(gs, ws):
            assert sorted(gc) == sorted(wc)
            assert all(np.array_equal(gc[c], wc[c]) for c in wc)


@pytest.mark.parametrize("exact", [0, 1])
@pytest.mark.parametrize("n_streams", [2, 16])
def test_split_prefetch_matches_blocking(seq, exact, n_streams):
    """streams of one frame taking their stacks from two different stack launches of the same
    parity: the first half of the streams get their inputs and their stack VoxelGrids launched
    (loam_mapper_prefetch), then the other half, whose stacks the solve launches; the frames queue
    behind each other.  The stack points are written by k_stack_ds on the second HIP stream and
    read by the kNN / insertion kernels on the first, on whichever XCD they land: k_frame_prep
    waits for each stream's own stack launch (relaxed agent-scope loads of the launch counter and
    of the stack sizes, which share cache lines), and the points themselves are ordered by kernel
    boundaries (k_stack_ds's end-of-kernel release before k_stack_done's counter store on its
    stream; the consumers' start-of-kernel acquire after k_frame_prep saw the counter; DESIGN.md
    §6).  At 16 streams the stacks of one frame come from both launches, blocks of many XCDs.
    Every pose and count equals the blocking solve"""
    half = n_streams // 2

    def row(m, s):
        st = m.stats(s)
        q, t = m.pose(s)
        return (q.tobytes(), t.tobytes(), st.corner_stack, st.surf_stack, tuple(st.corner_num), tuple(st.surf_num),
                st.lm[0].iterations, st.lm[1].iterations)

    def give(m, f, s):
        rec = seq[f + s % 4]
        m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])

    n = len(seq) - 3
    ref = BatchMapper(n_streams, exact_voxel_order=exact)
    want = []
    for f in range(n):
        for s in range(n_streams):
            give(ref, f, s)
        ref.solve()
        want.append([row(ref, s) for s in range(n_streams)])
    ref.close()
    m = BatchMapper(n_streams, exact_voxel_order=exact)
    got = []
    for f in range(n):
        for s in range(half):
            give(m, f, s)
        m.prefetch()  # the first half's stacks: their own launch
        for s in range(half, n_streams):
            give(m, f, s)
        m.solve_async()  # the second half's stacks launched here; queued behind frame f - 1
        if f:
            m.wait()
            got.append([row(m, s) for s in range(n_streams)])
    m.wait()
    got.append([row(m, s) for s in range(n_streams)])
    m.close()
    assert got == want


@pytest.mark.parametrize("exact", [0, 1])
def test_pipelined_frames_with_profiling(seq, exact):
    """bench.py's timed steps: each frame given and enqueued (loam_mapper_solve_async) before the
    previous one is waited for, with per-launch HIP events on.  At 8 streams (no hipGraph chain)
    the queued frame's stack VoxelGrid runs beside the frame in flight and the rest is enqueued by
    the wait that finishes it; a launch whose events have not passed when a frame is finished
    (that stack VoxelGrid) stays listed for a later frame instead of failing the read.  Poses and
    counts equal the blocking solve's; every family is timed, the stack's once per frame."""
    n_streams = 8

    def row(m, s):
        st = m.stats(s)
        q, t = m.pose(s)
        return (q.tobytes(), t.tobytes(), st.corner_stack, st.surf_stack, tuple(st.corner_num), tuple(st.surf_num),
                st.lm[0].iterations, st.lm[1].iterations)

    def give(m, f):
        for s in range(n_streams):
            rec = seq[f + s % 4]
            m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])

    n = len(seq) - 3
    ref = BatchMapper(n_streams, exact_voxel_order=exact)
    want = []
    for f in range(n):
        give(ref, f)
        ref.solve()
        want.append([row(ref, s) for s in range(n_streams)])
    ref.close()
    m = BatchMapper(n_streams, exact_voxel_order=exact)
    m.set_profiling(True)
    got = []
    give(m, 0)
    m.solve_async()
    for f in range(1, n + 1):
        if f < n:
            give(m, f)
            m.solve_async()  # its stack VoxelGrid beside frame f - 1
        m.wait()             # frame f - 1 (and frame f enqueued)
        got.append([row(m, s) for s in range(n_streams)])
    kt = m.kernel_times()
    m.close()
    assert got == want
    assert kt["stack_voxelgrid"]["launches"] == n, kt["stack_voxelgrid"]
    assert kt["correspondence"]["launches"] > 0 and kt["cube_revoxel"]["launches"] > 0
    assert all(v["ms"] >= 0.0 for v in kt.values())


def test_async_capacity_error_is_held_for_wait(seq):
    """loam_mapper_solve_async returns OK exactly when it enqueued its frame.  With two frames in
    the queue it first finishes the oldest; when that one fails (here: its submap exceeds
    max_submap_points, a LOAM_ERR_CAPACITY committed as computed), the status is held and the next
    wait returns LOAM_ERR_EARLIER, so a caller that re-submits on a failed solve_async cannot
    queue a frame twice.  Every frame runs exactly once: the poses equal the blocking solve's,
    which reports the same frames as failed."""
    from loam_amd._core import LoamError

    probe = BatchMapper(1)
    sizes = []
    for rec in seq:
        probe.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        probe.solve()
        st = probe.stats(0)
        sizes.append(max(st.corner_map, st.surf_map))
    probe.close()
    cap = sizes[5] + 1  # frames whose submap is larger fail from here on
    assert any(v >= cap for v in sizes[6:]), sizes

    def pose(m):
        q, t = m.pose(0)
        return np.concatenate([q, t]).tobytes()

    ref = BatchMapper(1, max_submap_points=cap)
    want, want_fail = [], []
    for rec in seq:
        ref.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        try:
            ref.solve()
            want_fail.append(False)
        except LoamError as e:
            assert e.rc == -3, e
            want_fail.append(True)
        want.append(pose(ref))
    ref.close()
    assert any(want_fail) and not all(want_fail), want_fail

    m = BatchMapper(1, max_submap_points=cap)
    earlier = 0
    for f, rec in enumerate(seq):
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve_async()  # never raises here: every frame is enqueued (two in the queue from f = 1)
    fails = 0
    for _ in range(3):  # the last two frames, then the held status of the earlier ones
        try:
            m.wait()
        except LoamError as e:
            assert e.rc in (-3, -7), e
            fails += 1
            earlier += e.rc == -7
    # the frames solve_async finished were failures held for a wait: at least one was reported
    assert earlier >= 1
    # every frame ran exactly once: the final pose is the blocking solve's
    assert pose(m) == want[-1]
    m.close()

    # loam_mapper_solve_pose: a failure found before the map update (here the submap size) is
    # returned by the call of its own frame, as by the blocking solve, with the same poses
    m = BatchMapper(1, max_submap_points=cap)
    got, got_fail = [], []
    for rec in seq:
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        try:
            m.solve_pose()
            got_fail.append(False)
        except LoamError as e:
            assert e.rc == -3, e
            got_fail.append(True)
        got.append(pose(m))
    m.close()
    assert got_fail == want_fail and got == want


@pytest.mark.parametrize("target", [35000, 46000])
def test_exact_refilter_of_a_cube_over_lds(seq, target):
    """PCL's order for a window cube of more than VH_MAX_N (30720) points: set through the API it
    is not a VoxelGrid fixed point, so the reference re-filters it (laser_mapping.cpp:795-808).  Up
    to VH_BIG_N (40000) the first partition runs in global memory and the parts in LDS
    (voxel_hot.h vh_sort_big); above it the whole sort runs in global memory.  The same frame
    through the oracle from the same state: equal poses within the solve tolerance, equal maps."""
    import loam_oracle as O
    from helpers import snapshot
    rec = seq[SNAP[0]]
    before = dict(rec["before"])
    surf = dict(before["surf"])
    cube = max(surf, key=lambda c: len(surf[c]))
    pts = surf[cube]
    lo, hi = pts[:, :3].min(0), pts[:, :3].max(0)
    rng = np.random.default_rng(3)
    n = target - len(pts)  # the cube's points in all; 5 cm quantization: many voxels of 3+ members
    extra = np.round(rng.uniform(lo, hi, (n, 3)) * 20) / 20
    surf[cube] = np.concatenate([pts, np.c_[extra, rng.uniform(0, 64, n)].astype(np.float32)])
    before["surf"] = surf
    assert len(surf[cube]) > 30720
    ref = O.LaserMapping()
    ref.set_state(before["cen"], before["q"], before["t"])
    for which, key in ((0, "corner"), (1, "surf")):
        for c, p in before[key].items():
            ref.set_cube(which, c, p)
    ref.input(rec["corner"], rec["surf"], None, rec["q_wodom"], rec["t_wodom"])
    ref.solve()
    after = snapshot(ref)
    m = BatchMapper(1, exact_voxel_order=1, max_submap_points=400000)
    load_state(m, 0, before)
    m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
    m.solve()
    q, t = m.pose(0)
    qr, tr = ref.pose()
    assert np.linalg.norm(t - tr) < 1e-4 and quat_angle(q, qr) < 1e-4
    _check_map(m, 0, after)
    assert len(after["surf"][cube]) < len(surf[cube])  # the re-filter merged the duplicates
    m.close()


@pytest.mark.parametrize("exact", [1, 0])
def test_cube_content_outside_its_bounds(seq, exact):
    """content set through the API need not lie in its cube: a merge of such a cube keys its
    voxels from the cube's corner only while every point lies in the cube's key box
    (VoxSeg::anchored), else it takes the full filter.  The centre cube (which every frame's
    insertion reaches) holds extra points 600 m above it (no query comes near them: a kNN of the
    cube's cell index, which keys cells inside the cube, and the oracle's KD-tree agree); three
    frames from that state against the oracle from the same state: poses, counts and (PCL order)
    maps as the oracle's"""
    import loam_oracle as O
    rec = seq[7]
    state = {k: (dict(v) if isinstance(v, dict) else v) for k, v in rec["before"].items()}
    c = rec["stats"].center
    cube = int(c[0] + 21 * c[1] + 441 * c[2])
    for key in ("corner", "surf"):
        pts = state[key].get(cube)
        assert pts is not None and len(pts) > 100
        far = pts[: len(pts) // 3].copy()
        far[:, 2] += 600.0
        state[key][cube] = np.concatenate([pts, far])
    ref = O.LaserMapping()
    ref.set_state(state["cen"], state["q"], state["t"])
    for which, key in ((0, "corner"), (1, "surf")):
        for cb, pts in state[key].items():
            ref.set_cube(which, cb, pts)
    m = BatchMapper(1, exact_voxel_order=exact)
    load_state(m, 0, state)
    for f in (7, 8, 9):
        r = seq[f]
        ref.input(r["corner"], r["surf"], None, r["q_wodom"], r["t_wodom"])
        ref.solve()
        m.input(0, r["corner"], r["surf"], r["q_wodom"], r["t_wodom"])
        m.solve()
        _check_frame(m, 0, dict(pose=ref.pose(), stats=ref.stats()))
    if exact:  # (points within a few ulps: the insertion poses differ by ~1e-9, Cholesky vs QR)
        _check_map(m, 0, {"corner": ref.cubes(0), "surf": ref.cubes(1)})
        assert len(m.cubes(0, 1)[cube]) == len(ref.cubes(1)[cube])
    m.close()
