"""GPU: the sharded LaserMapping (include/loam_core.h "Sharded LaserMapping").

One mapping stream split over R ranks (threads of this process on the one GPU of the box,
meeting in loam_amd.comm.ThreadGroup collectives or in the library's device-ordered transport
Comm.local_group; RCCL with one rank for the transport):
  - every rank ends every frame with the bit-identical pose (same all-reduced sums, same step);
  - poses, submap sizes, correspondence and LM iteration counts equal the unsharded mapper's;
  - the union of the ranks' cubes is the unsharded map, point for point (bit-exact), and every
    rank stores only points of the 4 m blocks it owns;
  - teacher-forced from the oracle's map state: the oracle's pose within 1e-4 m / 1e-4 rad and
    its correspondence counts.
"""
import threading

import numpy as np
import pytest

from helpers import load_state, quat_angle, run_sequence
from loam_amd.comm import Comm, ThreadGroup
from loam_amd.mapping import BatchMapper, shard_owner

pytestmark = pytest.mark.gpu

N_FRAMES = 12


@pytest.fixture(scope="module")
def seq():
    return run_sequence(seed=11, n_frames=N_FRAMES, snapshot_frames=(7,))


@pytest.fixture(scope="module")
def unsharded(seq):
    m = BatchMapper(1)
    out = []
    for rec in seq:
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        out.append((m.pose(0), _stat_tuple(m.stats(0))))
    maps = [m.cubes(0, 0), m.cubes(0, 1)]
    m.close()
    return out, maps


def _stat_tuple(st):
    return (st.optimized, st.corner_stack, st.surf_stack, st.corner_map, st.surf_map, tuple(st.corner_num),
            tuple(st.surf_num), st.lm[0].iterations, st.lm[1].iterations, tuple(st.center), st.valid_num)


def _run_ranks(size, body, transport="threads"):
    """body(rank, comm) on `size` threads; returns the per-rank results, re-raises failures.
    transport "threads": host-buffer callbacks meeting in Python (ThreadGroup); "device": the
    library's device-ordered transport (Comm.local_group: on-stream staging and sums, events)"""
    group = ThreadGroup(size) if transport == "threads" else None
    comms = [group.comm(r) for r in range(size)] if group else Comm.local_group(size)
    res, errs = [None] * size, []

    def run(r):
        try:
            res[r] = body(r, comms[r])
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            if group:
                group.barrier.abort()  # release the other ranks' collectives (device: they time out)

    th = [threading.Thread(target=run, args=(r,)) for r in range(size)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errs:
        raise errs[0]
    assert all(not t.is_alive() for t in th)
    if not group:
        for c in comms:
            c.close()
    return res


def _sequence_body(seq):
    def body(rank, comm):
        m = BatchMapper(1, comm=comm)
        poses, stats = [], []
        for rec in seq:
            m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
            m.solve()
            poses.append(m.pose(0))
            stats.append(_stat_tuple(m.stats(0)))
        maps = [m.cubes(0, 0), m.cubes(0, 1)]
        assert m.debug_counters()[40] == 0  # every rank's LM ended on rank 0's pose bits
        m.close()
        return poses, stats, maps
    return body


def _rows(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a[np.lexsort(a.T[::-1])] if len(a) else a


def test_single_rank_comm_matches_unsharded(seq, unsharded):
    """the sharded code path at one rank (trivial collectives) is the unsharded mapper"""
    ref, ref_maps = unsharded
    c = Comm.single()
    poses, stats, maps = _sequence_body(seq)(0, c)
    for (q, t), ((qr, tr), sr), st in zip(poses, ref, stats):
        assert st == sr
        assert np.linalg.norm(t - tr) < 1e-7 and quat_angle(q, qr) < 1e-7
    for which in range(2):
        assert sorted(maps[which]) == sorted(ref_maps[which])
        for cube, pts in ref_maps[which].items():
            assert np.array_equal(_rows(maps[which][cube]), _rows(pts))


@pytest.mark.parametrize("size,transport", [(2, "threads"), (3, "threads"), (2, "device"), (3, "device")])
def test_ranks_match_unsharded(seq, unsharded, size, transport):
    ref, ref_maps = unsharded
    res = _run_ranks(size, _sequence_body(seq), transport)
    for f in range(N_FRAMES):
        q0, t0 = res[0][0][f]
        for r in range(1, size):  # identical step on every rank
            q, t = res[r][0][f]
            assert np.array_equal(q, q0) and np.array_equal(t, t0), (f, r)
            assert res[r][1][f] == res[0][1][f]
        (qr, tr), sr = ref[f]
        st = res[0][1][f]
        assert st == sr, (f, st, sr)
        assert np.linalg.norm(t0 - tr) < 1e-6 and quat_angle(q0, qr) < 1e-6, f
    leaf = (0.4, 0.8)
    for which in range(2):
        cubes = set()
        for r in range(size):
            cubes |= set(res[r][2][which])
            for pts in res[r][2][which].values():  # each rank stores only its blocks
                for p in pts[:: max(1, len(pts) // 50)]:
                    assert shard_owner(p, leaf[which], size) == r
        assert cubes == set(ref_maps[which])
        for cube, pts in ref_maps[which].items():
            parts = [res[r][2][which][cube] for r in range(size) if cube in res[r][2][which]]
            assert np.array_equal(_rows(np.concatenate(parts)), _rows(pts)), (which, cube)


def test_teacher_forced_two_ranks(seq):
    rec = seq[7]

    def body(rank, comm):
        m = BatchMapper(1, comm=comm)
        load_state(m, 0, rec["before"])  # cube_set keeps this rank's blocks
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        out = m.pose(0), m.stats(0)
        m.close()
        return out

    for (q, t), st in _run_ranks(2, body):
        qr, tr = rec["pose"]
        sr = rec["stats"]
        assert np.linalg.norm(t - tr) < 1e-4 and quat_angle(q, qr) < 1e-4
        assert (st.corner_map, st.surf_map) == (sr.corner_map, sr.surf_map)
        assert list(st.corner_num) == list(sr.corner_num) and list(st.surf_num) == list(sr.surf_num)
        assert [st.lm[r].iterations for r in range(2)] == [sr.lm[r].iterations for r in range(2)]


def test_rccl_one_rank(seq, unsharded):
    """RCCL transport (run-time loaded librccl): one rank, collectives on the mapper's stream"""
    ref, _ = unsharded
    c = Comm.rccl(0, 1, Comm.rccl_unique_id(), 0)
    m = BatchMapper(1, comm=c)
    for rec, ((qr, tr), sr) in zip(seq[:6], ref[:6]):
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        m.solve()
        q, t = m.pose(0)
        assert _stat_tuple(m.stats(0)) == sr
        assert np.linalg.norm(t - tr) < 1e-7 and quat_angle(q, qr) < 1e-7
    m.close()
    c.close()


def test_device_group_mappers_in_turn(seq, unsharded):
    """two sharded mappers created one after the other on the same Comm.local_group: the group's
    LM peer buffer is re-bound (zeroed) for the second, whose epochs count from 1 again (before,
    the first mapper's larger flags let the second's leaders sum stale peer slots: ADVICE r5)"""
    ref, _ = unsharded

    def body(rank, comm):
        out = []
        for n in (N_FRAMES, 6):
            m = BatchMapper(1, comm=comm)
            poses = []
            for rec in seq[:n]:
                m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
                m.solve()
                poses.append((m.pose(0), _stat_tuple(m.stats(0))))
            m.close()
            out.append(poses)
        return out

    res = _run_ranks(2, body, "device")
    for run in range(2):
        for f, ((qr, tr), sr) in enumerate(ref[:len(res[0][run])]):
            (q0, t0), s0 = res[0][run][f]
            (q1, t1), s1 = res[1][run][f]
            assert np.array_equal(q0, q1) and np.array_equal(t0, t1), (run, f)
            assert s0 == sr and s1 == sr, (run, f)
            assert np.linalg.norm(t0 - tr) < 1e-6 and quat_angle(q0, qr) < 1e-6, (run, f)


def test_device_group_beside_a_busy_handle(seq, unsharded):
    """a 2-rank in-process group (persistent group LM: its leaders wait for each other inside one
    launch) solving while an unsharded 8-stream handle runs its own frames on the same GPU from a
    third thread: the group's leaders are dispatched whatever the other handle holds (its kernels
    end on their own), and both give the unsharded results bit for bit"""
    ref, _ = unsharded
    comms = Comm.local_group(2)
    res, errs = [None] * 3, []
    start = threading.Barrier(3)

    def ranks(r):
        try:
            m = BatchMapper(1, comm=comms[r])
            start.wait()
            out = []
            for rec in seq:
                m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
                m.solve()
                out.append((m.pose(0), _stat_tuple(m.stats(0))))
            m.close()
            res[r] = out
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            start.abort()

    def busy():
        try:
            m = BatchMapper(8)
            start.wait()
            out = []
            for rec in seq:
                for s in range(8):
                    m.input(s, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
                m.solve()
                out.append([(m.pose(s), _stat_tuple(m.stats(s))) for s in range(8)])
            m.close()
            res[2] = out
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            start.abort()

    th = [threading.Thread(target=ranks, args=(r,)) for r in range(2)] + [threading.Thread(target=busy)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for c in comms:
        c.close()
    if errs:
        raise errs[0]
    assert all(not t.is_alive() for t in th)
    for f, ((qr, tr), sr) in enumerate(ref):
        (q0, t0), s0 = res[0][f]
        (q1, t1), s1 = res[1][f]
        assert np.array_equal(q0, q1) and np.array_equal(t0, t1), f
        assert s0 == sr, (f, s0, sr)
        assert np.linalg.norm(t0 - tr) < 1e-6 and quat_angle(q0, qr) < 1e-6, f
        for (q, t), st in res[2][f]:  # the busy handle's streams: the unsharded mapper's bits
            assert st == sr and np.array_equal(q, qr) and np.array_equal(t, tr), f
