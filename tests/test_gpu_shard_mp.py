"""GPU: the sharded LaserMapping with one process per rank (the deployment model), ranks
exchanging through torch.distributed gloo, either as host-buffer callbacks
(loam_amd.comm.TorchDistComm) or as device-pointer callbacks on the mapper's HIP stream
(TorchDistStagedComm, the C-ABI's host_buffers = 0 transport); both processes share the box's one
GPU.  The LM either runs persistent, its per-iteration normal equations meeting in the ranks'
IPC-mapped peer buffers (loam_mapper_lm_path 3, the default across processes), or as two launches
per iteration with the transport's all-reduce between them (LOAM_PEER_LM=0, path 0).  Every rank's
pose equals the unsharded mapper's within 1e-6 and the ranks agree bit for bit; with the peer
wait's bound at 0 (LOAM_PEER_SPIN_LIMIT) the exhausted wait reaches both ranks as LOAM_ERR_SYNC."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import quat_angle, run_sequence
from loam_amd.mapping import BatchMapper

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_FRAMES = 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, frames, q, transport="host", env=None):
    for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(env or {})  # before the library reads it (handle creation)
    import torch.distributed as dist
    from loam_amd.comm import TorchDistComm, TorchDistStagedComm
    from loam_amd.mapping import BatchMapper
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = TorchDistComm.create() if transport == "host" else TorchDistStagedComm.create()
        m = BatchMapper(1, comm=comm)
        path = m.lm_path()
        poses, errors = [], []
        for corner, surf, qo, to in frames:
            m.input(0, corner, surf, qo, to)
            try:
                m.solve()
            except Exception as e:  # noqa: BLE001 - reported to the test (the spin-bound case)
                errors.append(str(e))
            qq, tt = m.pose(0)
            poses.append(np.concatenate([qq, tt]))
        counter = int(m.debug_counters()[40])
        m.close()
        comm.close()
        q.put((rank, np.array(poses), counter, path, errors))
    finally:
        dist.destroy_process_group()


def _run_two(frames, transport, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, frames, q, transport, env)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(2)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("lm", ["ipc", "two_kernel"])
@pytest.mark.parametrize("transport", ["host", "device"])
def test_two_processes_gloo(transport, lm):
    seq = run_sequence(seed=11, n_frames=N_FRAMES)
    frames = [(r["corner"], r["surf"], r["q_wodom"], r["t_wodom"]) for r in seq]
    ref = BatchMapper(1)
    want = []
    for corner, surf, qo, to in frames:
        ref.input(0, corner, surf, qo, to)
        ref.solve()
        qq, tt = ref.pose(0)
        want.append(np.concatenate([qq, tt]))
    ref.close()
    res = _run_two(frames, transport, {"LOAM_PEER_LM": "1" if lm == "ipc" else "0"})
    for r in range(2):
        assert res[r][3] == (3 if lm == "ipc" else 0), res[r][3]  # the LM schedule asked for
        assert res[r][4] == [], res[r][4]
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == 0 and res[1][2] == 0
    for f in range(N_FRAMES):
        got, w = res[0][1][f], want[f]
        assert np.linalg.norm(got[4:] - w[4:]) < 1e-6 and quat_angle(got[:4], w[:4]) < 1e-6, f


def test_two_processes_peer_wait_exhausted():
    """the cross-process LM with the peer wait bounded at 0 spins: at the first Ceres iteration
    the rank that arrives first finds the other's flag down and stops its LM, and the other then
    finds the stopped rank's next flag down: both solves return LOAM_ERR_SYNC (no hang)"""
    seq = run_sequence(seed=11, n_frames=3)
    frames = [(r["corner"], r["surf"], r["q_wodom"], r["t_wodom"]) for r in seq]
    res = _run_two(frames, "host", {"LOAM_PEER_LM": "1", "LOAM_PEER_SPIN_LIMIT": "0"})
    for r in range(2):
        assert res[r][3] == 3
        assert res[r][4], f"rank {r}: no error"
        assert "LOAM_ERR_SYNC" in res[r][4][0], res[r][4]
