"""GPU: the sharded LaserMapping with one process per rank (the deployment model), ranks
exchanging through torch.distributed gloo, either as host-buffer callbacks
(loam_amd.comm.TorchDistComm) or as device-pointer callbacks on the mapper's HIP stream
(TorchDistStagedComm, the C-ABI's host_buffers = 0 transport); both processes share the box's one
GPU.  Every rank's pose equals the unsharded mapper's within 1e-6 and the ranks agree bit for
bit."""
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


def _rank(rank, world, port, frames, q, transport="host"):
    for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from loam_amd.comm import TorchDistComm, TorchDistStagedComm
    from loam_amd.mapping import BatchMapper
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = TorchDistComm.create() if transport == "host" else TorchDistStagedComm.create()
        m = BatchMapper(1, comm=comm)
        poses = []
        for corner, surf, qo, to in frames:
            m.input(0, corner, surf, qo, to)
            m.solve()
            qq, tt = m.pose(0)
            poses.append(np.concatenate([qq, tt]))
        counter = int(m.debug_counters()[40])
        m.close()
        comm.close()
        q.put((rank, np.array(poses), counter))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["host", "device"])
def test_two_processes_gloo(transport):
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
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, frames, q, transport)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(2)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == 0 and res[1][2] == 0
    for f in range(N_FRAMES):
        got, w = res[0][1][f], want[f]
        assert np.linalg.norm(got[4:] - w[4:]) < 1e-6 and quat_angle(got[:4], w[:4]) < 1e-6, f
