"""CPU: the multi-rank path of bench.py with the gloo backend, world size 2 (127.0.0.1).

Each rank owns independent mapping streams (its own seed); the only cross-rank traffic is the
final reduction: LM iterations summed, wall time max over ranks (bench.py aggregate)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        iters, dt = bench.aggregate(100 * (rank + 1), 0.5 + rank, world, "cpu")
        dist.barrier()
        q.put((rank, iters, dt, bench.stream_seed(7, rank)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_aggregate_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    for rank, iters, dt, seed in res:
        assert iters == 300.0        # 100 + 200
        assert dt == 1.5             # max(0.5, 1.5)
    assert len({r[3] for r in res}) == world  # independent streams per rank


def test_aggregate_single_rank():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.aggregate(42, 0.25, 1, "cpu") == (42.0, 0.25)
