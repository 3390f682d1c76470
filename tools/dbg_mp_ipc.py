"""Two processes on the one GPU, sharded mapper over torch.distributed gloo (host or device
callbacks), the LM through IPC peer buffers: progress of every rank to gpurun_out/mp_ipc_r*.txt
(faulthandler dumps the stacks every 30 s), to find where a run stops."""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def rank_main(rank, port, transport, frames):
    out = open(os.path.join(ROOT, "gpurun_out", f"mp_ipc_r{rank}.txt"), "w", buffering=1)
    faulthandler.dump_traceback_later(30, repeat=True, file=out)
    import torch.distributed as dist
    from loam_amd.comm import TorchDistComm, TorchDistStagedComm
    from loam_amd.mapping import BatchMapper
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    print("init", file=out)
    comm = TorchDistComm.create() if transport == "host" else TorchDistStagedComm.create()
    print("comm", file=out)
    m = BatchMapper(1, comm=comm)
    print("mapper, lm_path", m.lm_path(), file=out)
    for k, (corner, surf, qo, to) in enumerate(frames):
        m.input(0, corner, surf, qo, to)
        t0 = time.time()
        try:
            m.solve()
            print("frame", k, "ok", m.pose(0)[1], f"{time.time() - t0:.3f}s", file=out)
        except Exception as e:  # noqa: BLE001
            print("frame", k, "error", e, file=out)
    m.close()
    comm.close()
    dist.destroy_process_group()
    print("done", file=out)
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    from helpers import run_sequence
    transport = sys.argv[1] if len(sys.argv) > 1 else "device"
    os.environ.setdefault("LOAM_PEER_SPIN_LIMIT", str(1 << 20))
    seq = run_sequence(seed=11, n_frames=6)
    frames = [(r["corner"], r["surf"], r["q_wodom"], r["t_wodom"]) for r in seq]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=rank_main, args=(r, port, transport, frames)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=150)
        print("exit", p.exitcode, flush=True)
    for p in ps:
        if p.is_alive():
            p.kill()
