"""Sharded mapper over in-process ranks (loam_comm_create_local): which frame / rank fails, for
several rank counts and LM workgroup counts (LOAM_LM_G)"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from helpers import run_sequence  # noqa: E402
from loam_amd.comm import Comm  # noqa: E402
from loam_amd.mapping import BatchMapper  # noqa: E402

seq = run_sequence(seed=11, n_frames=12)


def work(r):
    m = BatchMapper(1, comm=comms[r])
    for f, rec in enumerate(seq):
        m.input(0, rec["corner"], rec["surf"], rec["q_wodom"], rec["t_wodom"])
        try:
            m.solve()
            st = m.stats(0)
            out[r].append((f, "ok", st.lm[0].iterations, st.lm[1].iterations, st.lm[0].termination,
                           st.lm[1].termination))
        except Exception as e:  # noqa: BLE001
            out[r].append((f, "ERR", str(e)[:120]))
    m.close()


for R in [int(a) for a in sys.argv[1:]] or [3]:
    comms = Comm.local_group(R)
    out = [[] for _ in range(R)]
    th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    print("ranks", R, flush=True)
    for r in range(R):
        print("rank", r, out[r], flush=True)
    for c in comms:
        c.close()
