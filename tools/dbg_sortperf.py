"""k_sort_perm timing (std::sort emulation alone) for several sizes / key spreads"""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys, time
import numpy as np
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [os.path.join(R, 'vloam-noted_amd'), os.path.join(R, 'oracle')]
from loam_amd import prims
rng = np.random.default_rng(0)
for n, kv in [(1000, 100), (2000, 400), (8000, 1500), (30000, 3000), (30000, 30000)]:
    keys = rng.integers(0, kv, n).astype(np.uint32)
    for w in (1, 16):
        prims.sort_perm(keys, w)
        t0 = time.perf_counter()
        for _ in range(5):
            prims.sort_perm(keys, w)
        print(n, kv, w, f"{1e3 * (time.perf_counter() - t0) / 5:.3f} ms per call (incl. alloc/copies)", flush=True)
