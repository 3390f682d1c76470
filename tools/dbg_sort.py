import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys, numpy as np
sys.path[:0] = ['vloam-noted_amd', 'oracle']
from loam_amd import prims
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import loam_oracle as O
for n, kv in [(17, 2), (300, 7), (40, 2), (4000, 30)]:
    keys = np.random.default_rng(n).integers(0, kv, n).astype(np.uint32)
    for w in (1, 16):
        try:
            p = prims.sort_perm(keys, w)
            print(n, kv, w, 'ok' if np.array_equal(p, O.std_sort_perm(keys)) else 'MISMATCH', flush=True)
        except Exception as e:
            print(n, kv, w, 'ERR', e, flush=True)
