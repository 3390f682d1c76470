"""The concurrent-sector rule of scan registration's greedy picks (scanreg.hip sr_greedy_ring), on
the CPU: sectors picked independently, then a rerun of a sector only where the flags inherited
from the sector before hit one of its own first-5-point picks, give the reference's sequential
labels and pick order (scan_registration.cpp:352-493).  tools/sr_conc_check.py restates both
runs; here on street, quantized and column-major frames, where reruns do occur."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import sr_conc_check as C  # noqa: E402

import loam_oracle as O  # noqa: E402
from loam_amd import synth  # noqa: E402


def test_concurrent_sectors_equal_sequential():
    reruns = rings = 0
    for seed, f, flags in [(1, 0, 0), (6, 3, synth.QUANTIZE), (9, 4, synth.COLUMN_MAJOR | synth.LASER_AZ)]:
        xyz, _ = synth.frame(seed, f, 2000, flags=flags)
        ref = O.ScanRegistration()
        ref.input(xyz)
        L = ref.cloud(0)
        curv, _ = ref.curvature()
        ring = np.floor(L[:, 3]).astype(int)
        starts = np.flatnonzero(np.r_[True, ring[1:] != ring[:-1]])
        for a, b in zip(starts, np.r_[starts[1:], len(L)]):
            if b - 6 - (a + 5) >= 6:
                r, ok = C.ring_check(L, curv, a + 5, b - 6)  # asserts equality
                reruns += r
                rings += ok
    assert rings > 100 and reruns > 10
