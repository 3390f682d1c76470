"""Diagnostic: repeat GPU ScanRegistration on one frame and compare counts with the oracle."""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle")]
import loam_oracle as O  # noqa: E402
from loam_amd import synth  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

seed, frame = int(sys.argv[1]), int(sys.argv[2])
xyz, _ = synth.frame(seed, frame)
ref = O.ScanRegistration()
ref.input(xyz)
rc = [len(c) for c in ref.output()]
print("oracle", rc, flush=True)
g = ScanRegistration()
for rep in range(5):
    g.input(xyz)
    gc = [len(c) for c in g.output()]
    print("gpu", rep, gc, "ok" if gc == rc else "MISMATCH", flush=True)
g2 = ScanRegistration()
g2.input(xyz)
print("fresh handle", [len(c) for c in g2.output()], flush=True)
