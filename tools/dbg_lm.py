"""LM round phase cycles of a one-stream mapper (debug counters 15, 17..23) over 40 frames
after 120 map-building frames of the synthetic street (GPU scan registration + odometry)."""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd")]
import numpy as np  # noqa: E402

from loam_amd import synth  # noqa: E402
from loam_amd.mapping import BatchMapper  # noqa: E402
from loam_amd.odometry import BatchOdometry  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1)
for f in range(160):
    xyz, _ = synth.frame(1, f, 2000)
    sr.input(xyz)
    c = sr.output()
    od.input(0, c[1], c[2], c[3], c[4])
    od.solve()
    q, t, _, _, skip = od.output(0)
    mp.input(0, od.last_cloud(0, 0), od.last_cloud(0, 1), q, t)
    if f == 120:
        mp.debug_counters(reset=True)
    mp.solve()
c = mp.debug_counters().astype(np.float64)
passes = max(c[20], 1)
print(f"passes {c[20]:.0f}; per pass cycles: leader eval {c[17] / passes:.0f} (record loop {c[22] / passes:.0f}, "
      f"block reduction {c[23] / passes:.0f}), leader wait {c[18] / passes:.0f}, reduce + step {c[19] / passes:.0f} "
      f"(step alone {c[15] / passes:.0f}), member wait for x {c[21] / passes:.0f} (summed over members)")
