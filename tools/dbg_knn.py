"""Tile kNN phase cycles of a one-stream mapper (debug counters 50..56) over 40 frames
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
tiles = max(c[55], 1)
print(f"tiles {c[55]:.0f}, queries/tile {c[56] / tiles:.1f}, staged points/tile {c[57] / tiles:.1f}; cycles per tile: "
      f"record + queries {c[50] / tiles:.0f}, probes + cell starts {c[51] / tiles:.0f}, staging {c[52] / tiles:.0f}, "
      f"search {c[53] / tiles:.0f}, results {c[54] / tiles:.0f}")
