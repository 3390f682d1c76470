"""Re-VoxelGrid phase cycles (debug counters 0..16, 24..39) of a one-stream mapper over 40
frames after 120 map-building frames of the synthetic street (GPU scan registration +
odometry)."""
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
n = lambda k: max(c[k], 1)
print(f"items: merge {c[4]:.0f} full {c[5]:.0f} append {c[6]:.0f}; cycles per item: merge {c[0] / n(4):.0f} "
      f"full {c[1] / n(5):.0f} append {c[2] / n(6):.0f}")
print(f"merge phases per merge: bbox {c[11] / n(4):.0f} hash+passA {c[12] / n(4):.0f} sort {c[13] / n(4):.0f} "
      f"passB {c[14] / n(4):.0f}")
items = c[4] + c[5] + c[6]
print(f"cell index per item: {c[8] / max(items, 1):.0f} cycles (hash phase {c[16] / max(items, 1):.0f}), "
      f"{c[9] / max(items, 1):.0f} points")
print("by output size (<1k,2k,4k,8k,16k,32k,64k,more): items", c[24:32].astype(int).tolist())
print("  cycles per item", [int(c[32 + i] / max(c[24 + i], 1)) for i in range(8)])
print(f"stack phases per (frame, map): bbox {c[42] / 80:.0f} hash {c[43] / 80:.0f} sort+scan {c[44] / 80:.0f} "
      f"members+centroids {c[45] / 80:.0f}")
