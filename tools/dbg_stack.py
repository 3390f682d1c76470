"""Few-stream stack VoxelGrid (k_stack_part, laser_mapping.cpp:492-500) phase cycles of a
one-stream mapper over 40 frames after 120 map-building frames of the synthetic street (GPU scan
registration + odometry): debug counters 42..47 and 91, per part (K = 8 parts per (frame, map))."""
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
sizes = []
for f in range(160):
    xyz, _ = synth.frame(1, f, 2000)
    sr.input(xyz)
    c = sr.output()
    od.input(0, c[1], c[2], c[3], c[4])
    od.solve()
    q, t, _, _, skip = od.output(0)
    cn, sn = od.last_cloud(0, 0), od.last_cloud(0, 1)
    mp.input(0, cn, sn, q, t)
    if f == 120:
        mp.debug_counters(reset=True)
    if f >= 120:
        sizes.append((len(cn), len(sn)))
    mp.solve()
c = mp.debug_counters().astype(np.float64)
parts = 40 * 2 * 8
print(f"stack inputs (corner, surf) mean {np.mean(sizes, axis=0).round(0).tolist()}")
print(f"k_stack_part per part: bbox {c[42] / parts:.0f} histogram+cuts {c[91] / parts:.0f} hash {c[43] / parts:.0f} "
      f"sort+scan {c[44] / parts:.0f} members+centroids {c[45] / parts:.0f} (member lists {c[46] / parts:.0f}, "
      f"per-voxel sums {c[47] / parts:.0f})")
