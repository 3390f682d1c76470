"""Phase cycles of the per-ring PCL-order VoxelGrid (k_sr_ringvox) over 20 frames."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd")]
import numpy as np  # noqa: E402

from loam_amd import synth  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

sr = ScanRegistration()
frames = [synth.frame(1, f, 2000)[0] for f in range(20)]
for xyz in frames[:3]:
    sr.input(xyz)
sr.debug_counters(reset=True)
ms = []
for xyz in frames:
    sr.input(xyz)
    ms.append(sr.ms)
c = sr.debug_counters()
rings = 64 * len(frames)
print("scanreg ms/frame", np.mean(ms))
print("per ring cycles: keys %.0f  sort levels %.0f  final %.0f  centroids %.0f" % tuple(c[:4] / rings))
