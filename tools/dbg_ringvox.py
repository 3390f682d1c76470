"""Phase cycles of the per-ring PCL-order VoxelGrid (k_sr_ringvox) over 20 frames."""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd")]
import numpy as np  # noqa: E402

from loam_amd import synth  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

device = len(sys.argv) > 1 and sys.argv[1] == "device"  # inputs resident in HBM (input_device)
if device:  # torch's HIP runtime initialises before the library's
    import torch
    torch.cuda.init()
sr = ScanRegistration()
frames = [synth.frame(1, f, 2000)[0] for f in range(20)]
if device:
    dframes = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in frames]
    feed = lambda k: sr.input_device(dframes[k].data_ptr(), len(frames[k]), 3)
else:
    feed = lambda k: sr.input(frames[k])
for k in range(3):
    feed(k)
sr.debug_counters(reset=True)
ms = []
for k in range(len(frames)):
    feed(k)
    sr.counts()  # completes the frame
    ms.append(sr.ms)
c = sr.debug_counters()
rings = 64 * len(frames)
print("scanreg ms/frame", np.mean(ms))
print("per ring: hot sort cycles %.0f, hot centroids %.0f, filters with a hot voxel %.2f" % tuple(c[:3] / rings))
print("per ring: elements heap-sorted %.1f; sort phases setup / workgroup levels / wave subtrees / positions %s"
      % (c[8] / rings, [round(float(v) / rings) for v in c[9:13]]))
print("per ring: input-order filter %.0f cycles, points %.0f (max %d, max heap-sorted %d); slowest ring %d cycles"
      % (c[4] / rings, c[5] / rings, c[6], c[7], c[3]))
s16, s18 = int(c[16]), int(c[18])
print("slowest ring: %d cycles, %d points, %d heap-sorted, %d cycles after the input-order filter"
      % (s16 >> 32, s16 & 0xFFFF, (s16 >> 16) & 0xFFFF, s18 & 0xFFFFFFFF))
print("k_sr_select per ring: sector sorts %.0f (max %d), greedy %.0f (max %d) cycles; slowest ring %d"
      % (c[13] / rings, c[19], c[14] / rings, c[20], c[15]))
