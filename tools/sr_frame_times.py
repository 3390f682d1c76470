"""Per-frame device time of scan registration on the bench's sequence (seed 7, 2000 azimuths),
and for the slowest frames their slowest ring (phase counters: cycles, points, heap-sorted
elements).  python tools/sr_frame_times.py [first] [last]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd")]
import numpy as np  # noqa: E402

from loam_amd import synth  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

f0 = int(sys.argv[1]) if len(sys.argv) > 1 else 0
f1 = int(sys.argv[2]) if len(sys.argv) > 2 else 330
frames = {f: synth.frame(7, f, 2000)[0] for f in range(f0, f1)}
sr = ScanRegistration()
for f in range(f0, f0 + 3):
    sr.input(frames[f])
ms = {}
for f in range(f0, f1):
    sr.input(frames[f])
    sr.counts()
    ms[f] = sr.ms
sr.close()
v = np.array([ms[f] for f in range(f0, f1)])
print("frames %d..%d: mean %.4f ms, median %.4f, min %.4f, max %.4f" % (f0, f1 - 1, v.mean(), np.median(v), v.min(), v.max()))
for a, b in ((10, 305), (305, 325)):
    sel = [ms[f] for f in range(max(a, f0), min(b, f1))]
    if sel:
        print("frames %d..%d: mean %.4f ms" % (a, b - 1, np.mean(sel)))
os.environ["LOAM_PHASE_COUNTERS"] = "1"
sr = ScanRegistration()
worst = sorted(ms, key=ms.get)[-8:]
for f in sorted(worst + list(range(max(305, f0), min(312, f1)))):
    sr.input(frames[f])
    sr.debug_counters(reset=True)
    sr.input(frames[f])
    sr.counts()
    c = sr.debug_counters()
    s16 = int(c[16])
    print("frame %d: %.4f ms; slowest ring %d cycles, %d points, %d heap-sorted; select max %d; reruns %d"
          % (f, ms[f], s16 >> 32, s16 & 0xFFFF, (s16 >> 16) & 0xFFFF, c[15], c[21]))
