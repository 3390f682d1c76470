"""k_frame_prep phase cycles (debug counters 58..62) of a one-stream mapper running frames queued
behind each other (loam_mapper_solve_async) over the synthetic street (GPU scan registration +
odometry)."""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # (LOAM_PHASE_COUNTERS=0 to compare without)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vloam-noted_amd")]
import numpy as np  # noqa: E402

from loam_amd import synth  # noqa: E402
from loam_amd.mapping import BatchMapper  # noqa: E402
from loam_amd.odometry import BatchOdometry  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1)
inputs = []
for f in range(80):
    xyz, _ = synth.frame(1, f, 2000)
    sr.input(xyz)
    c = sr.output()
    od.input(0, c[1], c[2], c[3], c[4])
    od.solve()
    q, t, _, _, _ = od.output(0)
    inputs.append((od.last_cloud(0, 0), od.last_cloud(0, 1), q, t))
poses = {}
for mode in ("chained", "blocking"):
    m = BatchMapper(1)
    qd = rr = 0
    poses[mode] = []
    stamps = []
    for f, (a, b, q, t) in enumerate(inputs):
        m.input(0, a, b, q, t)
        if mode.startswith("chained"):
            m.solve_async()
            if f:
                m.wait()
        else:
            m.solve()
        if f or not mode.startswith("chained"):  # (a result call with only frame 0 queued would wait for it)
            st = m.stats(0)
            qd += st.queued
            rr += st.rerun
            poses[mode].append(np.concatenate(m.pose(0)))
    m.wait()
    if mode.startswith("chained"):
        poses[mode].append(np.concatenate(m.pose(0)))
    raw = m.debug_counters()
    c = raw.astype(np.float64)
    print(f"{mode}: frames queued {qd}, run again {rr}")
    n = max(c[62], 1)
    print(f"{mode}: launches {c[62]:.0f} (device-prepared {c[63]:.0f}); cycles per launch: FrameIn load {c[58] / n:.0f}, device prep {c[59] / n:.0f}, "
          f"stack counts {c[60] / n:.0f}, submap {c[61] / n:.0f}")
    m.close()
a, b = np.array(poses["chained"]), np.array(poses["blocking"])
print("frames", len(a), len(b), "max pose difference chained vs blocking", np.abs(a - b).max() if len(a) == len(b) else "n/a")
d = np.abs(a - b).max(axis=1)
print("first differing frames", np.nonzero(d > 0)[0][:10], d[np.nonzero(d > 0)[0][:10]])
