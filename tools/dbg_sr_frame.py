"""Compare the HIP ScanRegistration with the oracle on one synthetic frame (seed frame n_az):
counts of the five clouds, first differing points, curvature / label differences."""
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("vloam-noted_amd", "oracle", "tests")]
import numpy as np  # noqa: E402
import loam_oracle as O  # noqa: E402
from loam_amd import synth  # noqa: E402
from loam_amd.scanreg import ScanRegistration  # noqa: E402

seed, frame, n_az = (int(a) for a in sys.argv[1:4])
xyz, _ = synth.frame(seed, frame, n_az)
ref = O.ScanRegistration()
ref.input(xyz)
gpu = ScanRegistration()
gpu.input(xyz)
names = ("laserCloud", "sharp", "lessSharp", "flat", "lessFlat")
for w, (a, b) in enumerate(zip(gpu.output(), ref.output())):
    same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    print(names[w], a.shape, b.shape, "identical" if same else "DIFFERENT")
    if not same:
        n = min(len(a), len(b))
        d = np.flatnonzero(np.any(a[:n].view(np.uint32) != b[:n].view(np.uint32), axis=1))
        print("  first differing rows", d[:10], "of", len(d))
        for i in d[:4]:
            print("   gpu", a[i], "ref", b[i])
c, lab = gpu.curvature()
rc, rlab = ref.curvature()
dc = np.flatnonzero(c[5:-5].view(np.uint32) != rc[5:-5].view(np.uint32))
dl = np.flatnonzero(lab[5:-5] != rlab[5:-5])
print("curvature differs at", len(dc), "points", (dc[:10] + 5), "labels differ at", len(dl), (dl[:10] + 5))
for i in (dl[:6] + 5):
    print("  idx", i, "curv gpu", c[i], "ref", rc[i], "label gpu", lab[i], "ref", rlab[i], "intensity", ref.cloud(0)[i, 3])
