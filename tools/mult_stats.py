"""How many re-filtered cubes of a frame hold a voxel with 3 or more members (old content ++
inserted points)?  A voxel of 1 or 2 members sums the same in any order, so a cube without a
3-member voxel gets PCL's bits from the input-order filter (exact mode).

    python tools/mult_stats.py [frames]      (CPU only: the oracle pipeline)

New points: the frame's features downsampled with the mapper's leaves (0.4 / 0.8 m, laser_mapping.cpp:99-105) and moved to
the map with the frame's final pose; cubes by laser_mapping.cpp:747-756."""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from helpers import run_sequence  # noqa: E402
from scipy.spatial.transform import Rotation as R  # noqa: E402


def downsample(p, leaf):
    k = np.floor(p / leaf).astype(np.int64)
    _, inv = np.unique(k, axis=0, return_inverse=True)
    out = np.zeros((inv.max() + 1, 3))
    np.add.at(out, inv.ravel(), p)
    return out / np.bincount(inv.ravel())[:, None]


def cube_of(p, cen):
    c = np.floor((p + 25.0) / 50.0).astype(np.int64)
    return c + np.asarray(cen, np.int64)[None, :]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    frames = tuple(range(n - 5, n))
    seq = run_sequence(7, n, snapshot_frames=frames)
    tot = collections.Counter()
    for f in frames:
        rec = seq[f]
        q, t = rec["pose"]
        rot = R.from_quat(q)
        cen = rec["before"]["cen"]
        for key, leaf in (("corner", 0.4), ("surf", 0.8)):
            new = rot.apply(downsample(rec[key][:, :3].astype(np.float64), leaf)) + t
            nc = cube_of(new, cen)
            per_cube = collections.defaultdict(list)
            for i, c in enumerate(map(tuple, nc)):
                per_cube[c].append(new[i])
            q3 = 0
            m_hist = collections.Counter()
            for c, pts in per_cube.items():
                idx = c[0] + 21 * c[1] + 441 * c[2]
                old = rec["before"][key].get(idx)
                allp = np.asarray(pts)
                if old is not None and len(old):
                    allp = np.concatenate([old[:, :3].astype(np.float64), allp])
                k = np.floor(allp.astype(np.float32) * np.float32(1.0 / leaf)).astype(np.int64)
                _, cnt = np.unique(k, axis=0, return_counts=True)
                mx = int(cnt.max())
                m_hist[min(mx, 6)] += 1
                q3 += mx >= 3
            tot[(key, "cubes")] += len(per_cube)
            tot[(key, "3+")] += q3
            print(f"frame {f} {key}: {len(new)} new points in {len(per_cube)} cubes; "
                  f"cubes by largest voxel: {dict(sorted(m_hist.items()))}")
    for key in ("corner", "surf"):
        print(f"{key}: {tot[(key, '3+')]} of {tot[(key, 'cubes')]} cubes hold a voxel of 3+ members")


if __name__ == "__main__":
    main()
