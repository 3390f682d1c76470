"""Shape of libstdc++'s introsort on the exact mode's cube re-filters: for the
cubes a steady-state oracle frame re-filters, the (idx, point) sort of PCL's VoxelGrid over old
content ++ new points: partition levels, segments per level, depth-limit heap sorts, and how
many voxels hold 3+ members.

    python tools/introsort_stats.py [frames]      (CPU only: the oracle pipeline)"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
from helpers import run_sequence  # noqa: E402
from mult_stats import cube_of, downsample  # noqa: E402
from scipy.spatial.transform import Rotation as R  # noqa: E402


def introsort_shape(keys):
    """libstdc++ __introsort_loop on keys (comparisons on the key only): per level the segment
    lengths partitioned, and the heap-sort fallbacks"""
    a = list(keys)
    n = len(a)
    levels = collections.defaultdict(list)
    heaps = []
    if n <= 16:
        return levels, heaps
    stack = [(0, n, 2 * (n.bit_length() - 1), 0)]
    while stack:
        lo, hi, d, lev = stack.pop()
        while hi - lo > 16:
            if d == 0:
                heaps.append(hi - lo)
                a[lo:hi] = sorted(a[lo:hi])
                break
            d -= 1
            levels[lev].append(hi - lo)
            mid = lo + (hi - lo) // 2
            x, y, z = lo + 1, mid, hi - 1
            ea, eb, ec = a[x], a[y], a[z]
            if ea < eb:
                m = y if eb < ec else (z if ea < ec else x)
            elif ea < ec:
                m = x
            elif eb < ec:
                m = z
            else:
                m = y
            a[lo], a[m] = a[m], a[lo]
            p = a[lo]
            i, j = lo + 1, hi
            while True:
                while a[i] < p:
                    i += 1
                j -= 1
                while p < a[j]:
                    j -= 1
                if not i < j:
                    break
                a[i], a[j] = a[j], a[i]
                i += 1
            cut = i
            stack.append((cut, hi, d, lev + 1))
            hi = cut
            lev += 1
    return levels, heaps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    f = n - 1
    seq = run_sequence(7, n, snapshot_frames=(f,))
    rec = seq[f]
    q, t = rec["pose"]
    rot = R.from_quat(q)
    cen = rec["before"]["cen"]
    for key, leaf in (("corner", 0.4), ("surf", 0.8)):
        new = rot.apply(downsample(rec[key][:, :3].astype(np.float64), leaf)) + t
        per_cube = collections.defaultdict(list)
        for i, c in enumerate(map(tuple, cube_of(new, cen))):
            per_cube[c].append(new[i])
        for c, pts in sorted(per_cube.items(), key=lambda kv: -len(kv[1])):
            idx = c[0] + 21 * c[1] + 441 * c[2]
            old = rec["before"][key].get(idx)
            allp = np.asarray(pts, np.float32)
            n_old = 0 if old is None else len(old)
            if n_old:
                allp = np.concatenate([old[:, :3].astype(np.float32), allp])
            inv = np.float32(1.0 / leaf)
            mn = np.floor(allp.min(0) * inv).astype(np.int64)
            mx = np.floor(allp.max(0) * inv).astype(np.int64)
            dv = mx - mn + 1
            v = np.floor(allp * inv).astype(np.int64) - mn
            keys = (v[:, 0] + v[:, 1] * dv[0] + v[:, 2] * dv[0] * dv[1]).tolist()
            levels, heaps = introsort_shape(keys)
            _, cnt = np.unique(np.asarray(keys), return_counts=True)
            per_lev = [f"{len(levels[k])}:{max(levels[k])}" for k in sorted(levels)]
            print(f"{key} cube {idx}: {n_old} old + {len(pts)} new; levels {len(levels)} (segments:longest) "
                  f"{' '.join(per_lev)}; heap sorts {heaps}; voxels 3+ {int((cnt >= 3).sum())}")


if __name__ == "__main__":
    main()
