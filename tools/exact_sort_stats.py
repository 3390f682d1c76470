"""Work of PCL's VoxelGrid sort (libstdc++ introsort) on the exact mode's cube re-filters, and
how much of it a hot-pruned emulation keeps.  A voxel with at most 2 members sums
the same in any order; only segments holding a member of a 3+ voxel ("hot") need partitioning.

For each re-filtered cube of steady-state oracle frames: elements, partition levels, elements
partitioned over all levels (full emulation) and over hot segments only (pruned), and the
depth-limit heap sorts the keep rule cannot skip (literal, one lane).

    python tools/exact_sort_stats.py [first_frame] [frames]      (CPU only: the oracle pipeline)"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import loam_oracle as O  # noqa: E402
from helpers import run_sequence  # noqa: E402
from scipy.spatial.transform import Rotation as R  # noqa: E402


def pcl_keys(p, leaf):
    p = np.asarray(p, np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    mn = p.min(0)
    mx = p.max(0)
    mnb = np.floor(mn * inv).astype(np.int64)
    mxb = np.floor(mx * inv).astype(np.int64)
    dv = mxb - mnb + 1
    v = (np.floor(p * inv) - mnb.astype(np.float32)).astype(np.int64)
    return v[:, 0] + v[:, 1] * dv[0] + v[:, 2] * dv[0] * dv[1]


def seg_class(a, lo, hi, hot_el):
    """1: a hot element inside, 2: two hot elements, 3: two members of one hot voxel"""
    e = a[lo:hi]
    h = hot_el[e & ((1 << 20) - 1)]
    nh = int(h.sum())
    if nh == 0:
        return 0
    if nh == 1:
        return 1
    k = e[h] >> 20
    return 3 if len(np.unique(k)) < nh else 2


def introsort_work(keys, hot):
    """elements partitioned: all segments / by pruning rule; depth-limit segments (size, class, keep)"""
    n = len(keys)
    a = np.asarray(keys, np.int64) * (1 << 20) + np.arange(n)  # key-major, element in low bits
    kk = lambda v: v >> 20  # noqa: E731
    hot_el = hot[np.arange(n)]
    full = levels = 0
    pruned = [0, 0, 0]
    heaps = []
    if n <= 16:
        return full, pruned, levels, heaps
    stack = [(0, n, 2 * (n.bit_length() - 1), 0)]
    while stack:
        lo, hi, d, lev = stack.pop()
        while hi - lo > 16:
            cls = seg_class(a, lo, hi, hot_el)
            if d == 0:
                ks = np.sort(kk(a[lo:hi]))
                runs = np.diff(np.flatnonzero(np.diff(np.concatenate([[-1], ks, [1 << 62]])) != 0))
                keep = runs.max() <= 2 and ks[0] != ks[1] and ks[-1] != ks[-2]
                heaps.append((hi - lo, cls, bool(keep)))
                a[lo:hi] = np.sort(a[lo:hi])  # (order irrelevant for the stats)
                break
            d -= 1
            levels = max(levels, lev + 1)
            full += hi - lo
            for r in range(3):
                if cls >= r + 1:
                    pruned[r] += hi - lo
            cut = partition_elems(a, lo, hi)
            stack.append((cut, hi, d, lev + 1))
            hi = cut
            lev += 1
    return full, pruned, levels, heaps


def partition_elems(a, lo, hi):
    k = a >> 20
    mid = lo + (hi - lo) // 2
    x, y, z = lo + 1, mid, hi - 1
    ea, eb, ec = k[x], k[y], k[z]
    if ea < eb:
        m = y if eb < ec else (z if ea < ec else x)
    elif ea < ec:
        m = x
    elif eb < ec:
        m = z
    else:
        m = y
    a[[lo, m]] = a[[m, lo]]
    k = a >> 20
    p = k[lo]
    seg = k[lo + 1:hi]
    L = np.nonzero(~(seg < p))[0] + lo + 1
    Rr = np.concatenate([[lo], np.nonzero(~(p < seg))[0] + lo + 1])[::-1]
    kq = min(len(L), len(Rr))
    ok = L[:kq] < Rr[:kq]
    S = int(np.argmin(ok)) if not ok.all() else kq
    lK = L[S] if S < len(L) else 1 << 60
    rS = Rr[S - 1] if S >= 1 else hi
    cut = int(min(lK, rS))
    if S:
        xs, ys = L[:S], Rr[:S]
        a[xs], a[ys] = a[ys].copy(), a[xs].copy()
    return cut


def main():
    f0 = int(sys.argv[1]) if len(sys.argv) > 1 else 155
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    frames = tuple(range(f0, f0 + nf))
    seq = run_sequence(7, f0 + nf, snapshot_frames=frames)
    tot = collections.Counter()
    big = []
    for f in frames:
        rec = seq[f]
        q, t = rec["pose"]
        rot = R.from_quat(q)
        cen = rec["before"]["cen"]
        for key, leaf in (("corner", 0.4), ("surf", 0.8)):
            stack = O.voxel_grid(rec[key], leaf)
            new = (rot.apply(stack[:, :3].astype(np.float64)) + t).astype(np.float32)
            c = np.floor((new.astype(np.float64) + 25.0) / 50.0).astype(np.int64) + np.asarray(cen)[None, :]
            per_cube = collections.defaultdict(list)
            for i, cc in enumerate(map(tuple, c)):
                per_cube[cc].append(i)
            for cc, ids in per_cube.items():
                if not all(0 <= cc[i] < (21, 21, 11)[i] for i in range(3)):
                    continue
                idx = cc[0] + 21 * cc[1] + 441 * cc[2]
                old = rec["before"][key].get(idx)
                pts = new[ids]
                n_old = 0 if old is None else len(old)
                if n_old:
                    pts = np.concatenate([old[:, :3].astype(np.float32), pts])
                keys = pcl_keys(pts, leaf)
                u, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
                hot = cnt[inv] >= 3
                full, pruned, levels, heaps = introsort_work(keys, hot)
                lit = [h[0] for h in heaps if h[1] == 3]
                tot["cubes"] += 1
                tot["n"] += len(keys)
                tot["full"] += full
                for r in range(3):
                    tot["pruned%d" % (r + 1)] += pruned[r]
                tot["hot_cubes"] += int(hot.any())
                tot["hot_el"] += int(hot.sum())
                tot["heap_el"] += sum(h[0] for h in heaps)
                tot["heap_lit_el"] += sum(lit)
                tot["heap_lit_dup_el"] += sum(h[0] for h in heaps if h[1] == 3)
                tot["heap_lit_dup_max"] = max(tot["heap_lit_dup_el"] and max([h[0] for h in heaps if h[1] == 3] or [0]), tot["heap_lit_dup_max"])
                if len(keys) > 4000 or sum(lit) > 500:
                    big.append((f, key, idx, n_old, len(ids), levels, full, pruned[2], int(hot.sum()), lit))
    for b in big:
        print("frame %d %s cube %d: %d old + %d new, levels %d, partitioned %d (dup-rule %d), hot elements %d,"
              " literal heap sorts %s" % b)
    print(dict(tot))


if __name__ == "__main__":
    main()
