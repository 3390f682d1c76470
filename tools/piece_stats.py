"""How much of the exact mode's emulated sort (PCL VoxelGrid's std::sort, libstdc++ introsort) a
run-aware ("piece list") emulation would touch.  A cube re-filter sorts old content (the previous
filter's output: one point per voxel, ascending voxel index) ++ the frame's new points; the old
content moves through the Hoare partitions as slices of that ascending run (ascending or reversed),
so a partition could classify a slice by binary search and swap slices as intervals.

Per re-filtered cube of steady-state oracle frames: the elements the hot-pruned emulation partitions
(what the GPU does today) against the pieces those same segments hold (maximal position runs whose
original indices step by +1 or -1 and are old; every new element a piece of its own).

    python tools/piece_stats.py [first_frame] [frames]      (CPU only: the oracle pipeline)"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from exact_sort_stats import O, R, partition_elems, pcl_keys, run_sequence, seg_class  # noqa: E402


def pieces(a, lo, hi, n_old):
    e = (a[lo:hi] & ((1 << 20) - 1)).astype(np.int64)
    if len(e) == 0:
        return 0
    old = e < n_old
    d = np.diff(e)
    cont = old[1:] & old[:-1] & ((d == 1) | (d == -1))
    # a break wherever two neighbours are not one ascending / descending step of the old run; a
    # +1 step after a -1 step also breaks (direction change)
    br = ~cont
    dirchg = np.zeros_like(br)
    dirchg[1:] = cont[1:] & cont[:-1] & (d[1:] != d[:-1])
    return 1 + int((br | dirchg).sum())


def work(keys, hot, n_old):
    n = len(keys)
    a = np.asarray(keys, np.int64) * (1 << 20) + np.arange(n)
    hot_el = hot[np.arange(n)]
    el = pc = segs = heap = 0
    if n <= 16:
        return el, pc, segs, heap
    stack = [(0, n, 2 * (n.bit_length() - 1))]
    while stack:
        lo, hi, d = stack.pop()
        while hi - lo > 16:
            cls = seg_class(a, lo, hi, hot_el)
            if cls < 2:
                break
            if d == 0:
                if cls == 3:
                    heap += hi - lo
                a[lo:hi] = np.sort(a[lo:hi])
                break
            d -= 1
            el += hi - lo
            pc += pieces(a, lo, hi, n_old)
            segs += 1
            cut = partition_elems(a, lo, hi)
            stack.append((cut, hi, d))
            hi = cut
    return el, pc, segs, heap


def main():
    f0 = int(sys.argv[1]) if len(sys.argv) > 1 else 155
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    frames = tuple(range(f0, f0 + nf))
    seq = run_sequence(7, f0 + nf, snapshot_frames=frames)
    tot = collections.Counter()
    for f in frames:
        rec = seq[f]
        q, t = rec["pose"]
        rot = R.from_quat(q)
        cen = rec["before"]["cen"]
        for key, leaf in (("corner", 0.4), ("surf", 0.8)):
            stack = O.voxel_grid(rec[key], leaf)
            # the stack VoxelGrid itself (input: the feature cloud in scan order)
            sk = pcl_keys(rec[key][:, :3], leaf)
            u, inv, cnt = np.unique(sk, return_inverse=True, return_counts=True)
            # stacks have no old run: count pieces as key-monotone runs instead
            se, _, ss, sh = work(sk, cnt[inv] >= 3, 0)
            tot["stack_el"] += se
            tot["stack_heap"] += sh
            ks = np.asarray(sk)
            dd = np.sign(np.diff(ks))
            tot["stack_n"] += len(ks)
            tot["stack_monotone_runs"] += 1 + int((dd[1:] * dd[:-1] < 0).sum())
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
                el, pc, segs, heap = work(keys, hot, n_old)
                tot["cubes"] += 1
                tot["n"] += len(keys)
                tot["new"] += len(ids)
                tot["el"] += el
                tot["pieces"] += pc
                tot["segs"] += segs
                tot["heap"] += heap
                if len(keys) > 4000:
                    print("frame %d %s cube %d: %d old + %d new: partitioned %d elements in %d segments, %d pieces,"
                          " heap %d" % (f, key, idx, n_old, len(ids), el, segs, pc, heap))
    print(dict(tot))


if __name__ == "__main__":
    main()
