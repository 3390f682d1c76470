"""CPU check of the exactness argument behind stdsort.h ss_depth_limit.

libstdc++'s introsort (restated here serially, as tests/cxx/stdsort_model.cpp does) is run on
the (voxel idx, point) pairs of cube-shaped clouds (sorted VoxelGrid output with a few points
appended: median-of-3 degenerates and the depth limit is reached on long segments).  At each
depth-limit segment the device keeps a (key, element) sort instead of the heap sort when no run
of equal keys inside it is longer than 2 and neither end key is a pair.  The test runs introsort
both ways and checks that every VoxelGrid centroid (float32 sums from 0 in the sorted order,
divided by the count, PCL voxel_grid.hpp) is bit-identical, and that the permutation of the
literal version equals std::sort's own (the oracle library's std_sort_perm)."""
import numpy as np
import pytest

import loam_oracle as O


def _adjust(E, first, hole, length, value):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if E[first + second][0] < E[first + second - 1][0]:
            second -= 1
        E[first + hole] = E[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        E[first + hole] = E[first + second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and E[first + parent][0] < value[0]:
        E[first + hole] = E[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    E[first + hole] = value


def _heap_sort(E, lo, hi, pops=None):
    """__make_heap + __sort_heap on E[lo, hi); pops: only the first that many pops"""
    n = hi - lo
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            _adjust(E, lo, parent, n, E[lo + parent])
            if parent == 0:
                break
            parent -= 1
    last = hi
    end = lo + 1 if pops is None else max(lo + 1, hi - pops)
    while last > end:
        last -= 1
        v = E[last]
        E[last] = E[lo]
        _adjust(E, lo, 0, last - lo, v)


def _order_free(seg):
    """ss_depth_limit's rule for VoxelGrid (free_run 2) on the segment's keys"""
    keys = sorted(k for k, _ in seg)
    if any(keys[i - 2] == keys[i] for i in range(2, len(keys))):
        return False
    return not (len(keys) >= 2 and (keys[0] == keys[1] or keys[-2] == keys[-1]))


def _introsort(pairs, relaxed):
    """libstdc++ std::sort on (key, element) pairs compared by key; relaxed: depth-limit
    segments that pass the rule are sorted by (key, element) instead of heap-sorted"""
    E = list(pairs)
    n = len(E)
    used = [0, 0]
    stack = [(0, n, 2 * (n.bit_length() - 1))] if n > 16 else []
    while stack:
        lo, hi, d = stack.pop()
        while hi - lo > 16:
            if d == 0:
                if relaxed and _order_free(E[lo:hi]):
                    E[lo:hi] = sorted(E[lo:hi])
                    used[0] += 1
                else:
                    _heap_sort(E, lo, hi)
                    used[1] += 1
                break
            d -= 1
            mid = lo + (hi - lo) // 2
            x, y, z = lo + 1, mid, hi - 1
            a, b, c = E[x][0], E[y][0], E[z][0]
            if a < b:
                m = y if b < c else (z if a < c else x)
            elif a < c:
                m = x
            elif b < c:
                m = z
            else:
                m = y
            E[lo], E[m] = E[m], E[lo]
            p = E[lo][0]
            i, j = lo + 1, hi
            while True:
                while E[i][0] < p:
                    i += 1
                j -= 1
                while p < E[j][0]:
                    j -= 1
                if not i < j:
                    break
                E[i], E[j] = E[j], E[i]
                i += 1
            stack.append((i, hi, d))
            hi = i
    # __final_insertion_sort: stable within the final segments = a stable sort by key here
    out = sorted(range(n), key=lambda t: E[t][0])  # stable: keeps E's order among equal keys
    return [E[t] for t in out], used


def _centroids(pts, order, keys):
    out = []
    i = 0
    while i < len(order):
        j = i
        s = np.zeros(4, np.float32)
        while j < len(order) and keys[order[j]] == keys[order[i]]:
            s = s + pts[order[j]]  # float32 sums from 0 in the sorted order
            j += 1
        out.append(s / np.float32(j - i))
        i = j
    return np.asarray(out, np.float32)


def _cube_cloud(n_old, n_single, n_pair, seed, leaf):
    rng = np.random.default_rng(seed)
    side = int(round(n_old ** (1 / 3) * 1.6))
    xyz = rng.uniform(0, side * leaf, (n_old * 3, 3)).astype(np.float32)
    old = O.voxel_grid(np.concatenate([xyz, rng.uniform(0, 50, (len(xyz), 1)).astype(np.float32)], 1), leaf)
    pick = rng.choice(len(old), n_single + n_pair, replace=False)
    jitter = lambda: np.float32(0.01 * leaf) * rng.uniform(-1, 1, 4).astype(np.float32)  # noqa: E731
    new = [old[i] + jitter() for i in pick[:n_single]]
    new += [old[i] + jitter() for i in pick[n_single:] for _ in range(2)]
    return np.concatenate([old, np.asarray(new, np.float32)]).astype(np.float32)


def _keys(pts, leaf):
    inv = np.float32(1.0) / np.float32(leaf)
    v = np.floor(pts[:, :3] * inv).astype(np.int64)
    mn = v.min(0)
    dv = v.max(0) - mn + 1
    v = v - mn
    return (v[:, 0] + v[:, 1] * dv[0] + v[:, 2] * dv[0] * dv[1]).astype(np.int64)


@pytest.mark.parametrize("n_old,n_single,n_pair", [(4300, 100, 3), (2000, 40, 6), (2000, 5, 0), (1500, 30, 0)])
def test_depth_limit_rule_keeps_pcl_centroids(n_old, n_single, n_pair):
    pts = _cube_cloud(n_old, n_single, n_pair, n_old + n_pair, 0.4)
    keys = _keys(pts, 0.4)
    pairs = [(int(k), i) for i, k in enumerate(keys)]
    lit, used_lit = _introsort(pairs, relaxed=False)
    rel, used = _introsort(pairs, relaxed=True)
    assert used_lit[1] > 0, "the inputs must reach the depth limit"
    assert sum(used) == used_lit[1]  # the same depth-limit segments, kept or heap-sorted
    perm = O.std_sort_perm(keys.astype(np.uint32))
    assert [e for _, e in lit] == list(perm)  # the serial restatement is std::sort itself
    a = _centroids(pts, [e for _, e in lit], keys)
    b = _centroids(pts, [e for _, e in rel], keys)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), used


# ---------------------------------------------------------------------------------------------
# The hot-pruned emulation (voxel_pcl.h vx_pcl_fixup).  A voxel with at most two
# members sums alike in any order, so only voxels of 3+ members ("hot") need std::sort's order,
# and that order is the position order of their members once the partitions (and depth-limit
# heap sorts) are done: __final_insertion_sort is stable and never moves an element out of its
# final segment.  So the device
#   * does not partition a segment holding fewer than two hot elements (no hot voxel can have two
#     members inside it, so nothing below it can reorder a hot voxel);
#   * heap-sorts a depth-limit segment literally only when two members of one hot voxel lie in it,
#     and stops once every element with a key not less than the smallest shared hot key is popped
#     (voxel_hot.h vh_pops_needed: pops go in descending key order, what is left is never read);
#   * skips the final insertion sort, and sums each hot voxel in its members' position order.
# The restatement below does that and must give std::sort's centroids bit for bit.
# ---------------------------------------------------------------------------------------------
def _partition(E, lo, hi):
    mid = lo + (hi - lo) // 2
    x, y, z = lo + 1, mid, hi - 1
    a, b, c = E[x][0], E[y][0], E[z][0]
    if a < b:
        m = y if b < c else (z if a < c else x)
    elif a < c:
        m = x
    elif b < c:
        m = z
    else:
        m = y
    E[lo], E[m] = E[m], E[lo]
    p = E[lo][0]
    i, j = lo + 1, hi
    while True:
        while E[i][0] < p:
            i += 1
        j -= 1
        while p < E[j][0]:
            j -= 1
        if not i < j:
            return i
        E[i], E[j] = E[j], E[i]
        i += 1


def _hot_pruned_positions(pairs, hot):
    """E after the pruned emulation; hot[key]: the voxel has 3+ members"""
    E = list(pairs)
    n = len(E)
    stats = dict(partitioned=0, pruned=0, heap=0, heap_skipped=0)
    stack = [(0, n, 2 * (n.bit_length() - 1))] if n > 16 else []
    while stack:
        lo, hi, d = stack.pop()
        if hi - lo <= 16:
            continue
        hk = [k for k, _ in E[lo:hi] if hot[k]]
        if len(hk) < 2:
            stats["pruned"] += 1
            continue
        if d == 0:
            if len(set(hk)) < len(hk):
                kmin = min(k for k in set(hk) if hk.count(k) > 1)
                pops = sum(1 for k, _ in E[lo:hi] if k >= kmin)
                _heap_sort(E, lo, hi, pops)
                stats["heap"] += 1
                stats["pops_saved"] = stats.get("pops_saved", 0) + (hi - lo - 1) - min(pops, hi - lo - 1)
            else:
                stats["heap_skipped"] += 1
            continue
        stats["partitioned"] += hi - lo
        cut = _partition(E, lo, hi)
        # any processing order gives std::sort's result: the smaller part first, as the device does
        parts = sorted([(lo, cut), (cut, hi)], key=lambda t: t[1] - t[0])
        stack.append((parts[1][0], parts[1][1], d - 1))
        stack.append((parts[0][0], parts[0][1], d - 1))
    return E, stats


def _hot_pruned_centroids(pts, keys):
    uniq, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
    hot = {int(k): c >= 3 for k, c in zip(uniq, cnt)}
    E, stats = _hot_pruned_positions([(int(k), i) for i, k in enumerate(keys)], hot)
    members = [[] for _ in uniq]
    for i in range(len(keys)):  # cold voxels: any order (here the input order)
        if not hot[int(keys[i])]:
            members[inv[i]].append(i)
    for k, e in E:  # hot voxels: the position order
        if hot[k]:
            members[inv[e]].append(e)
    out = []
    for mem in members:
        s = np.zeros(4, np.float32)
        for e in mem:
            s = s + pts[e]
        out.append(s / np.float32(len(mem)))
    return np.asarray(out, np.float32), stats


def _stack_cloud(n, n_vox, seed, leaf):
    """raw-feature-like input: n points in n_vox voxels, scan order (not sorted by voxel)"""
    rng = np.random.default_rng(seed)
    ctr = rng.uniform(0, 40, (n_vox, 3)).astype(np.float32)
    ctr = (np.floor(ctr / leaf) + 0.5) * leaf
    which = rng.integers(0, n_vox, n)
    which[: n // 3] = np.sort(which[: n // 3])  # partly ordered runs, like ring scans
    xyz = ctr[which] + rng.uniform(-0.45 * leaf, 0.45 * leaf, (n, 3)).astype(np.float32)
    return np.concatenate([xyz, rng.uniform(0, 50, (n, 1)).astype(np.float32)], 1).astype(np.float32)


def _triples_cloud(n_old, n_new, seed, leaf):
    """cube-shaped: sorted fixed-point content with new points, some voxels reaching 3+ members"""
    rng = np.random.default_rng(seed)
    base = _cube_cloud(n_old, 1, 0, seed, leaf)[:-1]
    pick = rng.choice(len(base), n_new, replace=True)  # repeats make 3+ member voxels
    new = base[pick] + np.float32(0.01 * leaf) * rng.uniform(-1, 1, (n_new, 4)).astype(np.float32)
    return np.concatenate([base, new.astype(np.float32)]).astype(np.float32)


@pytest.mark.parametrize("kind,n,m,seed", [("cube", 4300, 300, 1), ("cube", 2000, 120, 2), ("cube", 6000, 40, 3),
                                           ("cube", 1500, 600, 4), ("stack", 6000, 3000, 5), ("stack", 9000, 1200, 6),
                                           ("stack", 3000, 200, 7), ("stack", 800, 790, 8)])
def test_hot_pruned_rule_keeps_pcl_centroids(kind, n, m, seed):
    leaf = 0.4
    pts = _triples_cloud(n, m, seed, leaf) if kind == "cube" else _stack_cloud(n, m, seed, leaf)
    keys = _keys(pts, leaf)
    perm = O.std_sort_perm(keys.astype(np.uint32))
    ref = _centroids(pts, list(perm), keys)  # std::sort's (PCL's) centroids
    got, stats = _hot_pruned_centroids(pts, keys)
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32)), stats
    if kind == "cube":
        assert stats["heap"] + stats["heap_skipped"] > 0, "cube inputs reach the depth limit"
