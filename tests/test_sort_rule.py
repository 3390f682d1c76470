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


def _heap_sort(E, lo, hi):
    n = hi - lo
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            _adjust(E, lo, parent, n, E[lo + parent])
            if parent == 0:
                break
            parent -= 1
    last = hi
    while last - lo > 1:
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
