"""The rank form of libstdc++'s first introsort partition (voxel_hot.h vh_big_partition) on the
CPU: __move_median_to_first(first, first + 1, mid, last - 1) then __unguarded_partition, against
the same steps as a scanning loop.  The k-th left stop (key not below the pivot, ascending) swaps
with the k-th right stop (key not above it, descending) while l_k < r_k, and the cut is
min(l_{S+1}, r_S).  Keys with heavy duplication: only the order of equal keys is at stake."""
import random


def _median_to_first(a):
    n = len(a)
    x, y, z = 1, n // 2, n - 1
    k = [e[0] for e in a]
    if k[x] < k[y]:
        m = y if k[y] < k[z] else (z if k[x] < k[z] else x)
    else:
        m = x if k[x] < k[z] else (z if k[y] < k[z] else y)
    a[0], a[m] = a[m], a[0]


def _scanning(a):
    a = list(a)
    _median_to_first(a)
    p, f, last = a[0][0], 1, len(a)
    while True:
        while a[f][0] < p:
            f += 1
        last -= 1
        while p < a[last][0]:
            last -= 1
        if not f < last:
            return a, f
        a[f], a[last] = a[last], a[f]
        f += 1


def _ranked(a):
    a = list(a)
    _median_to_first(a)
    n, p = len(a), a[0][0]
    L = [i for i in range(1, n) if not a[i][0] < p]
    R = [i for i in range(n - 1, 0, -1) if not p < a[i][0]]
    S = 0
    while S < min(len(L), len(R)) and L[S] < R[S]:
        S += 1
    for j in range(S):
        a[L[j]], a[R[j]] = a[R[j]], a[L[j]]
    return a, min(L[S] if S < len(L) else n, R[S - 1] if S >= 1 else n)


def test_rank_form_equals_scanning_partition():
    rnd = random.Random(1)
    for _ in range(3000):
        n = rnd.randint(17, 400)
        nk = rnd.choice([1, 2, 3, 5, n])
        a = [(rnd.randrange(nk), i) for i in range(n)]
        assert _ranked(a) == _scanning(a)
