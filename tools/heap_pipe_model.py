"""Model of the pipelined __sort_heap of voxel_hot.h (vh_sort_heap_pipe), lane by lane, checked
on the CPU against libstdc++'s sequential __sort_heap (restated: __pop_heap = hole to a leaf along
the larger children, right unless right < left, then __push_heap).

A pop of libstdc++'s __sort_heap is the same as a top-down sift of its value v from the root: the
larger child moves up while it is not less than v (ties keep descending), and v lands at the first
node whose larger child is less than it (or at a leaf).  Top-down, pops pipeline: every in-flight
pop advances one level per round; a start is considered every second round (round A, then round
B) and happens when every unfinished older pop is at least two levels deep (a pop at depth d reads
depth d + 1 and writes depth d) and none can still end at the tail position L the new pop takes v
from (hole an ancestor of L, or L, and E[L] not less than its v).  A pop's output (the old root to
L) is written when its slot (16, round robin) starts its next pop, or after the last rounds.

    python tools/heap_pipe_model.py [trials]"""
import random
import sys


def key(x):
    return x >> 16


def seq_sort_heap(E):
    """libstdc++ __sort_heap on a heap E (list of words, compared by key only)"""
    E = list(E)
    last = len(E)
    while last > 1:
        last -= 1
        v = E[last]
        E[last] = E[0]
        n = last
        hole, top = 0, 0
        sc = 0
        while sc < (n - 1) // 2:
            sc = 2 * (sc + 1)
            if key(E[sc]) < key(E[sc - 1]):
                sc -= 1
            E[hole] = E[sc]
            hole = sc
        if (n & 1) == 0 and sc == (n - 2) // 2:
            sc = 2 * (sc + 1)
            E[hole] = E[sc - 1]
            hole = sc - 1
        parent = (hole - 1) // 2
        while hole > top and key(E[parent]) < key(v):
            E[hole] = E[parent]
            hole = parent
            parent = (hole - 1) // 2
        E[hole] = v
    return E


def make_heap(E):
    E = list(E)
    n = len(E)
    if n < 2:
        return E
    for parent in range((n - 2) // 2, -1, -1):
        v = E[parent]
        hole, top, sc = parent, parent, parent
        while sc < (n - 1) // 2:
            sc = 2 * (sc + 1)
            if key(E[sc]) < key(E[sc - 1]):
                sc -= 1
            E[hole] = E[sc]
            hole = sc
        if (n & 1) == 0 and sc == (n - 2) // 2:
            sc = 2 * (sc + 1)
            E[hole] = E[sc - 1]
            hole = sc - 1
        p = (hole - 1) // 2
        while hole > top and key(E[p]) < key(v):
            E[hole] = E[p]
            hole = p
            p = (hole - 1) // 2
        E[hole] = v
    return E


def depth(x):
    return (x + 1).bit_length() - 1


def anc_or_eq(x, y):
    """node x is an ancestor of node y, or y itself"""
    dx, dy = depth(x), depth(y)
    return dx <= dy and ((y + 1) >> (dy - dx)) == x + 1


def pipe_sort_heap(E, S=16):
    """vh_sort_heap_pipe's schedule; returns (array, rounds)"""
    E = list(E)
    npops = len(E) - 1
    if npops < 1:
        return E, 0
    D = len(E).bit_length() - 1
    lanes = [dict(h=0, n=0, L=-1, v=0, top=0) for _ in range(S)]
    tail = rounds = 0

    def step():
        reads = []
        for p in lanes:
            c1 = 2 * p["h"] + 1
            ca = min(c1, npops - 1)
            reads.append((c1, E[ca], E[ca + 1]))
        for p, (c1, a, b) in zip(lanes, reads):
            n = p["n"]
            right = c1 + 1 < n and key(b) >= key(a)
            cv = b if right else a
            go = c1 < n and key(cv) >= key(p["v"])
            if n != 0:
                E[p["h"]] = cv if go else p["v"]
            if go:
                p["h"] = c1 + (1 if right else 0)
            else:
                p["n"] = 0

    while tail < npops:
        Ln = npops - tail
        eln = E[Ln]
        blk = any(p["n"] != 0 and (p["h"] < 3 or (anc_or_eq(p["h"], Ln) and key(eln) >= key(p["v"])))
                  for p in lanes)
        if not blk:
            p = lanes[tail % S]
            if p["L"] >= 0:
                E[p["L"]] = p["top"]
            p.update(v=E[Ln], top=E[0], h=0, n=Ln, L=Ln)
            tail += 1
        step()  # round A (the new pop moves in it too)
        step()  # round B
        rounds += 2
    for _ in range(D + 1):
        step()
        rounds += 1
    for p in lanes:
        if p["L"] >= 0:
            E[p["L"]] = p["top"]
    return E, rounds


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rnd = random.Random(5)
    tot_pops = tot_rounds = 0
    for t in range(trials):
        n = rnd.choice([2, 3, 4, 5, 17, 64, 100, 395, 512, 928, 1024, 1500])
        nk = rnd.choice([1, 2, 3, 8, max(1, n // 10), n])
        keys = [rnd.randrange(nk) for _ in range(n)]
        E = [(k << 16) | i for i, k in enumerate(keys)]
        H = make_heap(E)
        want = seq_sort_heap(H)
        got, rounds = pipe_sort_heap(H)
        assert got == want, (t, n, nk)
        tot_pops += n - 1
        tot_rounds += rounds
    print(f"{trials} heaps: pipelined order == libstdc++ __sort_heap; {tot_rounds / tot_pops:.2f} rounds per pop")


if __name__ == "__main__":
    main()
