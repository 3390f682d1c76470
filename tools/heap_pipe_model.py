"""Model of the pipelined __sort_heap of voxel_hot.h (vh_sort_heap_pipe), checked on the CPU
against libstdc++'s sequential __sort_heap (restated: __pop_heap = hole to a leaf along the larger
children, right unless right < left, then __push_heap).

A pop of libstdc++'s __sort_heap is the same as a top-down sift of its value v from the root: the
larger child moves up while it is not less than v (ties keep descending), and v lands at the first
node whose larger child is less than it (or at a leaf).  Top-down, pops pipeline: every in-flight
pop advances one level per round, a pop starts when every older one is at least two levels deep
(a pop at depth d reads depth d + 1 and writes depth d), and when no older pop can still end at the
tail position the new pop takes its v from (an older pop whose hole is an ancestor of it or the
node itself).  A pop's output write (the old root to its tail position) waits until every older
pop has finished (older pops may still read that position as a child): a pop takes at most D + 1
rounds (D: the heap's depth), so the lane writes it in the pop's (D + 1)-th round.

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
    """the schedule of vh_sort_heap_pipe, lane by lane; returns (array, rounds, stall rounds)"""
    E = list(E)
    len_ = len(E)
    npops = len_ - 1
    D = len_.bit_length() - 1
    lanes = [dict(act=False, done=True, h=0, dep=0, n=0, L=0, age=0, v=0, top=0) for _ in range(S)]
    tail = rounds = stalls = 0
    while True:
        start = -1
        if tail < npops:
            Ln = npops - tail
            blk = any(p["act"] and not p["done"] and (p["dep"] < 2 or anc_or_eq(p["h"], Ln)) for p in lanes)
            busy = lanes[tail % S]["act"]
            if not blk and not busy:
                start = tail % S
                lanes[start].update(act=True, done=False, h=0, dep=0, n=Ln, L=Ln, age=0)
                tail += 1
            else:
                stalls += 1
        elif not any(p["act"] for p in lanes):
            break
        rounds += 1
        reads = []
        for i, p in enumerate(lanes):  # reads of the round
            st = p["act"] and not p["done"]
            c1 = 2 * p["h"] + 1
            a = E[c1] if st and c1 < p["n"] else 0
            b = E[c1 + 1] if st and c1 + 1 < p["n"] else 0
            if i == start:
                p["v"], p["top"] = E[p["L"]], E[0]
            reads.append((st, c1, a, b))
        for p, (st, c1, a, b) in zip(lanes, reads):  # writes
            if not st:
                continue
            h1, h2 = c1 < p["n"], c1 + 1 < p["n"]
            right = h2 and not key(b) < key(a)
            cv = b if right else a
            go = h1 and not key(cv) < key(p["v"])
            E[p["h"]] = cv if go else p["v"]
            if go:
                p["h"], p["dep"] = c1 + (1 if right else 0), p["dep"] + 1
            else:
                p["done"] = True
        for p in lanes:  # outputs
            if p["act"]:
                p["age"] += 1
                if p["age"] == D + 1:
                    E[p["L"]] = p["top"]
                    p["act"] = False
    return E, rounds, stalls


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rnd = random.Random(5)
    tot_pops = tot_rounds = tot_stalls = 0
    for t in range(trials):
        n = rnd.choice([2, 3, 4, 5, 17, 64, 100, 395, 512, 928, 1024, 1500])
        nk = rnd.choice([1, 2, 3, 8, max(1, n // 10), n])
        keys = [rnd.randrange(nk) for _ in range(n)]
        E = [(k << 16) | i for i, k in enumerate(keys)]
        H = make_heap(E)
        want = seq_sort_heap(H)
        got, rounds, stalls = pipe_sort_heap(H)
        assert got == want, (t, n, nk)
        tot_pops += n - 1
        tot_rounds += rounds
        tot_stalls += stalls
    print(f"{trials} heaps: pipelined order == libstdc++ __sort_heap; {tot_rounds / tot_pops:.2f} rounds per pop, "
          f"{tot_stalls / tot_pops:.3f} stall rounds per pop")


if __name__ == "__main__":
    main()
