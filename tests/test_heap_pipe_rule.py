"""The pipelined heap pops of the PCL-order sort (voxel_hot.h vh_sort_heap_pipe) on the CPU:
tools/heap_pipe_model.py restates the kernel's schedule lane by lane (two-level spacing, the
tail-position ancestor rule, outputs on slot reuse) and must give libstdc++'s __sort_heap
permutation, keys with many duplicates included (only the order of equal keys is at stake)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import heap_pipe_model as M  # noqa: E402


def test_pipelined_pops_equal_sort_heap():
    rnd = random.Random(11)
    for n in (2, 3, 4, 5, 17, 100, 192, 395, 928, 1500):
        for nk in (1, 2, 3, max(1, n // 10), n):
            keys = [rnd.randrange(nk) for _ in range(n)]
            H = M.make_heap([(k << 16) | i for i, k in enumerate(keys)])
            got, _ = M.pipe_sort_heap(H)
            assert got == M.seq_sort_heap(H), (n, nk)
