"""Checks the concurrent-sector rule of scanreg.hip's sr_greedy_ring on the CPU: the six sectors of
a ring picked independently (flags written only inside the sector, suppression past its end kept
as a spill mask), then a rerun of sector j with the inherited flags only where j - 1's spill hits
one of j's own picks among its first 5 points, must give the reference's sequential labels
(scan_registration.cpp:352-493, restated in oracle/loam_oracle.cpp).  Prints how often a rerun
happens.  Sector order: (curvature, index), the same in both runs (the rule does not depend on it).

    python tools/sr_conc_check.py [frames]          (CPU only)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "vloam-noted_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import loam_oracle as O  # noqa: E402
from loam_amd import synth  # noqa: E402


def gap_ok(L, k):
    d = L[k + 1, :3] - L[k, :3]
    return float(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) <= 0.05


def greedy(L, curv, order, lo, hi, picked, label, conc):
    """one sector's two passes; picked / label arrays over the ring's cloud; returns (picks, spill, head)"""
    spill = head = 0
    picks = []

    def mark(q):
        nonlocal spill
        if not conc or lo <= q <= hi:
            picked[q] = 1
        elif q > hi:
            spill |= 1 << (q - hi - 1)

    def suppress(ind):
        for l in range(1, 6):
            if not gap_ok(L, ind + l - 1):
                break
            mark(ind + l)
        for l in range(1, 6):
            if not gap_ok(L, ind - l):
                break
            mark(ind - l)

    cnt = 0
    for ind in order[::-1]:
        if picked[ind] == 0 and curv[ind] > 0.1:
            cnt += 1
            if cnt > 20:
                break
            label[ind] = 2 if cnt <= 2 else 1
            picks.append(ind)
            if ind - lo < 5:
                head |= 1 << (ind - lo)
            picked[ind] = 1
            suppress(ind)
    cnt = 0
    for ind in order:
        if picked[ind] == 0 and curv[ind] < 0.1:
            label[ind] = -1
            picks.append(ind)
            if ind - lo < 5:
                head |= 1 << (ind - lo)
            cnt += 1
            if cnt >= 4:
                break
            picked[ind] = 1
            suppress(ind)
    return picks, spill, head


def ring_check(L, curv, s, e):
    sect = []
    for j in range(6):
        sp = s + (e - s) * j // 6
        ep = s + (e - s) * (j + 1) // 6 - 1
        idx = np.arange(sp, ep + 1)
        order = idx[np.lexsort((idx, curv[sp:ep + 1]))]
        sect.append((sp, ep, order))
    n = len(L)
    picked = np.zeros(n, np.int8)
    lab_seq = np.zeros(n, np.int8)
    seq = [greedy(L, curv, o, lo, hi, picked, lab_seq, False)[0] for lo, hi, o in sect]
    if min(hi - lo + 1 for lo, hi, _ in sect) < 8:
        return 0, 0
    picked = np.zeros(n, np.int8)
    lab = np.zeros(n, np.int8)
    res = [list(greedy(L, curv, o, lo, hi, picked, lab, True)) for lo, hi, o in sect]
    reruns = 0
    for j in range(1, 6):
        inh = res[j - 1][1]
        if not inh & res[j][2]:
            continue
        lo, hi, o = sect[j]
        picked[lo:hi + 1] = 0
        lab[lo:hi + 1] = 0
        for b in range(5):
            if inh >> b & 1:
                picked[lo + b] = 1
        res[j] = list(greedy(L, curv, o, lo, hi, picked, lab, True))
        reruns += 1
    assert np.array_equal(lab, lab_seq), "labels differ"
    assert [r[0] for r in res] == seq, "pick order differs"
    return reruns, 1


def main():
    nframes = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    tot_r = tot_rings = 0
    cases = [(seed, f, flags) for seed in (1, 2, 9) for f in range(nframes)
             for flags in (0, synth.QUANTIZE, synth.COLUMN_MAJOR | synth.LASER_AZ)]
    for seed, f, flags in cases:
        xyz, _ = synth.frame(seed, f, 2000, flags=flags)
        ref = O.ScanRegistration()
        ref.input(xyz)
        L = ref.cloud(0)
        curv, _ = ref.curvature()
        ring = np.floor(L[:, 3]).astype(int)
        starts = np.flatnonzero(np.r_[True, ring[1:] != ring[:-1]])
        ends = np.r_[starts[1:], len(L)]
        for a, b in zip(starts, ends):
            s, e = a + 5, b - 6
            if e - s < 6:
                continue
            r, ok = ring_check(L, curv, s, e)
            tot_r += r
            tot_rings += ok
    print(f"{len(cases)} frames, {tot_rings} rings with concurrent sectors: labels and picks equal the "
          f"sequential run; {tot_r} sector reruns ({tot_r / max(tot_rings, 1):.3f} per ring)")


if __name__ == "__main__":
    main()
