"""Long-stream fixture: BASELINE configs[3] at its stated length (10,000-frame synthetic stream).

Runs the CPU oracle chain (oracle/loam_oracle.cpp; test infrastructure) over a 10 km drive of
the synthetic street (64 x 2000 HDL-64E frames, csrc/synth.cpp): ScanRegistration ->
LaserOdometry -> LaserMapping, the mapper twice on the same features and priors:
  pcl   VoxelGrid voxels summed in PCL's order (libstdc++ sort permutation, the reference's)
  input VoxelGrid voxels summed in input order (the GPU mapper's default, exact_voxel_order 0)
Scan registration always uses PCL's order (scan_registration.cpp:497-501 on the device too).

Per frame it records what the GPU test (tests/test_gpu_long_stream.py) compares: the feature
counts, the odometry pose / correspondences / LM iterations, and for both mapper modes the pose
and every count of LaserMapping::solveMapping (stack, submap, correspondences per round, LM
iterations per round, cube-grid centre, valid cubes, the grid's cen after recentering).  At 1 m
per frame the window recentres
(laser_mapping.cpp:252-444) about every 50 frames and map coordinates reach 10^4 m, where the
insert / re-filter path (:741-808) has not been exercised before.

Three processes (the mapper modes need their own oracle instance: the VoxelGrid order is a
process-global switch of the oracle): the front (synthetic scans on a thread pool, oracle scan
registration + odometry) feeds the two mappers through bounded queues.

    python tests/golden/make_long_stream.py [--frames 10000]   # rewrites tests/golden/long_stream.npz
"""
import argparse
import multiprocessing as mp
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "vloam-noted_amd")]

SEED, N_AZ = 23, 2000
# mapper stats columns of the fixture (loam_map_stats / oracle MapStats)
MAP_COLS = ("optimized", "corner_stack", "surf_stack", "corner_map", "surf_map", "corner_num0", "corner_num1",
            "surf_num0", "surf_num1", "iters0", "iters1", "cen_i", "cen_j", "cen_k", "valid_num")


def map_row(st):
    return [st.optimized, st.corner_stack, st.surf_stack, st.corner_map, st.surf_map, st.corner_num[0],
            st.corner_num[1], st.surf_num[0], st.surf_num[1], st.lm[0].iterations, st.lm[1].iterations,
            st.center[0], st.center[1], st.center[2], st.valid_num]


def front(n_frames, queues):
    import loam_oracle as O
    from loam_amd import synth
    O.set_voxel_order(0)
    sr, od = O.ScanRegistration(), O.LaserOdometry()
    out = dict(sr_counts=[], od_q=[], od_t=[], od_corr=[], od_iters=[])
    chunk = 32
    with ThreadPoolExecutor(max_workers=3) as ex:
        nxt = ex.map(lambda f: synth.frame(SEED, f, N_AZ)[0], range(0, min(chunk, n_frames)))
        for c0 in range(0, n_frames, chunk):
            raw = list(nxt)
            c1 = c0 + chunk
            if c1 < n_frames:
                nxt = ex.map(lambda f: synth.frame(SEED, f, N_AZ)[0], range(c1, min(n_frames, c1 + chunk)))
            for xyz in raw:
                sr.input(xyz)
                clouds = sr.output()
                od.input(*clouds)
                od.solve()
                q, t, _, _, _ = od.output()
                corr, lm = od.stats()
                out["sr_counts"].append([len(c) for c in clouds])
                out["od_q"].append(q)
                out["od_t"].append(t)
                out["od_corr"].append(corr)
                out["od_iters"].append([lm[0].iterations, lm[1].iterations])
                item = (od.cloud(0), od.cloud(1), q, t)
                for qu in queues:
                    qu.put(item)
    for qu in queues:
        qu.put(None)
    return {k: np.asarray(v) for k, v in out.items()}


def mapper(order, qu, res):
    import loam_oracle as O
    O.set_voxel_order(order)
    m = O.LaserMapping()
    q_all, t_all, rows, cens = [], [], [], []
    t0 = time.time()
    while True:
        item = qu.get()
        if item is None:
            break
        corner, surf, q, t = item
        m.input(corner, surf, None, q, t)
        m.solve()
        qm, tm = m.pose()
        q_all.append(qm)
        t_all.append(tm)
        rows.append(map_row(m.stats()))
        cens.append(m.get_state()[0])  # laserCloudCenWidth / Height / Depth (moves on recentering)
        if len(rows) % 500 == 0:
            print(f"mapper order {order}: {len(rows)} frames, {time.time() - t0:.0f} s", flush=True)
    res.put((order, np.asarray(q_all), np.asarray(t_all), np.asarray(rows, np.int32), np.asarray(cens, np.int32)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--out", default=os.path.join(HERE, "long_stream.npz"))
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    qs = [ctx.Queue(maxsize=48), ctx.Queue(maxsize=48)]
    res = ctx.Queue()
    procs = [ctx.Process(target=mapper, args=(order, qs[k], res)) for k, order in enumerate((0, 1))]
    for p in procs:
        p.start()
    t0 = time.time()
    fr = front(a.frames, qs)
    got = {}
    for _ in procs:
        order, q, t, rows, cens = res.get()
        got[order] = (q, t, rows, cens)
    for p in procs:
        p.join()
    out = dict(seed=np.int64(SEED), n_az=np.int64(N_AZ), frames=np.int64(a.frames),
               map_cols=np.array(MAP_COLS), **fr)
    for order, name in ((0, "pcl"), (1, "input")):
        q, t, rows, cens = got[order]
        out[f"{name}_q"], out[f"{name}_t"], out[f"{name}_stats"], out[f"{name}_cen"] = q, t, rows, cens
    np.savez_compressed(a.out, **out)
    cen = got[0][3]
    shifts = int(np.sum(np.any(np.diff(cen, axis=0) != 0, axis=1)))
    print(f"{a.frames} frames in {time.time() - t0:.0f} s -> {a.out}; window recenterings {shifts}; "
          f"final t {got[0][1][-1]}")


if __name__ == "__main__":
    main()
