"""BASELINE configs[3] at its stated length: a 10,000-frame synthetic mapping stream, free-running
on the GPU against the oracle chain's committed per-frame record (tests/golden/long_stream.npz,
made by tests/golden/make_long_stream.py).

The whole HIP chain runs on the raw scans (ScanRegistration -> LaserOdometry -> LaserMapping,
device pointers between the stages) with two mappers fed the same features and priors:
  exact_voxel_order = 1 (PCL's VoxelGrid summation order) against the oracle in PCL's order,
  exact_voxel_order = 0 (input order, the library default) against the oracle in input order.
The PCL-order mapper solves frame by frame (loam_mapper_solve, device inputs); the input-order
mapper queues every frame behind the one in flight (loam_mapper_solve_async, host inputs): the
device prepares its stream records from the frame before, and frames the host foresees (or the
device finds) recentering or compacting run on the host-prepared path.
Every frame: the scan-registration feature counts equal, the odometry correspondences and LM
iterations equal and its pose within 1e-4, and for both mappers every solveMapping count equal
(stacks, submaps, correspondences and LM iterations per round, grid centre, valid cubes) and the
pose within 1e-4 m / 1e-4 rad.  A 10 km drive recentres the cube window
(laser_mapping.cpp:252-444) ~200 times and compacts every map arena hundreds of times; map
coordinates reach 10^4 m, where insertion and re-filtering (:741-808) run on large floats.
"""
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from helpers import quat_angle

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "long_stream.npz")
TOL = 1e-4


def _row(st):
    return [st.optimized, st.corner_stack, st.surf_stack, st.corner_map, st.surf_map, st.corner_num[0],
            st.corner_num[1], st.surf_num[0], st.surf_num[1], st.lm[0].iterations, st.lm[1].iterations,
            st.center[0], st.center[1], st.center[2], st.valid_num]


@pytest.mark.timeout(900)
def test_long_stream_10k_frames_both_orders():
    from loam_amd import synth
    from loam_amd.mapping import BatchMapper
    from loam_amd.odometry import BatchOdometry
    from loam_amd.scanreg import ScanRegistration

    G = dict(np.load(FIXTURE))  # materialised once (NpzFile decompresses on every access)
    seed, n_az, N = int(G["seed"]), int(G["n_az"]), int(G["frames"])
    assert N >= 10000
    sr, od = ScanRegistration(), BatchOdometry(1)
    mp = {"pcl": BatchMapper(1, exact_voxel_order=1), "input": BatchMapper(1, exact_voxel_order=0)}
    for m in mp.values():
        m.debug_counters(reset=True)
    bad = {k: [] for k in ("sr", "od", "pcl", "input")}
    err = {k: np.zeros((N, 2)) for k in mp}
    cen_prev, shifts = None, 0

    def check(name, m, f):
        qm, tm = m.pose(0)
        st = m.stats(0)
        e = (float(np.linalg.norm(tm - G[f"{name}_t"][f])), quat_angle(qm, G[f"{name}_q"][f]))
        err[name][f] = e
        cen = tuple(m.get_state(0)[0])
        if (_row(st) != list(G[f"{name}_stats"][f]) or cen != tuple(G[f"{name}_cen"][f])
                or e[0] >= TOL or e[1] >= TOL):
            bad[name].append(f)
        return cen
    t0 = time.time()
    chunk = 64
    workers = min(16, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=workers) as ex:
        nxt = ex.map(lambda f: synth.frame(seed, f, n_az)[0], range(0, min(chunk, N)))
        for c0 in range(0, N, chunk):
            raw = list(nxt)
            if c0 + chunk < N:
                nxt = ex.map(lambda f: synth.frame(seed, f, n_az)[0], range(c0 + chunk, min(N, c0 + 2 * chunk)))
            for k, xyz in enumerate(raw):
                f = c0 + k
                sr.input(xyz)
                if list(sr.counts()) != list(G["sr_counts"][f]):
                    bad["sr"].append(f)
                ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
                od.input_device(0, ptrs, counts)
                od.solve()
                q, t, _, _, _ = od.output(0)
                ost = od.stats(0)
                if ([ost.corner_num[0], ost.surf_num[0], ost.corner_num[1], ost.surf_num[1]] != list(G["od_corr"][f])
                        or [ost.lm[0].iterations, ost.lm[1].iterations] != list(G["od_iters"][f])
                        or np.linalg.norm(t - G["od_t"][f]) >= TOL or quat_angle(q, G["od_q"][f]) >= TOL):
                    bad["od"].append(f)
                (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
                mp["pcl"].input_device(0, pc, nc, ps, ns, q, t)
                mp["pcl"].solve()
                cen = check("pcl", mp["pcl"], f)
                shifts += cen_prev is not None and cen != cen_prev  # a recentering (laser_mapping.cpp:252-444)
                cen_prev = cen
                # host inputs: copied on the mapper's stack stream before the odometry moves on
                mi = mp["input"]
                mi.input(0, od.last_cloud(0, 0), od.last_cloud(0, 1), q, t)
                mi.solve_async()  # queued behind frame f - 1
                if f:
                    mi.wait()  # frame f - 1
                    check("input", mi, f - 1)
            if c0 % 2048 == 0:
                print(f"frame {c0}: {time.time() - t0:.0f} s", flush=True)
    mp["input"].wait()
    check("input", mp["input"], N - 1)
    compactions = {name: m.debug_counters()[48:50].tolist() for name, m in mp.items()}
    for h in (sr, od, *mp.values()):
        h.close()
    for name in mp:
        e = err[name]
        print(f"{name}: trans rms {np.sqrt(np.mean(e[:, 0] ** 2)):.3e} max {e[:, 0].max():.3e} m, rot max "
              f"{e[:, 1].max():.3e} rad; compactions corner/surf {compactions[name]}")
    print(f"{N} frames in {time.time() - t0:.0f} s, recenterings {shifts}, final x {G['pcl_t'][-1][0]:.0f} m")
    assert {k: v[:5] for k, v in bad.items() if v} == {}, {k: len(v) for k, v in bad.items()}
    assert shifts >= 100
    for name in mp:
        assert min(compactions[name]) >= 10, compactions
