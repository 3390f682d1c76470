"""exact-mode phase counters: one mapping stream over a synthetic sequence (device-side
voxel_grid_pcl phase cycles of the stack [42..45] and cube [11..14] filters, re-VoxelGrid cycles
per cube-size bucket [24..39])"""
import os
os.environ.setdefault("LOAM_PHASE_COUNTERS", "1")  # the handles below count phase cycles
import sys, time
import numpy as np
sys.path[:0] = ['vloam-noted_amd', 'oracle', 'tests']
from loam_amd import synth
from loam_amd.scanreg import ScanRegistration
from loam_amd.odometry import BatchOdometry
from loam_amd.mapping import BatchMapper
NF = int(os.environ.get("DBG_FRAMES", "170"))
for exact in (1, 0):
    sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1, exact_voxel_order=exact)
    t_all = 0.0
    for f in range(NF):
        xyz, _ = synth.frame(11, f, 2000)
        sr.input(xyz)
        ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
        od.input_device(0, ptrs, counts); od.solve()
        q, t, _, _, _ = od.output(0)
        (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
        if f == NF - 20:
            mp.debug_counters(reset=True)
        mp.input_device(0, pc, nc, ps, ns, q, t)
        t0 = time.perf_counter(); mp.solve(); dt = time.perf_counter() - t0
        if f >= NF - 20:
            t_all += dt
    dc = [int(v) for v in mp.debug_counters()]
    st = mp.stats(0)
    cnt, cyc = dc[24:32], dc[32:40]
    per = [round(c / max(n, 1) / 1e3, 1) for n, c in zip(cnt, cyc)]
    print(f"exact={exact}: {1e3 * t_all / 20:.3f} ms/frame; stack phases (Mcycles/frame) {[round(v / 20e6, 3) for v in dc[42:46]]}; "
          f"cube phases {[round(v / 20e6, 3) for v in dc[11:15] + [dc[64]]]}; revox items merge/full/append {dc[4:7]} "
          f"filter Mcycles {[round(v / 20e6, 2) for v in dc[0:3]]} index {round(dc[8] / 20e6, 2)}; "
          f"cubes per size bucket (<1k,<2k,..) {cnt}; kcycles per cube {per}; depth-limit segments cubes {dc[66]} of {dc[67]} elements, stacks {dc[68]} of {dc[69]}; "
          f"hot fix-ups cubes: sort/centroid Mcycles {[round(v / 20e6, 3) for v in dc[50:52]]} in {dc[52]} filters, heap-sorted {dc[72]}, "
          f"sort phases setup/wg/waves/positions {[round(v / 20e6, 3) for v in dc[73:77]]}; "
          f"stacks: {[round(v / 20e6, 3) for v in dc[54:56]]} in {dc[56]}, heap-sorted {dc[77]}, phases {[round(v / 20e6, 3) for v in dc[78:82]]}; "
          f"cube wave partitions by class (<=65,129,257,513,1025) {dc[82:87]}, wave busy Mcycles {round(dc[87] / 20e6, 3)}, "
          f"longest drain Mcycles {round(dc[88] / 1e6, 3)}, heap Mcycles {round(dc[89] / 20e6, 3)}, subtrees {dc[90]}; "
          f"stacks {st.corner_stack},{st.surf_stack}", flush=True)
