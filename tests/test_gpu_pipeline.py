"""Full LOAM pipeline on the GPU, zero-copy between stages, against the oracle pipeline.

GPU:    ScanRegistration -> LaserOdometry -> LaserMapping, each stage reading the previous
        stage's outputs in HBM (loam_scanreg_device_ptr -> loam_odometry_input_device ->
        loam_odometry_last_cloud -> loam_mapper_input_device), as LidarOdometryMapping calls
        them (lidar_odometry_mapping.cpp:75-176).
Oracle: the same three stages on the CPU.
Free-running over 12 frames: odometry and mapping poses within 1e-4 m / 1e-4 rad (the mapper
with exact_voxel_order = 1: free-running trajectories follow the reference bit for bit only
with PCL's VoxelGrid summation order, tests/test_gpu_steady_state.py).
"""
import numpy as np
import pytest

import loam_oracle as O
from helpers import quat_angle
from loam_amd import synth
from loam_amd.trajectory import KittiTrajectoryWriter, parse_rows
from loam_amd.mapping import BatchMapper
from loam_amd.odometry import BatchOdometry
from loam_amd.scanreg import ScanRegistration

pytestmark = pytest.mark.gpu


def test_pipeline_zero_copy():
    seed, n_frames = 17, 12
    sr_o, od_o, mp_o = O.ScanRegistration(), O.LaserOdometry(), O.LaserMapping()
    sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1, exact_voxel_order=1)
    worst = [0.0, 0.0, 0.0, 0.0]
    # LO / MO trajectory files as the driver writes them (vloam_main_node.cpp:192-198)
    lo, mo, lo_o, mo_o = (KittiTrajectoryWriter(None) for _ in range(4))
    for f in range(n_frames):
        xyz, _ = synth.frame(seed, f)
        # oracle
        sr_o.input(xyz)
        c = sr_o.output()
        od_o.input(*c)
        od_o.solve()
        qo, to, _, _, skip_o = od_o.output()
        mp_o.input(od_o.cloud(0), od_o.cloud(1), None, qo, to, skip_o)
        mp_o.solve()
        qm_o, tm_o = mp_o.pose()
        # GPU, device pointers end to end
        sr.input(xyz)
        ptrs, counts = zip(*(sr.device_ptr(k) for k in (1, 2, 3, 4)))
        od.input_device(0, ptrs, counts)
        od.solve()
        q, t, _, _, skip = od.output(0)
        (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
        mp.input_device(0, pc, nc, ps, ns, q, t, skip)
        mp.solve()
        qm, tm = mp.pose(0)
        for w, (qq, tt) in zip((lo, mo, lo_o, mo_o), ((q, t), (qm, tm), (qo, to), (qm_o, tm_o))):
            w.write(f, qq, tt)
        worst[0] = max(worst[0], float(np.linalg.norm(t - to)))
        worst[1] = max(worst[1], quat_angle(q, qo))
        worst[2] = max(worst[2], float(np.linalg.norm(tm - tm_o)))
        worst[3] = max(worst[3], quat_angle(qm, qm_o))
    assert max(worst) < 1e-4, worst
    for a, b in ((lo, lo_o), (mo, mo_o)):
        assert len(a.rows) == n_frames
        assert np.abs(parse_rows("".join(a.rows)) - parse_rows("".join(b.rows))).max() < 2e-4
    sr.close()
    od.close()
    mp.close()


def test_cxx_shim_frames(tmp_path):
    """the header-only C++ shim (include/loam_core.hpp) driving six frames through
    ScanRegistration -> LaserOdometry -> LaserMapping with host clouds between the stages, as the
    reference nodes would (tests/cxx/shim_check.cpp), against the oracle pipeline: within 1e-4,
    with the blocking solveMapping, with frames queued (solveMappingAsync / waitMapping) and with
    solveMappingPose"""
    import os
    import subprocess
    from conftest import ROOT
    from loam_amd import _core
    lib_dir = os.path.dirname(_core.LIB_PATH)
    oracle_dir = os.path.join(ROOT, "oracle", "_build")
    exe = str(tmp_path / "shim_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cxx", "shim_check.cpp"), "-o", exe, "-L", lib_dir, "-lloam_core",
                    "-lloam_synth", "-L", oracle_dir, "-lloam_oracle", f"-Wl,-rpath,{lib_dir}",
                    f"-Wl,-rpath,{oracle_dir}", "-Wl,-rpath,/opt/rocm/lib"], check=True, capture_output=True, text=True)
    r = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "blocking frame 5" in r.stdout and "queued frame 5" in r.stdout and "pose frame 5" in r.stdout


def test_pipelined_chain_matches_sequential():
    """bench.pipelined_chain (scan registration f + 1 | odometry f | mapping f - 1 on two host
    threads, inputs copied into device rings) gives every mapping pose of the sequential chain
    bit for bit"""
    import sys

    from conftest import ROOT
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench

    seed, n_frames = 23, 10
    scans = []
    for f in range(n_frames):
        xyz, _ = synth.frame(seed, f)
        scans.append(np.ascontiguousarray(np.concatenate([xyz, np.zeros((len(xyz), 1), np.float32)], axis=1)))
    sr, od, mp = ScanRegistration(), BatchOdometry(1), BatchMapper(1)
    ref = []
    for f in range(n_frames):
        sr.input(scans[f])
        ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
        od.input_device(0, ptrs, counts)
        od.solve()
        q, t, _, _, _ = od.output(0)
        (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
        mp.input_device(0, pc, nc, ps, ns, q, t)
        mp.solve()
        ref.append(mp.pose(0))
    for h in (sr, od, mp):
        h.close()
    out = bench.pipelined_chain(scans, 0, n_frames, 4)
    assert len(out["poses"]) == n_frames
    for f, ((q, t), (qr, tr)) in enumerate(zip(out["poses"], ref)):
        assert np.array_equal(q, qr) and np.array_equal(t, tr), f
