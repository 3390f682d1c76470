"""bench.py — scan-to-map LM iterations/sec on 64-ring KITTI-shaped clouds (BASELINE.json).

Workload (BASELINE.json configs[3]): LaserMapping::solveMapping (laser_mapping.cpp:212-814)
over a synthetic HDL-64E street sequence, voxel-hashed local map resident in HBM.  A step is
one full solveMapping frame — map window / recentering, stack VoxelGrid, submap hash build,
2 x (correspondences + <= 4 LM iterations), insertion and per-cube re-VoxelGrid — for each
of `--streams` independent mapping streams held by one handle (one launch sequence per step).
LM iterations are counted like Ceres' summary.iterations.size() - 1 (trust-region steps).

Inputs are produced before the timed region, on the GPU: synthetic raw scans
(vloam-noted_amd/csrc/synth.cpp) -> HIP ScanRegistration -> HIP LaserOdometry -> lessSharp /
lessFlat clouds kept in HBM + the odometry pose as the mapping prior (--prior drift: ground
truth plus a seeded random walk instead).  Stream b
replays the sequence from frame b * --stride.  --map-frames M untimed steps (always run,
independent of --warmup) build every stream's map (the 5x5x3-cube window saturates after
~150 m of travel; the default M = 300 also puts the window recentering of frames ~386 and
~436 inside the timed steps), then W untimed warmup steps, then the K timed steps: the timed
steps run at the steady-state map size of a long stream (BASELINE configs[3], 10k-frame
stream), whatever W the caller passes.

value = sum of LM iterations of all streams on all ranks / max over ranks of the timed
wall time.  roofline: the kernel family with the largest device time, algorithmic bytes /
its average launch duration (HIP events around every launch inside the library, on the
library's streams, over the timed region).  cpu_baseline (rank 0, N = 1): the CPU oracle
(single-threaded restatement of the reference: PCL KD-tree + VoxelGrid + Ceres-LM
semantics) fed stream 0's inputs: frames 0 .. M+W-1 untimed, then exactly the K frames
stream 0 processed inside the timed steps, timed.  Its poses give pose_rmse_vs_cpu (the
second half of the metric): GPU stream 0 against the oracle, both free-running from frame 0
on identical features and priors.  cpu_all_cores: one oracle replica per core (stream c on
core c), map building untimed, the K timed frames of every replica bracketed by a barrier.

Usage: python bench.py [--gpus N --steps K --warmup W --streams B]; for N > 1 launch with
torch.distributed.run, one rank per GPU (streams shard across ranks, no data-path
collective: "scaling": "weak").
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vloam-noted_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SHARD_LEG_LIMIT_S = 240.0  # watchdog of the sharded leg (its RCCL collectives are the only exchange)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5, help="untimed steps after --map-frames")
    ap.add_argument("--map-frames", type=int, default=300,
                    help="untimed map-building steps, always run before --warmup (steady-state maps)")
    ap.add_argument("--streams", type=int, default=128, help="mapping streams per GPU")
    ap.add_argument("--stride", type=int, default=1, help="frame offset between streams")
    ap.add_argument("--handles", type=int, default=2,
                    help="mapper handles, each driven by its own host thread (B / handles streams each)")
    ap.add_argument("--map-points", type=int, default=4194304,
                    help="max_map_points per stream and map (arena size; fewer compactions)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--n-az", type=int, default=2000)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="oracle replicas of the all-cores CPU figure (0: min(16, usable cores): the GPU pool "
                         "allots 16 host CPUs to one GPU, whatever the affinity mask shows)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="no per-launch HIP events")
    ap.add_argument("--prior", choices=["odometry", "drift"], default="odometry",
                    help="mapping prior: GPU LaserOdometry output (default) or ground truth + random walk")
    ap.add_argument("--no-single-stream", action="store_true",
                    help="skip the single-stream (latency view) timing")
    ap.add_argument("--no-depth", action="store_true", help="skip the VO depth-association stage")
    ap.add_argument("--exact-voxel-order", type=int, choices=[0, 1], default=0,
                    help="mapper VoxelGrids of the headline in PCL's summation order (1) or input order (0, the "
                         "library default; maps differ by summation-order ulps)")
    ap.add_argument("--shard-streams", type=int, default=32,
                    help="streams of the sharded leg (every stream split over all ranks; 0: skip the leg)")
    ap.add_argument("--pipelined", action="store_true",
                    help="(the default for the timed steps; kept for older command lines)")
    ap.add_argument("--pose-first", action="store_true",
                    help="with --blocking: each step by loam_mapper_solve_pose (returns at the poses; the map "
                         "update finishes beside the next step's stack VoxelGrid)")
    ap.add_argument("--blocking", action="store_true",
                    help="timed steps one after the other (loam_mapper_solve): step k + 1's input and stack "
                         "VoxelGrid only after step k has finished.  Default: pipelined, each handle queues step "
                         "k + 1 (its stack VoxelGrid runs beside step k) before waiting for step k "
                         "(loam_mapper_solve_async)")
    ap.add_argument("--no-exact-leg", action="store_true",
                    help="skip the second (exact_voxel_order = 1) measurement of the same workload")
    ap.add_argument("--shard", action="store_true",
                    help="sharded mapping (SURVEY.md §8e): every stream split over all N ranks, map "
                         "blocks owned per rank, RCCL all-gather of 5-NN candidates per round and "
                         "all-reduce of the normal equations per LM iteration (strong scaling)")
    return ap.parse_args()


def drift_priors(seed, n, q_gt, t_gt):
    """odometry-like prior: ground truth composed with a random-walk drift (2 cm, 0.03 deg / frame)"""
    from scipy.spatial.transform import Rotation as R
    rng = np.random.default_rng(seed + 99)
    dt = np.cumsum(rng.normal(0, 0.02, (n, 3)), axis=0)
    dr = np.cumsum(rng.normal(0, np.radians(0.03), (n, 3)), axis=0)
    q = np.empty((n, 4))
    t = np.empty((n, 3))
    for i in range(n):
        rq = R.from_rotvec(dr[i]) * R.from_quat(q_gt[i])
        q[i] = rq.as_quat()
        t[i] = t_gt[i] + dt[i]
    return q, t


def scanreg_bytes(n_in):
    """scan registration's algorithmic bytes per frame: 16 B per raw point read,
    4 B of curvature and 4 B of label written per point"""
    return 24.0 * n_in


def odometry_bytes(counts, st):
    """scan-to-scan odometry's algorithmic bytes per frame: the last clouds read
    once into the cell tables (16 B per point); per outer round the sharp + flat queries (16 B each)
    and every LM pass over the factor records (the initial evaluation plus one per iteration; 60 B
    per edge record, 44 B per plane record, as the mapper's LM family counts them)"""
    n_sharp, n_flat = int(counts[0]), int(counts[2])
    b = 16.0 * (st.n_corner_last + st.n_surf_last)
    for r in range(2):
        b += 16.0 * (n_sharp + n_flat)
        b += (st.lm[r].iterations + 1) * (60.0 * st.corner_num[r] + 44.0 * st.surf_num[r])
    return b


def make_frames(seed, n_frames, n_az, device, raw_frames=(), prior="odometry"):
    """raw scans (threads) -> HIP ScanRegistration -> HIP LaserOdometry -> features in HBM
    (torch tensors, plus host copies for the CPU legs) + the odometry pose (the mapping prior,
    laser_odometry.cpp:660-679); the raw scans of the frames in raw_frames are kept for the
    CPU stage baselines"""
    import torch
    from loam_amd import synth
    from loam_amd.odometry import BatchOdometry
    from loam_amd.scanreg import ScanRegistration

    raw_frames = set(raw_frames)
    sr = ScanRegistration(device=device)
    od = BatchOdometry(1, device=device)
    frames = []
    stage_ms = {"scan_registration": [], "odometry": [], "odometry_iters": [],
                "scan_registration_bytes": [], "odometry_bytes": []}
    chunk = 64
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        for c0 in range(0, n_frames, chunk):
            raw = list(ex.map(lambda f: synth.frame(seed, f, n_az), range(c0, min(n_frames, c0 + chunk))))
            for k, (xyz, gt) in enumerate(raw):
                sr.input(xyz)
                ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
                od.input_device(0, ptrs, counts)
                od.solve()
                q, t, _, _, _ = od.output(0)
                ost = od.stats(0)
                stage_ms["scan_registration"].append(sr.ms)
                stage_ms["odometry"].append(ost.ms)
                stage_ms["odometry_iters"].append(ost.lm[0].iterations + ost.lm[1].iterations)
                stage_ms["scan_registration_bytes"].append(scanreg_bytes(len(xyz)))
                stage_ms["odometry_bytes"].append(odometry_bytes(counts, ost))
                corner = sr.cloud(2)  # cornerPointsLessSharp -> laserCloudCornerLast
                surf = sr.cloud(4)    # surfPointsLessFlat   -> laserCloudSurfLast
                dev = f"cuda:{device}"
                frames.append(dict(corner=torch.from_numpy(corner).to(dev),
                                   surf=torch.from_numpy(surf).to(dev),
                                   # the sharp / flat queries too: the batched odometry stage
                                   sharp=torch.from_numpy(sr.cloud(1)).to(dev),
                                   flat=torch.from_numpy(sr.cloud(3)).to(dev),
                                   corner_h=corner, surf_h=surf,
                                   gt=gt, q=q, t=t, raw=xyz if c0 + k in raw_frames else None))
    sr.close()
    od.close()
    if prior == "drift":
        q_gt = np.array([f["gt"][:4] for f in frames])
        t_gt = np.array([f["gt"][4:] for f in frames])
        q, t = drift_priors(seed, n_frames, q_gt, t_gt)
        for i, f in enumerate(frames):
            f["q"], f["t"] = q[i], t[i]
    torch.cuda.synchronize(device)
    return frames, stage_ms


def step_inputs(frames, streams, stride, k, first=0):
    """batched input arrays for step k (stream b consumes frame b*stride + k); streams
    first .. first + streams - 1 of the run, numbered from 0 in their handle"""
    from loam_amd.mapping import BatchMapper
    fs = [frames[(first + b) * stride + k] for b in range(streams)]
    return BatchMapper.batch_args(np.arange(streams, dtype=np.int32),
                                  np.array([f["corner"].data_ptr() for f in fs], dtype=np.uint64),
                                  np.array([len(f["corner"]) for f in fs], dtype=np.int32),
                                  np.array([f["surf"].data_ptr() for f in fs], dtype=np.uint64),
                                  np.array([len(f["surf"]) for f in fs], dtype=np.int32),
                                  np.array([f["q"] for f in fs]), np.array([f["t"] for f in fs]))


def run_steps(mapper, plan, first, count, poses=None, pose_first=False):
    """count solveMapping steps from the precomputed per-step input arrays; with `poses`, the
    pose of the handle's stream 0 after every step is appended (a host read of the records
    the solve already copied back).  pose_first: loam_mapper_solve_pose, which returns at the
    frame's pose and finishes its map update beside the next frame"""
    iters = 0
    for k in range(first, first + count):
        mapper.input_device_batch_args(plan[k])
        if pose_first:
            mapper.solve_pose()
        else:
            mapper.solve()
        iters += mapper.total_iterations()
        if poses is not None:
            poses.append(mapper.pose(0))
    return iters


def run_steps_pipelined(mapper, plan, first, count, poses=None):
    """count solveMapping steps, each enqueued behind the one in flight (loam_mapper_solve_async
    queues it on the device, its records prepared there: include/loam_core.h) before that one is
    waited for: the same results as run_steps, frame after frame, without the host round trip
    between frames"""
    iters = 0
    mapper.input_device_batch_args(plan[first])
    mapper.solve_async()
    for k in range(first + 1, first + count + 1):
        if k < first + count:
            mapper.input_device_batch_args(plan[k])
            mapper.solve_async()  # queued behind frame k - 1
        mapper.wait()  # frame k - 1
        iters += mapper.total_iterations()  # (results: frame k - 1, the newest finished)
        if poses is not None:
            poses.append(mapper.pose(0))
    return iters


def run_handles(mappers, plans, first, count, poses=None, pipelined=False, pose_first=False):
    """run_steps (or run_steps_pipelined) on every handle, one host thread each (ctypes releases
    the GIL in the library calls): one handle's host work overlaps the others' kernels"""
    if pipelined:
        run_one = lambda h: run_steps_pipelined(mappers[h], plans[h], first, count, poses if h == 0 else None)  # noqa: E731
    else:
        run_one = lambda h: run_steps(mappers[h], plans[h], first, count, poses if h == 0 else None,  # noqa: E731
                                      pose_first=pose_first)
    if len(mappers) == 1:
        return run_one(0)
    import threading
    out = [0] * len(mappers)
    errs = []

    def work(h):
        try:
            out[h] = run_one(h)
        except Exception as e:  # surfaced after the join
            errs.append(e)

    ts = [threading.Thread(target=work, args=(h,)) for h in range(len(mappers))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    return sum(out)


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import loam_oracle as O
    return O


def cpu_baseline(frames, pre, n):
    """oracle LaserMapping fed stream 0's inputs (the GPU's features and priors, host copies):
    frames 0 .. pre-1 untimed (map building), then frames pre .. pre+n-1 -- exactly the frames
    stream 0 processed inside the GPU's timed steps -- timed by the oracle's own steady_clock
    around each solveMapping.  Returns (iterations, ms, poses of every frame)."""
    O = _oracle()
    mp = O.LaserMapping()
    iters, ms, poses = 0, 0.0, []
    for k, f in enumerate(frames[:pre + n]):
        mp.input(f["corner_h"], f["surf_h"], None, f["q"], f["t"])
        mp.solve()
        poses.append(mp.pose())
        if k < pre:
            continue
        st = mp.stats()
        iters += st.lm[0].iterations + st.lm[1].iterations
        ms += st.ms_total
    return iters, ms, poses


def cpu_stages(frames, first, n):
    """oracle ScanRegistration and LaserOdometry on the raw scans of frames first-1 ..
    first+n-1 (the first only primes the odometry's last clouds); their own timers over the
    last n frames"""
    O = _oracle()
    sr, od = O.ScanRegistration(), O.LaserOdometry()
    st = {"scan_registration": 0.0, "odometry": 0.0, "odometry_iters": 0}
    for k in range(first - 1, first + n):
        sr.input(frames[k]["raw"])
        od.input(*sr.output())
        od.solve()
        if k < first:
            continue
        st["scan_registration"] += sr.ms
        st["odometry"] += od.ms
        _, lm = od.stats()
        st["odometry_iters"] += lm[0].iterations + lm[1].iterations
    return st


def cpu_all_cores(frames, cores, stride, pre, n):
    """all-cores CPU figure: `cores` independent oracle LaserMapping replicas,
    one host thread each (ctypes releases the GIL inside the oracle), replica c on stream c's
    inputs.  Map building (pre frames) is untimed; the n timed frames of all replicas run
    between two barriers.  Returns (iterations, wall seconds)."""
    import threading
    O = _oracle()
    bar = threading.Barrier(cores + 1)
    out = [0] * cores
    errs = []

    def work(c):
        try:
            mp = O.LaserMapping()
            fs = frames[c * stride: c * stride + pre + n]
            for k, f in enumerate(fs):
                if k == pre:
                    bar.wait()
                mp.input(f["corner_h"], f["surf_h"], None, f["q"], f["t"])
                mp.solve()
                if k >= pre:
                    st = mp.stats()
                    out[c] += st.lm[0].iterations + st.lm[1].iterations
        except Exception as e:
            errs.append(e)
            bar.abort()
        finally:
            try:
                bar.wait()
            except threading.BrokenBarrierError:
                pass

    ts = [threading.Thread(target=work, args=(c,)) for c in range(cores)]
    for t in ts:
        t.start()
    bar.wait()  # every replica has built its map
    t0 = time.perf_counter()
    bar.wait()  # every replica has run its timed frames
    dt = time.perf_counter() - t0
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    return sum(out), dt


def quat_angle(q1, q2):
    """rotation angle (rad) of q1^-1 q2 (xyzw); atan2 form, exact for tiny angles"""
    q1 = np.asarray(q1, dtype=np.float64) / np.linalg.norm(q1)
    q2 = np.asarray(q2, dtype=np.float64) / np.linalg.norm(q2)
    v = q1[3] * q2[:3] - q2[3] * q1[:3] - np.cross(q1[:3], q2[:3])
    return 2.0 * np.arctan2(float(np.linalg.norm(v)), abs(float(np.dot(q1, q2))))


def pose_errors(gpu, cpu):
    """translation (m) and rotation-angle (rad) differences, RMS and max, of two pose lists"""
    dt = np.array([np.linalg.norm(np.asarray(g[1]) - np.asarray(c[1])) for g, c in zip(gpu, cpu)])
    dr = np.array([quat_angle(g[0], c[0]) for g, c in zip(gpu, cpu)])
    return {"trans_rms_m": float(np.sqrt(np.mean(dt ** 2))), "trans_max_m": float(dt.max()),
            "rot_rms_rad": float(np.sqrt(np.mean(dr ** 2))), "rot_max_rad": float(dr.max()),
            "frames": int(len(dt))}


def scanreg_batched_stage(seed, device, n_az, frames=64, reps=5):
    """BASELINE configs[1] as throughput: `frames` synthetic 64 x n_az scans resident in HBM
    through one batched ScanRegistration launch sequence (loam_scanreg_input_batch: every kernel
    runs the frames in grid rows), the device time of a launch (HIP events on the handle's
    stream), median of `reps`; bytes as the per-frame roofline (24 B per raw point)"""
    import torch
    from loam_amd import synth
    from loam_amd.scanreg import ScanRegistrationBatch
    raws = [synth.frame(seed, 1000 + f, n_az)[0] for f in range(frames)]
    dev = [torch.from_numpy(np.ascontiguousarray(r, dtype=np.float32)).to(f"cuda:{device}") for r in raws]
    ptrs = [t.data_ptr() for t in dev]
    ns = [len(r) for r in raws]
    b = ScanRegistrationBatch(frames, device=device)
    b.input_batch_device(ptrs, ns, stride=3)  # warm-up
    times = []
    for _ in range(reps):
        b.input_batch_device(ptrs, ns, stride=3)
        times.append(b.ms)
    b.close()
    ms = float(np.median(times))
    byts = scanreg_bytes(float(np.sum(ns)))
    ach = byts / (ms * 1e-3) / 1e9
    return {"frames_per_launch": frames, "launch_ms": round(ms, 4), "frames_per_s": round(frames / (ms * 1e-3), 1),
            "ms_per_frame": round(ms / frames, 5),
            "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_launch": round(byts, 1),
                         "traffic": None},
            "mode": "loam_scanreg_create_batch / loam_scanreg_input_batch: the scans in HBM, one launch sequence"}


def odometry_batched_stage(frames, device, streams=64, steps=10, warmup=3, spacing=4):
    """BASELINE configs[2] as throughput: `streams` independent LaserOdometry streams in one
    handle (BatchOdometry, every kernel of a solve covers all of them), stream b fed frames
    b*spacing, b*spacing + 1, ... of the sequence (features resident in HBM from the HIP
    ScanRegistration); the first frame of each stream only primes its last clouds, then `warmup`
    untimed and `steps` timed solves.  Device time per solve from the handle's HIP events
    (loam_odom_stats.ms: the whole launch sequence), wall time around the host calls too; bytes as
    the one-stream roofline (odometry_bytes), summed over the streams of a launch"""
    import torch
    from loam_amd.odometry import BatchOdometry
    need = (streams - 1) * spacing + warmup + steps + 1
    if need > len(frames):
        return {"error": f"needs {need} frames, {len(frames)} built"}
    od = BatchOdometry(streams, device=device)
    ms, byts, iters = [], [], 0
    t_wall = 0.0
    for k in range(warmup + steps + 1):
        for b in range(streams):
            f = frames[b * spacing + k]
            cl = (f["sharp"], f["corner"], f["flat"], f["surf"])
            od.input_device(b, [c.data_ptr() for c in cl], [len(c) for c in cl])
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        od.solve()
        dt = time.perf_counter() - t0
        if k <= warmup:
            continue
        t_wall += dt
        ms.append(od.stats(0).ms)
        for b in range(streams):
            f = frames[b * spacing + k]
            st = od.stats(b)
            iters += st.lm[0].iterations + st.lm[1].iterations
            byts.append(odometry_bytes((len(f["sharp"]), len(f["corner"]), len(f["flat"]), len(f["surf"])), st))
    od.close()
    dev_s = float(np.sum(ms)) * 1e-3
    bpl = float(np.sum(byts)) / steps
    ach = bpl / (dev_s / steps) / 1e9
    return {"streams_per_launch": streams, "steps": steps, "launch_ms": round(1e3 * dev_s / steps, 4),
            "frames_per_s": round(streams * steps / dev_s, 1), "ms_per_frame": round(1e3 * dev_s / (streams * steps), 5),
            "lm_iters_per_s": round(iters / dev_s, 1),
            "wall_frames_per_s": round(streams * steps / t_wall, 1),
            "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_launch": round(bpl, 1),
                         "traffic": None},
            "mode": f"BatchOdometry of {streams} streams (loam_odometry_solve: 2 x (k_od_corr -> k_od_lm) -> "
                    f"k_od_build over every stream per launch), stream b on frames b*{spacing} + k; device time "
                    f"from the handle's HIP events, wall time around the blocking solve beside it"}


def depth_stage(seed, device, n_frames=64, n_queries=2800, n_az=2000, with_cpu=True):
    """VO depth association (point_cloud_util.cpp:183-487): one stream
    per frame (device time of projectPointCloud + downsamplePointCloud) and n_frames streams in
    one launch sequence (wall time, clouds resident in HBM), plus queryDepth of n_queries image
    points per frame (the reference queries ~1400 matches x 2 clouds, visual_odometry.cpp:371-372);
    the oracle's own timers on the same frames as the CPU baseline."""
    import torch
    from loam_amd import synth
    from loam_amd.depth import KITTI_CAM_T_VELO, KITTI_P_RECT0, KITTI_RECT0_T_CAM, BatchDepth
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        clouds = list(ex.map(lambda f: synth.frame(seed + 77, f, n_az)[0], range(n_frames)))
    rng = np.random.default_rng(seed)
    qs = [np.stack([rng.uniform(0, 1242, n_queries), rng.uniform(0, 375, n_queries)], 1).astype(np.float32)
          for _ in range(n_frames)]
    one = BatchDepth(1, device=device)
    ms1, qms1, pts, front, dnsp = [], [], 0, 0, 0
    for f in range(n_frames):
        one.input(0, clouds[f])
        one.process()
        ms1.append(one.ms)
        t0 = time.perf_counter()
        one.query(0, qs[f])
        qms1.append(1e3 * (time.perf_counter() - t0))
        nf, nd = one.counts(0)
        pts, front, dnsp = pts + len(clouds[f]), front + nf, dnsp + nd
    one.close()
    many = BatchDepth(n_frames, device=device)
    dev = [torch.from_numpy(c).to(f"cuda:{device}") for c in clouds]
    dq = torch.from_numpy(np.concatenate(qs)).to(f"cuda:{device}")
    dqs = torch.repeat_interleave(torch.arange(n_frames, dtype=torch.int32), n_queries).to(f"cuda:{device}")
    dd = torch.empty(n_frames * n_queries, dtype=torch.float32, device=f"cuda:{device}")
    torch.cuda.synchronize(device)
    reps, t_all = 10, 0.0
    for r in range(reps + 2):
        t0 = time.perf_counter()
        for f in range(n_frames):
            many.input_device(f, dev[f].data_ptr(), len(clouds[f]), 3)
        many.process()
        many.query_device(n_frames * n_queries, dqs.data_ptr(), dq.data_ptr(), dd.data_ptr())
        if r >= 2:
            t_all += time.perf_counter() - t0
    many.close()
    g1 = float(np.mean(ms1[4:]))
    alg = (12.0 * pts + 12.0 * front + 12.0 * dnsp) / n_frames  # points in, point_cloud_2d, dnsp out
    e = {"gpu_ms_per_frame": round(g1, 4), "gpu_query_ms_per_frame": round(float(np.mean(qms1[4:])), 4),
         "queries_per_frame": n_queries,
         "batched_frames_per_s": round(n_frames * reps / t_all, 1),
         "batched": f"{n_frames} streams per launch sequence + {n_frames * n_queries} queries, wall time",
         "algorithmic_bytes_per_frame": round(alg, 1),
         "achieved_gbs_one_stream": round(alg / (g1 * 1e-3) / 1e9, 2),
         "points_per_frame": pts // n_frames, "front_per_frame": front // n_frames, "dnsp_per_frame": dnsp // n_frames}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import loam_oracle as O
        u = O.PointCloudUtil(KITTI_CAM_T_VELO, KITTI_RECT0_T_CAM, KITTI_P_RECT0)
        cms, cq = [], []
        for f in range(min(n_frames, 32)):
            u.process(clouds[f])
            cms.append(u.ms)
            u.query(qs[f])
            cq.append(u.query_ms)
        c = float(np.mean(cms)) + float(np.mean(cq))
        e.update(cpu_ms_per_frame=round(float(np.mean(cms)), 4), cpu_query_ms_per_frame=round(float(np.mean(cq)), 4),
                 cpu_cores=1, cpu_kind="port",
                 speedup_one_stream=round(c / (g1 + e["gpu_query_ms_per_frame"]), 2),
                 speedup_batched=round((n_frames * reps / t_all) * c * 1e-3, 2))
    return e


def vo_stage(seed, device, n_problems=256, with_cpu=True):
    """VO pose solve (VisualOdometry::solveNlsAll, visual_odometry.cpp:304-509; SURVEY.md §8f
    rank 4): synthetic frame pairs of ~1400 matches (the reference's count, :339), 60% with a
    LiDAR depth (CostFunctor32) and 40% without (CostFunctor22), HuberLoss, max 100 iterations.
    One problem alone and n_problems in one launch (wall time incl. the host copies); the oracle
    (Jet autodiff + Ceres TR-LM restatement) on the same problems as the CPU baseline."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from vo_problems import make_problem
    from loam_amd import vo
    rng = np.random.default_rng(seed + 5)
    probs = [make_problem(rng, n32=840, n22=560, w=rng.normal(0, 0.02, 3), t=(0.02, -0.01, -1.0))[0]
             for _ in range(n_problems)]
    vo.solve(probs[:2])  # warm the kernel
    t0 = time.perf_counter()
    for k in range(16):
        _, st1 = vo.solve([probs[k]])
    one = (time.perf_counter() - t0) / 16
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        _, st = vo.solve(probs)
    dt = (time.perf_counter() - t0) / reps
    iters = sum(x.iterations for x in st)
    e = {"gpu_ms_one_problem": round(1e3 * one, 4), "batched_problems": n_problems,
         "batched_ms": round(1e3 * dt, 4), "batched_problems_per_s": round(n_problems / dt, 1),
         "batched_lm_iters_per_s": round(iters / dt, 1), "mean_iterations": round(iters / n_problems, 2),
         "residual_blocks_per_problem": 1400}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import loam_oracle as O
        n = min(32, n_problems)
        ci = 0
        t0 = time.perf_counter()
        for F in probs[:n]:
            _, ost = O.vo_solve(F, np.zeros(6), 100)
            ci += ost.iterations
        cdt = time.perf_counter() - t0
        e.update(cpu_ms_per_problem=round(1e3 * cdt / n, 4), cpu_lm_iters_per_s=round(ci / cdt, 1), cpu_cores=1,
                 cpu_kind="port", speedup_batched=round((n_problems / dt) / (n / cdt), 2))
    return e


def pipeline_stage(seed, device, n_frames=160, timed=80, n_az=2000):
    """the whole LOAM chain on one stream, frame after frame (scanRegistrationIO ->
    laserOdometryIO -> laserMappingIO, lidar_odometry_mapping.cpp:40-176): raw scan in host
    memory -> features -> odometry -> mapping, all device-resident between stages.  'sequential'
    copies each scan from pageable memory when its frame starts; 'overlapped' queues the next
    scan's copy + scan registration (pinned ingest buffer, loam_scanreg_input_async) before the
    current frame's mapping solve.  Wall time over the last `timed` frames."""
    from loam_amd import synth
    from loam_amd.mapping import BatchMapper
    from loam_amd.odometry import BatchOdometry
    from loam_amd.scanreg import ScanRegistration
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        scans = list(ex.map(lambda f: synth.frame(seed + 31, f, n_az)[0], range(n_frames)))
    # pcl::PointXYZ layout (x, y, z, pad): 16 B per point like the reference's input cloud
    scans = [np.ascontiguousarray(np.concatenate([c, np.zeros((len(c), 1), np.float32)], axis=1)) for c in scans]
    out = {}
    poses = {"sequential": [], "overlapped": []}
    for mode in ("sequential", "overlapped"):
        sr, od, mp = ScanRegistration(device=device), BatchOdometry(1, device=device), BatchMapper(1, device=device)
        t0 = None
        if mode == "overlapped":
            sr.input_async(scans[0])
        for f in range(n_frames):
            if f == n_frames - timed:
                t0 = time.perf_counter()
            if mode == "sequential":
                sr.input(scans[f])
            else:
                sr.wait()
            ptrs, counts = zip(*(sr.device_ptr(w) for w in (1, 2, 3, 4)))
            od.input_device(0, ptrs, counts)
            od.solve()
            q, t, _, _, _ = od.output(0)
            (pc, nc), (ps, ns) = od.last_cloud_device(0, 0), od.last_cloud_device(0, 1)
            mp.input_device(0, pc, nc, ps, ns, q, t)
            if mode == "overlapped" and f + 1 < n_frames:
                sr.input_async(scans[f + 1])
            mp.solve()
            poses[mode].append(mp.pose(0))
        dt = time.perf_counter() - t0
        out[mode] = {"ms_per_frame": round(1e3 * dt / timed, 4), "frames_per_s": round(timed / dt, 1)}
        for h in (sr, od, mp):
            h.close()
    pl = pipelined_chain(scans, device, n_frames, timed)
    same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
               for a, b in zip(pl.pop("poses"), poses["sequential"]))
    out["pipelined"] = {**pl, "poses_identical_to_sequential": bool(same)}
    out["frames"] = f"{timed} timed after {n_frames - timed}, {n_az} azimuths x 64 rings, one stream"
    return out


def pipelined_chain(scans, device, n_frames, timed):
    """The same chain as a three-stage frame pipeline, the way the reference's ROS nodes run
    (scanRegistration / laserOdometry / laserMapping as concurrent nodes): frame f + 1's scan
    registration (queued asynchronously) and frame f's odometry on one host thread, frame
    f - 1's mapping solve on another; the three handles' HIP streams overlap on the GPU.  Each
    stage's input is copied (device to device, on a non-blocking stream) out of the producing
    handle's buffers, which its next frame rewrites, into a two-deep ring.  Every frame's
    inputs and results are those of the sequential chain; only the order in time changes.
    Returns ms per frame over the last `timed` frames and the mapping poses (checked against
    the sequential chain by the caller and by tests/test_gpu_pipeline.py)."""
    import ctypes

    from loam_amd.mapping import BatchMapper
    from loam_amd.odometry import BatchOdometry
    from loam_amd.scanreg import ScanRegistration
    hip = ctypes.CDLL("libamdhip64.so")  # ring buffers and copies straight through HIP (no torch)
    vp = ctypes.c_void_p
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipFree.argtypes = [vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipStreamDestroy.argtypes = [vp]
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    cap = 1 << 19  # points per ring slot and cloud
    assert hip.hipSetDevice(device) == 0
    base, cs = vp(), vp()
    assert hip.hipMalloc(ctypes.byref(base), 12 * cap * 16) == 0  # 2 slots x (4 feature + 2 last clouds)
    # a high-priority stream for the ring copies: HIP maps streams onto the process's few
    # hardware queues (GPU_MAX_HW_QUEUES = 4) in creation order, and a copy stream sharing the
    # mapper's queue waits behind its kernels (measured: 0.95-1.03 ms per frame against 0.70);
    # a high-priority stream gets a queue of its own
    hip.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(vp), ctypes.c_uint, ctypes.c_int]
    assert hip.hipStreamCreateWithPriority(ctypes.byref(cs), 1, -1) == 0  # non-blocking, high priority

    def slot(k, w):  # ring slot k, cloud w (0-3 features, 4-5 odometry last clouds)
        return base.value + ((k * 6 + w) * cap) * 16

    sr, od, mp = ScanRegistration(device=device), BatchOdometry(1, device=device), BatchMapper(1, device=device)

    def stash(dst, src):  # device-to-device copy of one cloud into a ring slot
        p, n = src
        assert n <= cap, n
        if n:
            rc = hip.hipMemcpyAsync(dst, p, 16 * n, 3, cs)
            assert rc == 0, rc
        return dst, n

    def front(f):  # odometry of frame f; scan registration of f + 1 queued beside it
        sr.wait()
        feats = [stash(slot(f % 2, w - 1), sr.device_ptr(w)) for w in (1, 2, 3, 4)]
        assert hip.hipStreamSynchronize(cs) == 0
        if f + 1 < n_frames:
            sr.input_async(scans[f + 1])
        ptrs, counts = zip(*feats)
        od.input_device(0, ptrs, counts)
        od.solve()
        q, t, _, _, _ = od.output(0)
        clouds = [stash(slot(f % 2, 4 + w), od.last_cloud_device(0, w)) for w in (0, 1)]
        assert hip.hipStreamSynchronize(cs) == 0
        return clouds, q, t

    def back(job):  # mapping of the frame front() returned
        (pc, nc), (ps, ns) = job[0]
        mp.input_device(0, pc, nc, ps, ns, job[1], job[2])
        mp.solve()
        return mp.pose(0)

    poses = []
    sr.input_async(scans[0])
    with ThreadPoolExecutor(max_workers=1) as ex:
        prev = front(0)
        t0 = None
        for f in range(1, n_frames):  # the last `timed` of these iterations are timed
            if f == n_frames - timed:
                t0 = time.perf_counter()
            fut = ex.submit(back, prev)
            prev = front(f)
            poses.append(fut.result())
        dt = time.perf_counter() - t0
        poses.append(back(prev))
    for h in (sr, od, mp):
        h.close()
    hip.hipStreamDestroy(cs)
    hip.hipFree(base)
    return {"ms_per_frame": round(1e3 * dt / timed, 4), "frames_per_s": round(timed / dt, 1),
            "poses": poses}


def _pmc_file():
    """the newest committed PMC traffic summary (tools/pmc_traffic.py -> profiles/rN_pmc_traffic.json)"""
    for r in (6, 5, 4, 3, 2):
        path = os.path.join(ROOT, "profiles", f"r{r}_pmc_traffic.json")
        if os.path.exists(path):
            return path
    return None


PMC_TRAFFIC = _pmc_file()


def pmc_traffic(family):
    """HBM bytes per launch of a kernel family measured by the rocprofv3 PMC passes of this
    bench configuration (tools/pmc_traffic.py), or None"""
    try:
        return json.load(open(PMC_TRAFFIC))["families"][family]["bytes_per_launch"]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def family_rooflines(kt, with_traffic):
    """every kernel family of the mapper step against the HBM roofline: algorithmic bytes per
    launch (counted by the library) / mean launch time (HIP events on the
    library's streams over the timed steps), and the PMC-measured memory-side bytes per launch
    of the same family with their ratio to the algorithmic bytes (wasted traffic when > 1)"""
    out = {}
    for name, v in kt.items():
        if v["ms"] <= 0 or v["launches"] <= 0:
            continue
        alg = v["bytes"] / v["launches"]
        us = 1e3 * v["ms"] / v["launches"]
        ach = alg / (us * 1e-6) / 1e9
        tr = pmc_traffic(name) if with_traffic else None
        out[name] = {"algorithmic_bytes_per_launch": round(alg, 1), "avg_launch_us": round(us, 3),
                     "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 5), "launches": v["launches"],
                     "traffic": round(tr, 1) if tr is not None else None,
                     "traffic_over_algorithmic": round(tr / alg, 3) if tr is not None and alg > 0 else None}
    return out


def aggregate(iters, dt, world, device):
    """whole-job totals: LM iterations summed over ranks, wall time = max over ranks"""
    if world <= 1:
        return float(iters), float(dt)
    import torch
    import torch.distributed as dist
    it_t = torch.tensor([float(iters)], dtype=torch.float64, device=device)
    dt_t = torch.tensor([float(dt)], dtype=torch.float64, device=device)
    dist.all_reduce(it_t, op=dist.ReduceOp.SUM)
    dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    return float(it_t.item()), float(dt_t.item())


def stream_seed(seed, rank):
    """each rank owns its own independent streams (weak scaling, no data-path collective)"""
    return seed + 1000 * rank


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)

    from loam_amd.mapping import BatchMapper

    B, K, W, M = args.streams, args.steps, args.warmup, args.map_frames
    pre = M + W  # untimed steps: map building, then warmup
    n_frames = (B - 1) * args.stride + pre + K
    with_cpu = not args.no_cpu and world == 1 and rank == 0
    cores = args.cpu_cores or min(16, len(os.sched_getaffinity(0)))
    cores = min(cores, B)
    # sharded: every rank runs the same streams (identical inputs, one share of each map)
    frames, stage_ms = make_frames(stream_seed(args.seed, 0 if args.shard else rank), n_frames, args.n_az, local,
                                   raw_frames=range(pre - 1, pre + K) if with_cpu else (), prior=args.prior)
    H = 1 if args.shard else max(1, args.handles)
    if B % H:
        raise SystemExit("--streams must be divisible by --handles")
    Bh = B // H
    comm = None
    if args.shard:
        from loam_amd.comm import Comm
        uid = [Comm.rccl_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        # RCCL prints its banner on stdout at init: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            comm = Comm.rccl(rank, world, uid[0], local)
        finally:
            os.dup2(saved, 1)
            os.close(saved)

    def timed_run(exact):
        """map building (untimed), then the K timed steps; returns (iterations, seconds, kernel
        family totals, stream 0's pose after every step)"""
        if H > 1:
            # persistent LM grids sized so that every handle's fits at once: G <= CUs / all streams
            # (speed: 2 beat 4 workgroups per stream; correctness needs no residency, lm.h)
            cus = torch.cuda.get_device_properties(local).multi_processor_count
            os.environ["LOAM_LM_G"] = os.environ.get("BENCH_LM_G") or str(max(1, cus // B))
        mappers = [BatchMapper(Bh, device=local, max_map_points=args.map_points, comm=comm,
                               exact_voxel_order=exact) for _ in range(H)]
        os.environ.pop("LOAM_LM_G", None) if H > 1 else None  # read at create; not for later handles
        poses = []  # stream 0 after every step (free-running trajectory vs the oracle's)
        run_handles(mappers, plans, 0, pre, poses)
        for m in mappers:
            if not args.no_prof:
                m.set_profiling(True)
            m.reset_kernel_times()
            if os.environ.get("BENCH_DEBUG_COUNTERS"):
                m.debug_counters(reset=True)  # the timed steps only
        barrier()
        t0 = time.perf_counter()
        it = run_handles(mappers, plans, pre, K, poses, pipelined=not args.blocking, pose_first=args.pose_first)
        barrier()
        secs = time.perf_counter() - t0
        fam = {}
        for m in mappers:
            for f, v in m.kernel_times().items():
                acc = fam.setdefault(f, {"ms": 0.0, "bytes": 0.0, "launches": 0})
                for key in acc:
                    acc[key] += v[key]
            m.set_profiling(False)
        if os.environ.get("BENCH_DEBUG_COUNTERS"):
            print(json.dumps({"debug_counters": [int(v) for v in mappers[0].debug_counters()]}), file=sys.stderr,
                  flush=True)
        for m in mappers:
            m.close()
        return it, secs, fam, poses

    def barrier():
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()

    plans = [[step_inputs(frames, Bh, args.stride, k, first=h * Bh) for k in range(pre + K)] for h in range(H)]
    iters, dt, kt, poses0 = timed_run(args.exact_voxel_order)
    iters_all, dt_max = aggregate(iters, dt, world, f"cuda:{local}")
    if args.shard:  # every rank counted the same iterations of the same streams
        iters_all = iters_all / world

    exact_leg = None
    if not args.no_exact_leg and not args.shard and not args.exact_voxel_order:
        ei, edt, ekt, eposes = timed_run(1)
        ei_all, edt_max = aggregate(ei, edt, world, f"cuda:{local}")
        exact_leg = {"value": ei_all / edt_max, "ms_per_step": 1e3 * edt_max / K, "poses": eposes,
                     "kernel_ms_per_step": {k: round(v["ms"] / K, 4) for k, v in ekt.items()}}
        if ekt:  # its own roofline: the family with the largest device time in this mode
            edom = max(ekt, key=lambda k: ekt[k]["ms"])
            ed = ekt[edom]
            each = ed["bytes"] / (ed["ms"] * 1e-3) / 1e9 if ed["ms"] > 0 else 0.0
            exact_leg["roofline"] = {"bound": "hbm", "kernel": edom, "achieved": round(each, 2),
                                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(each / HBM_PEAK_GBS, 5),
                                     "traffic": None, "launches": ed["launches"],
                                     "avg_launch_us": round(1e3 * ed["ms"] / max(1, ed["launches"]), 3),
                                     "algorithmic_bytes_per_launch": round(ed["bytes"] / max(1, ed["launches"]), 1),
                                     "families": family_rooflines(ekt, False)}

    # the north-star multi-GPU design beside the replica headline: Bs streams, each
    # split over all ranks (block-owned map shards, RCCL all-gather of the 5-NN candidates per
    # round, all-reduce of the normal equations per LM iteration): strong scaling of a fixed load

    def run_shard_leg():
        """the sharded leg (every rank in it together); returns its JSON object"""
        Bs = args.shard_streams
        n_s = (Bs - 1) * args.stride + pre + K
        if world == 1 and n_s <= len(frames):
            sframes = frames
        else:  # identical inputs on every rank
            sframes, _ = make_frames(stream_seed(args.seed, 0), n_s, args.n_az, local, prior=args.prior)
        from loam_amd.comm import Comm
        uid = [Comm.rccl_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)  # RCCL's banner stays off the JSON line
        try:
            scomm = Comm.rccl(rank, world, uid[0], local)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        splan = [step_inputs(sframes, Bs, args.stride, k) for k in range(pre + K)]

        def sharded_run(two_kernel):
            """map building untimed, then K timed steps of the sharded handle.  Default: the LM
            schedule the library picks (one persistent round per outer round; across processes
            the per-iteration sums meet in IPC-mapped peer buffers, loam_mapper_lm_path 3), its
            cross-rank wait bounded to ~1 s (LOAM_PEER_SPIN_LIMIT) so that a transport that never
            delivers ends in LOAM_ERR_SYNC, counted, not in a hang.  two_kernel: the LM forced to
            eval -> all-reduce -> step launches per pass (LOAM_LM_PERSISTENT=0, read at create).
            Every rank solves every frame whatever an earlier one returned (the collectives stay
            matched); the failures are summed over the ranks"""
            env = {"LOAM_LM_PERSISTENT": "0"} if two_kernel else {"LOAM_PEER_SPIN_LIMIT": str(1 << 20)}
            saved_env = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                sm = BatchMapper(Bs, device=local, max_map_points=args.map_points, comm=scomm)
            finally:
                for k, v in saved_env.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            path = sm.lm_path()
            errs = {"n": 0, "last": None}

            def steps(first, count):
                it = 0
                for k in range(first, first + count):
                    sm.input_device_batch_args(splan[k])
                    try:
                        sm.solve()
                        it += sm.total_iterations()
                    except Exception as e:  # noqa: BLE001 - counted, reported in the line
                        errs["n"] += 1
                        errs["last"] = repr(e)[:300]
                return it

            steps(0, pre)
            barrier()
            t0 = time.perf_counter()
            it = steps(pre, K)
            barrier()
            dt = time.perf_counter() - t0
            sm.close()
            nerr = errs["n"]
            if world > 1:
                t = torch.tensor([nerr], dtype=torch.int64, device=f"cuda:{local}")
                dist.all_reduce(t)
                nerr = int(t.item())
            return it, dt, {"lm_path": path, "failed_solves": nerr, "last_error": errs["last"]}

        sit, sdt, sinfo = sharded_run(False)
        # the per-iteration cost a multi-rank RCCL group pays without the peer buffers (10 eval /
        # all-reduce / step launch triples per frame), measured here at this world size (at one
        # rank the all-reduce is RCCL's one-rank identity on the stream)
        tit, tdt, tinfo = sharded_run(True)
        scomm.close()
        sit_all, sdt_max = aggregate(sit, sdt, world, f"cuda:{local}")
        tit_all, tdt_max = aggregate(tit, tdt, world, f"cuda:{local}")
        # the same streams and frames through an unsharded handle on this GPU (the reference
        # point of the sharding overhead at one rank)
        um = BatchMapper(Bs, device=local, max_map_points=args.map_points)
        run_steps(um, splan, 0, pre)
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        uit = run_steps(um, splan, pre, K)
        torch.cuda.synchronize(local)
        udt = time.perf_counter() - t0
        um.close()
        thread_ranks = thread_rank_overhead(splan, pre) if world == 1 else None
        return {"value": round(sit_all / world / sdt_max, 3), "unit": "LM iters/s",
                "ms_per_step": round(1e3 * sdt_max / K, 4), "streams": Bs, "ranks": world, "scaling": "strong",
                "frames_per_step": Bs, "unsharded_same_streams": round(uit / udt, 3),
                "sharded_over_unsharded": round((sit_all / world / sdt_max) / (uit / udt), 4),
                **sinfo,
                "two_kernel_lm": {"value": round(tit_all / world / tdt_max, 3),
                                  "ms_per_step": round(1e3 * tdt_max / K, 4),
                                  "over_persistent": round((tit_all / tdt_max) / (sit_all / sdt_max), 4),
                                  **tinfo,
                                  "mode": "the same sharded handle with LOAM_LM_PERSISTENT=0: per LM pass "
                                          "k_lm_eval -> RCCL all-reduce (29 f64 per stream) -> k_lm_step, the "
                                          "schedule of RCCL groups of more than one rank"},
                "transport": ("RCCL (5-NN all-gather, submap sizes, pose agreement); the LM's per-iteration "
                              "sums in IPC-mapped peer buffers when lm_path is 3" if world > 1 else
                              "one rank: every collective is the identity"),
                "mode": "every stream split over all ranks (block-owned map shards, per-round 5-NN all-gather, "
                        "per-LM-iteration normal-equation all-reduce); iterations counted once per stream",
                "thread_ranks": thread_ranks}

    def thread_rank_overhead(splan, pre, n_streams=8, steps=10):
        """the multi-rank schedule on this one GPU: R = 2, 3 ranks as host threads,
        each a sharded handle of the first n_streams streams, exchanging through the library's
        device-ordered transport (loam_comm_create_local: collectives staged and summed on the
        ranks' HIP streams, ordered by events); every rank's kernels share the GPU, so the time
        includes R times the redundant per-rank work plus the exchanges, against the unsharded
        handle on the same streams and frames"""
        import threading
        from loam_amd.comm import Comm
        plan = [BatchMapper.batch_args(*(a[:n_streams] for a in step[-1])) for step in splan[:pre + steps]]
        um = BatchMapper(n_streams, device=local, max_map_points=args.map_points)
        run_steps(um, plan, 0, pre)
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        uit = run_steps(um, plan, pre, steps)
        torch.cuda.synchronize(local)
        u_rate = uit / (time.perf_counter() - t0)
        um.close()
        res = {"streams": n_streams, "steps": steps, "unsharded": round(u_rate, 1),
               "transport": "loam_comm_create_local: ranks as threads on one GPU; the submap sizes, 5-NN "
                            "candidates and poses staged and summed on the ranks' own HIP streams, ordered by "
                            "events (threads meet only when they enqueue them); every LM pass's normal equations "
                            "meet inside the persistent LM round (peer slots and flags, lm.h)"}
        for R in (2, 3):
            comms = Comm.local_group(R, local)
            times, iters, errs = [0.0] * R, [0] * R, []
            start = threading.Barrier(R)

            def work(r):
                try:
                    m = BatchMapper(n_streams, device=local, max_map_points=args.map_points, comm=comms[r])
                    run_steps(m, plan, 0, pre)
                    torch.cuda.synchronize(local)
                    start.wait()
                    t1 = time.perf_counter()
                    iters[r] = run_steps(m, plan, pre, steps)
                    torch.cuda.synchronize(local)
                    times[r] = time.perf_counter() - t1
                    m.close()
                except BaseException as e:  # noqa: BLE001 - recorded below
                    errs.append(repr(e))
                    start.abort()  # (the other ranks' collectives fail at the group's timeout)

            th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            if errs or any(t.is_alive() for t in th):
                res[f"ranks_{R}"] = {"error": errs[0] if errs else "timeout"}
                continue
            for c in comms:
                c.close()
            rate = iters[0] / max(times)
            res[f"ranks_{R}"] = {"value": round(rate, 1), "over_unsharded": round(rate / u_rate, 4),
                                 "ms_per_step": round(1e3 * max(times) / steps, 3)}
        return res

    def single_stream(exact):
        """B = 1 on stream 0's frames (the latency view): map building untimed, then K frames,
        frame after frame.  Pipelined: frame f + 1's input and stack VoxelGrid are queued while
        frame f is in flight (loam_mapper_solve_async / _prefetch / _wait, the same results);
        the blocking loam_mapper_solve beside it"""
        out = {}
        for mode in ("pipelined", "blocking", "pose_first"):
            m1 = BatchMapper(1, device=local, exact_voxel_order=exact)
            plan1 = [step_inputs(frames, 1, args.stride, k) for k in range(pre + K)]
            run_steps(m1, plan1, 0, pre)
            torch.cuda.synchronize(local)
            t1 = time.perf_counter()
            if mode == "pipelined":
                it1 = run_steps_pipelined(m1, plan1, pre, K)
            else:
                it1 = run_steps(m1, plan1, pre, K, pose_first=mode == "pose_first")
            torch.cuda.synchronize(local)  # (every stream of the device: the last map update too)
            d1 = time.perf_counter() - t1
            m1.close()
            out[mode] = {"value": it1 / d1, "ms_per_frame": 1e3 * d1 / K, "iterations": it1}
        return {**out["pipelined"], "blocking_value": out["blocking"]["value"],
                "blocking_ms_per_frame": out["blocking"]["ms_per_frame"],
                "pose_first_value": out["pose_first"]["value"],
                "pose_first_ms_per_frame": out["pose_first"]["ms_per_frame"]}

    single = single_exact = None
    if not args.no_single_stream and rank == 0 and world == 1 and not args.shard:
        single = single_stream(args.exact_voxel_order)
        if not args.no_exact_leg and not args.exact_voxel_order:
            single_exact = single_stream(1)

    if rank == 0:
        dom = max(kt, key=lambda k: kt[k]["ms"])
        d = kt[dom]
        achieved = d["bytes"] / (d["ms"] * 1e-3) / 1e9 if d["ms"] > 0 else 0.0
        traffic = None if args.shard else pmc_traffic(dom)  # PMC passes are of the default mode
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                    "traffic": round(traffic, 1) if traffic is not None else None,
                    "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) if traffic is not None else None,
                    "launches": d["launches"], "avg_launch_us": round(1e3 * d["ms"] / max(1, d["launches"]), 3),
                    "algorithmic_bytes_per_launch": round(d["bytes"] / max(1, d["launches"]), 1),
                    "families": family_rooflines(kt, not args.shard)}
        cpu = cpu_st = rmse = allc = None
        if with_cpu:
            ci, cms, cposes = cpu_baseline(frames, pre, K)
            cpu = {"value": round(ci / (cms * 1e-3), 3), "unit": "LM iters/s", "cores": 1, "kind": "port",
                   "sample": f"stream 0's inputs, frames {pre}..{pre + K - 1} (the frames stream 0 processed in "
                             f"the timed steps) after {pre} untimed map-building frames: oracle solveMapping "
                             f"(KD-tree, VoxelGrid, Ceres-LM/DENSE_QR restatement), {ci} LM iterations in "
                             f"{cms / 1e3:.3f} s",
                   "ms_per_frame": round(cms / K, 3)}
            rmse = {"timed_frames": pose_errors(poses0[pre:pre + K], cposes[pre:pre + K]),
                    "all_frames": pose_errors(poses0, cposes),
                    "mode": "free-running: GPU stream 0 and the oracle each from frame 0 on identical "
                            "features and priors, no state shared; oracle VoxelGrids in PCL's order, GPU "
                            f"mapper in {'PCL' if args.exact_voxel_order else 'input'} order"}
            if exact_leg is not None:
                exact_leg["pose_rmse_vs_cpu"] = {"timed_frames": pose_errors(exact_leg["poses"][pre:pre + K],
                                                                             cposes[pre:pre + K]),
                                                 "all_frames": pose_errors(exact_leg["poses"], cposes)}
            # the reference against itself: the same oracle with VoxelGrid voxels summed in input
            # order instead of libstdc++'s sort permutation (a build of the reference whose sort
            # differs); the divergence a different summation order alone produces free-running
            O = _oracle()
            with O.voxel_order(1):
                _, _, cposes_in = cpu_baseline(frames, pre, K)
            rmse["reference_self_divergence"] = {
                **pose_errors(cposes_in, cposes),
                "mode": "oracle with input-order VoxelGrid sums vs oracle with PCL's order, free-running"}
            cpu_st = cpu_stages(frames, pre, K)
            ai, adt = cpu_all_cores(frames, cores, args.stride, pre, K)
            visible = len(os.sched_getaffinity(0))
            allc = {"value": round(ai / adt, 3), "unit": "LM iters/s", "cores": cores, "kind": "port",
                    "nproc": os.cpu_count(), "visible_cores": visible,
                    "core_cap": ("replicas capped at 16: the GPU pool allots 16 host CPUs to one GPU (its "
                                 "process guard and OMP_NUM_THREADS=16), although the affinity mask shows "
                                 f"{visible}; the figure is {cores} cores, not the whole host"),
                    "per_core": round(ai / adt / cores, 3),
                    "whole_host_estimate": {
                        "value": round(ai / adt / cores * visible, 1), "cores": visible,
                        "how": "per-replica rate x visible cores (an extrapolation, not a measurement)"},
                    "sample": f"{cores} oracle replicas, one thread each, replica c on stream c's inputs: "
                              f"{pre} untimed map-building frames, then its {K} timed frames between two "
                              f"barriers; {ai} LM iterations in {adt:.3f} s"}
        out = {
            "metric": "scan-to-map LM iters/sec on 64-ring KITTI-shaped cloud",
            "value": round(iters_all / dt_max, 3),
            "unit": "LM iters/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(1e3 * dt_max / K, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.shard else "weak",
            "vs_baseline": None,
            "dtype": "fp64 pose/normal equations, fp32 points",
            "data": "synthetic HDL-64E street sequence (64 rings x 2000 azimuths); GPU scan registration "
                    f"features; mapping prior from {'GPU LaserOdometry' if args.prior == 'odometry' else 'ground truth + random walk'}; "
                    f"maps built by {pre} untimed steps before the timed ones",
            "config": {"workload": "laserMapping solveMapping, voxel-hashed map resident in HBM "
                                   "(BASELINE configs[3])",
                       "streams_per_gpu": B, "frames_per_step": B if args.shard else B * world,
                       "n_az": args.n_az, "map_frames_before_timing": pre, "stride": args.stride,
                       "voxel_order": "PCL (exact)" if args.exact_voxel_order else "input order",
                       "parallelism": (f"{B} streams, each sharded over {world} GPU(s): RCCL all-gather of the "
                                       f"5-NN candidates per round, all-reduce of the normal equations per LM "
                                       f"iteration" if args.shard else
                                       f"{world} GPU x {B} independent streams"
                                       + (f" ({H} handles x {Bh}, one host thread each)" if H > 1 else "")),
                       "steps": ("blocking: one after the other" if args.blocking else
                                 "pipelined: each handle queues step k + 1 (its stack VoxelGrid runs beside step k) "
                                 "before waiting for step k")},
            "lm_iterations": int(iters_all),
            "kernel_ms_per_step": {k: round(v["ms"] / K, 4) for k, v in kt.items()},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pose_rmse_vs_cpu": rmse,
            "cpu_all_cores": allc,
        }
        if single is not None:
            out["single_stream"] = {k: round(v, 4) for k, v in single.items()}
        if single_exact is not None:
            out["single_stream_exact_voxel_order"] = {k: round(v, 4) for k, v in single_exact.items()}
        if exact_leg is not None:
            exact_leg.pop("poses")
            exact_leg["value"] = round(exact_leg["value"], 3)
            exact_leg["ms_per_step"] = round(exact_leg["ms_per_step"], 4)
            exact_leg["mode"] = ("the same workload with exact_voxel_order = 1 (the mapper's VoxelGrids in PCL's "
                                 "summation order: free-running poses follow the oracle bit for bit)")
            out["exact_voxel_order"] = exact_leg
        # the stages before the mapper (BASELINE configs[1], configs[2]): one stream, device time
        # per frame (HIP events around each call) over the cpu_baseline frames (all frames after
        # the first 10 without the CPU leg), and the oracle's own timers over the same frames
        stages = {}
        for name in ("scan_registration", "odometry"):
            sl = slice(pre, pre + K) if cpu_st is not None else slice(10, None)
            g = np.array(stage_ms[name][sl], dtype=np.float64)
            if not len(g):
                continue
            e = {"gpu_ms_per_frame": round(float(g.mean()), 4), "gpu_frames": int(len(g)),
                 "gpu_frames_per_s": round(1e3 / float(g.mean()), 1)}
            ga = np.array(stage_ms[name][10:], dtype=np.float64)
            if cpu_st is not None and len(ga):
                # the frames above are the cpu_baseline's (a 20-frame sample); every frame after
                # the first 10 of the sequence, for the distribution (per-frame time varies with
                # the scene: the nearest ring's sort for scan registration)
                e["gpu_all_frames"] = {"ms_per_frame": round(float(ga.mean()), 4), "frames": int(len(ga)),
                                       "median_ms": round(float(np.median(ga)), 4),
                                       "p90_ms": round(float(np.percentile(ga, 90)), 4)}
            # the stage against the HBM roofline: its algorithmic bytes per frame / its device time
            # per frame (every kernel of the stage, one stream: latency bound)
            bpf = float(np.mean(stage_ms[name + "_bytes"][sl]))
            ach = bpf / (float(g.mean()) * 1e-3) / 1e9
            e["roofline"] = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 6), "algorithmic_bytes_per_frame": round(bpf, 1),
                             "traffic": None, "bytes": ("24 B per raw point" if name == "scan_registration" else
                                                         "last clouds + queries + LM passes x records")}
            if name == "odometry":
                it = float(np.sum(stage_ms["odometry_iters"][sl]))
                e["gpu_lm_iters_per_s"] = round(it / (float(g.sum()) * 1e-3), 1)
            if cpu_st is not None:
                c = cpu_st[name] / K
                e.update(cpu_ms_per_frame=round(c, 4), cpu_cores=1, cpu_kind="port",
                         speedup=round(c / float(g.mean()), 2))
                if name == "odometry":
                    e["cpu_lm_iters_per_s"] = round(cpu_st["odometry_iters"] / (cpu_st[name] * 1e-3), 1)
            stages[name] = e
        if world == 1 and "scan_registration" in stages:
            stages["scan_registration"]["batched"] = scanreg_batched_stage(args.seed, local, args.n_az)
        if world == 1 and "odometry" in stages:
            stages["odometry"]["batched"] = odometry_batched_stage(frames, local)
        if not args.no_depth and world == 1:
            stages["depth_association"] = depth_stage(args.seed, local, with_cpu=not args.no_cpu)
            stages["vo_solve"] = vo_stage(args.seed, local, with_cpu=not args.no_cpu)
            stages["pipeline_one_stream"] = pl = pipeline_stage(args.seed, local)
            if cpu_st is not None:  # the oracle's three stages back to back, one core
                c = (cpu_st["scan_registration"] + cpu_st["odometry"]) / K + cpu["ms_per_frame"]
                pl["cpu_ms_per_frame"] = round(c, 3)
                pl["cpu_sample"] = ("oracle scan registration + odometry + mapping per frame, one core, on the "
                                    "cpu_baseline frames (same sequence shape, steady-state map)")
                for mode in ("sequential", "overlapped", "pipelined"):
                    pl[mode]["speedup_vs_cpu"] = round(c / pl[mode]["ms_per_frame"], 2)
        out["stages"] = stages
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(out["value"] / cpu["value"], 2)
            out["speedup_vs_cpu_all_cores"] = round(out["value"] / allc["value"], 2)
            # against the whole host (every visible core as an oracle replica, extrapolated from the
            # 16 measured replicas): the framing of the 128-stream batch against one core flatters
            out["speedup_vs_cpu_whole_host_estimate"] = round(out["value"] / allc["whole_host_estimate"]["value"], 2)
            if single is not None:
                out["single_stream"]["speedup_vs_cpu_baseline"] = round(single["value"] / cpu["value"], 2)
                out["single_stream"]["blocking_speedup_vs_cpu_baseline"] = round(single["blocking_value"] / cpu["value"], 2)
                out["single_stream"]["pose_first_speedup_vs_cpu_baseline"] = round(
                    single["pose_first_value"] / cpu["value"], 2)
            if single_exact is not None:
                out["single_stream_exact_voxel_order"]["speedup_vs_cpu_baseline"] = round(
                    single_exact["value"] / cpu["value"], 2)
    # the sharded leg last, so that it cannot cost the headline line: it is the one place where
    # ranks exchange data (RCCL), so a failure there is recorded in the line, and a hang ends at
    # a watchdog that prints the line without it
    if args.shard_streams > 0 and not args.shard:
        import threading

        def on_timeout():
            # a hung collective is a failure: the line is printed (the headline stands, the
            # sharded leg carries the error) and every rank exits non-zero
            if rank == 0:
                out["sharded"] = {"error": f"sharded leg did not finish within {SHARD_LEG_LIMIT_S} s"}
                print(json.dumps(out), flush=True)
            sys.stderr.write(f"bench.py: sharded leg hung (> {SHARD_LEG_LIMIT_S} s), exiting 3\n")
            sys.stderr.flush()
            os._exit(3)

        dog = threading.Timer(SHARD_LEG_LIMIT_S, on_timeout)
        dog.daemon = True
        dog.start()
        try:
            shard_leg = run_shard_leg()
        except Exception as e:  # noqa: BLE001 - recorded in the line, the headline stands
            shard_leg = {"error": repr(e)}
        dog.cancel()
        if rank == 0:
            out["sharded"] = shard_leg
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
