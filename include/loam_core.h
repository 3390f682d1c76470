/*
 * loam_core.h — C-ABI of the MI355X-native LOAM scan-matching core.
 *
 * Drop-in boundary for the hot path of liuzm-slam/VLOAM-NOTED src/lidar_odometry_mapping
 * (paths below are relative to /root/reference/src/lidar_odometry_mapping/).  Every entry
 * point cites the reference interface it replaces.  Plain pointers and sizes only; points
 * are 4 floats (x, y, z, intensity) like pcl::PointXYZI (include/.../common.h:42); poses are
 * double quaternions in xyzw storage order (para_q / parameters[0..3]) plus xyz translation.
 *
 * Threading: a handle is not thread-safe (neither is the reference: static broadcaster at
 * laser_mapping.cpp:873, static work arrays at scan_registration.h:91-94).  Each handle owns
 * one HIP stream on its device; calls block until their results are on the host.
 *
 * Errors: every function returns LOAM_OK (0) or a negative status.  Degenerate-but-valid
 * situations the reference only logs (too few map points, laser_mapping.cpp:514-735; fewer
 * than 10 correspondences, laser_odometry.cpp:493-496) return LOAM_OK and set flags in the
 * stats structs, reproducing the reference's skip semantics instead of aborting.
 */
#ifndef LOAM_CORE_H
#define LOAM_CORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LOAM_OK 0
#define LOAM_ERR_ARG (-1)       /* null handle / pointer, bad index or size */
#define LOAM_ERR_HIP (-2)       /* HIP runtime error (message: loam_last_error) */
#define LOAM_ERR_CAPACITY (-3)  /* a device buffer would overflow (see loam_params caps) */
#define LOAM_ERR_STATE (-4)     /* call out of order (e.g. solve without input) */
#define LOAM_ERR_NODEVICE (-5)  /* no HIP device / wrong architecture */
#define LOAM_ERR_SYNC (-6)      /* a bounded device wait ran out: a persistent LM round's workgroup
                                   hand-off (lm.h), the frame's stack VoxelGrid, or a wave's wait in
                                   the PCL-order sort's subtree drain (voxel_hot.h); the frame's state
                                   is not trustworthy: reset the stream */
#define LOAM_ERR_EARLIER (-7)   /* loam_mapper_wait / _solve: the frame this call finished is fine,
                                   but an earlier one, finished by loam_mapper_solve_async to make
                                   room, failed with LOAM_ERR_CAPACITY or _SYNC (loam_last_error
                                   names it); that frame was committed as computed */

/* ROS parameters of loam_velodyne_HDL_64_kitti.launch:3-16 + vloam_main.launch:4, plus
 * device capacities.  loam_params_default() gives the KITTI launch values. */
typedef struct loam_params {
  int32_t scan_line;                /* 64 (scan_registration.cpp:50) */
  double minimum_range;             /* 5.0 m (scan_registration.cpp:53) */
  int32_t mapping_skip_frame;       /* 1 (laser_odometry.cpp:53) */
  int32_t map_pub_number;           /* 20 (laser_mapping.cpp:127) */
  double mapping_line_resolution;   /* 0.4 m (laser_mapping.cpp:99) */
  double mapping_plane_resolution;  /* 0.8 m (laser_mapping.cpp:101) */
  int32_t detach_vo_lo;             /* 1 (laser_odometry.cpp:47); 0: coupled mode, loam_odometry_set_prior
                                       is required before every solve (:237-250) */
  int32_t verbose_level;            /* loam_verbose_level */
  /* device capacities (per stream) */
  int32_t max_input_points;         /* max points per input cloud (default 262144) */
  int32_t max_map_points;           /* arena capacity per map (corner/surf) (default 2097152) */
  int32_t max_submap_points;        /* 5x5x3-cube submap capacity per map (default 524288) */
  /* the mapper's VoxelGrids (stacks, laser_mapping.cpp:492-500; cube re-filter, :795-808):
   * 1 = PCL's within-voxel summation order (the libstdc++ sort permutation of voxel_grid.hpp;
   * bit-exact with the reference arithmetic), 0 = input order (no sort emulation, merge path for
   * cubes that gain a few points; centroids differ from PCL's within the float summation-order
   * bound).  ScanRegistration's per-ring filter always uses PCL's order.  Default 0: the exact
   * order costs ~7x in mapping throughput; teacher-forced per-scan poses agree
   * with the reference within 1e-4 either way, free-running trajectories bit-for-bit only with 1. */
  int32_t exact_voxel_order;
} loam_params;

void loam_params_default(loam_params* p);
const char* loam_last_error(void);
int32_t loam_version(void);

/* --------------------------------------------------------------------------------------
 * Per-call statistics (the reference's TicToc probes, laser_mapping.cpp:502-811, and the
 * Ceres summaries it discards).
 * ------------------------------------------------------------------------------------ */
typedef struct loam_lm_stats {
  int32_t iterations;   /* trust-region steps (Ceres summary.iterations.size() - 1) */
  int32_t successful;   /* accepted steps */
  int32_t invalid;      /* steps with model_cost_change <= 0 */
  int32_t termination;  /* 0 max-iter, 1 function tol, 2 parameter tol, 3 gradient tol,
                           4 no residuals, 5 failure */
  double initial_cost;
  double final_cost;
} loam_lm_stats;

typedef struct loam_map_stats {
  int32_t optimized;             /* 0: map too small, no optimisation (laser_mapping.cpp:514) */
  int32_t corner_stack, surf_stack;
  int32_t corner_map, surf_map;  /* submap sizes (laserCloudCornerFromMapNum, ...) */
  int32_t corner_num[2], surf_num[2];  /* factors per outer round */
  loam_lm_stats lm[2];
  int32_t center[3];             /* centerCubeI/J/K after recentering */
  int32_t valid_num;             /* laserCloudValidNum */
  double ms_total;               /* device time of the whole solveMapping (0 when queued) */
  double ms_opt;                 /* device time of the optimisation block (:516-729) */
  int32_t queued;                /* 1: ran queued behind another frame, records prepared on the
                                  * device (loam_mapper_solve_async) */
  int32_t rerun;                 /* 1: deferred by the device (recentering / compaction due) and
                                  * run again on the host-prepared path */
} loam_map_stats;

/* --------------------------------------------------------------------------------------
 * ScanRegistration (scan_registration.h:64-81): one frame per call, outputs stay in HBM.
 * ------------------------------------------------------------------------------------ */
typedef struct loam_scanreg loam_scanreg;

/* ScanRegistration::init (scan_registration.cpp:42-92); scan_line 16/32/64 */
int32_t loam_scanreg_create(const loam_params* p, int32_t device, loam_scanreg** out);
int32_t loam_scanreg_destroy(loam_scanreg* h);
/* ScanRegistration::input (scan_registration.cpp:144-513): n points, `stride` floats per
 * point (x, y, z first), host or device memory */
int32_t loam_scanreg_input(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride);
int32_t loam_scanreg_input_device(loam_scanreg* h, const float* d_xyz, int32_t n, int32_t stride);
/* ingest (the PointCloud2 -> pcl conversion of vloam_main_node.cpp:160):
 * a page-locked host buffer of cap_points x 4 floats owned by the handle.  A PointCloud2's
 * data can be written there directly; its point_step / 4 is the stride. */
int32_t loam_scanreg_host_buffer(loam_scanreg* h, float** ptr, int32_t* cap_points);
/* loam_scanreg_input without waiting: the H2D copy and the kernels are queued on the handle's
 * stream and overlap whatever the caller does next (e.g. the previous frame's
 * loam_mapper_solve).  Host memory must stay untouched until loam_scanreg_wait.  The copy is
 * asynchronous only from loam_scanreg_host_buffer memory; every other loam_scanreg_* call
 * waits first. */
int32_t loam_scanreg_input_async(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride);
int32_t loam_scanreg_wait(loam_scanreg* h);
/* ScanRegistration::output (scan_registration.cpp:566-577): which = 0 laserCloud,
 * 1 cornerPointsSharp, 2 cornerPointsLessSharp, 3 surfPointsFlat, 4 surfPointsLessFlat */
int32_t loam_scanreg_counts(loam_scanreg* h, int32_t* counts5);
/* copies cloud `which` (4 floats / point) into out (capacity cap points); returns count */
int32_t loam_scanreg_copy(loam_scanreg* h, int32_t which, float* out, int32_t cap);
/* device pointer of cloud `which`, valid until the next input; returns count */
int32_t loam_scanreg_device_ptr(loam_scanreg* h, int32_t which, const float** ptr);
/* per-point curvature and label of laserCloud (cloudCurvature / cloudLabel) */
int32_t loam_scanreg_curvature(loam_scanreg* h, float* curv, int32_t* label, int32_t cap);
/* device time of the last input (ms) */
double loam_scanreg_ms(loam_scanreg* h);
/* Batched ScanRegistration: up to max_frames independent scans per launch sequence (every kernel
 * runs frame f in grid row f), for throughput on many streams or sensors.  A batch handle also
 * takes every single-frame call above (frame 0).  loam_scanreg_input_batch runs n_frames scans
 * (xyz[f]: host or, with on_device != 0, device pointers as integers; n[f] points each, stride
 * floats per point) and waits; each frame's clouds are then read by frame index.  Results are
 * bit-identical to one loam_scanreg_input per scan. */
int32_t loam_scanreg_create_batch(const loam_params* p, int32_t device, int32_t max_frames, loam_scanreg** out);
int32_t loam_scanreg_input_batch(loam_scanreg* h, int32_t n_frames, const uint64_t* xyz, const int32_t* n,
                                 int32_t stride, int32_t on_device);
int32_t loam_scanreg_frame_counts(loam_scanreg* h, int32_t frame, int32_t* counts5);
int32_t loam_scanreg_frame_device_ptr(loam_scanreg* h, int32_t frame, int32_t which, const float** ptr);
int32_t loam_scanreg_frame_copy(loam_scanreg* h, int32_t frame, int32_t which, float* out, int32_t cap);
/* cumulative device cycle counters of scan registration, summed over rings and frames unless
 * "max": the per-ring PCL-order VoxelGrid (k_sr_ring_features' second phase): [0] cycles of the sort emulation
 * (libstdc++ introsort) for the voxels of 3+ members, [1] of their centroids, [2] rings that had
 * such a voxel, [3] max cycles of one ring, [4] cycles of the input-order filter, [5] points,
 * [6] max points of one ring, [7] max elements heap-sorted in one ring, [8] elements heap-sorted
 * at the depth limit, [9..12] cycles of the sort's setup, workgroup levels, wave subtrees and
 * positions; the feature selection (its first phase): [13] cycles of the sector sorts, [14] of the
 * greedy picks, [15] max cycles of one ring, [19] / [20] max of one ring's sector sorts / greedy
 * picks; [16] the slowest VoxelGrid ring: its cycles << 32 | heap-sorted elements << 16 | points,
 * [18] its cycles << 32 | its cycles after the input-order filter.  Counted only in a handle
 * created with LOAM_PHASE_COUNTERS=1 in the environment.  Always counted: [21] sectors whose
 * greedy picks were rerun with the flags inherited from the sector before, [22] rings whose
 * sectors ran concurrently.  reset = 1 zeroes them after the copy. */
#define LOAM_SR_DEBUG_COUNTERS 24
int32_t loam_scanreg_debug_counters(loam_scanreg* h, uint64_t* out, int32_t n, int32_t reset);

/* --------------------------------------------------------------------------------------
 * LaserOdometry (laser_odometry.h:70-84) — scan-to-scan odometry, n_streams independent
 * instances per handle.  One solve = laserOdometryIO's input + solveLO (laser_odometry.cpp:
 * 137-584) for every stream that received an input.
 * ------------------------------------------------------------------------------------ */
typedef struct loam_odometry loam_odometry;

typedef struct loam_odom_stats {
  int32_t corner_num[2], surf_num[2];  /* corner / plane correspondences per round */
  loam_lm_stats lm[2];
  int32_t n_corner_last, n_surf_last;  /* laserCloudCornerLast / SurfLast sizes after the swap */
  double ms;                           /* device time of the whole call (all streams) */
} loam_odom_stats;

/* LaserOdometry::init (laser_odometry.cpp:46-126); mapping_skip_frame from params */
int32_t loam_odometry_create(const loam_params* p, int32_t device, int32_t n_streams, loam_odometry** out);
int32_t loam_odometry_destroy(loam_odometry* h);
int32_t loam_odometry_reset(loam_odometry* h);
/* LaserOdometry::input (laser_odometry.cpp:137-150): cornerPointsSharp, cornerPointsLessSharp,
 * surfPointsFlat, surfPointsLessFlat (4 floats / point, host memory, copied) */
int32_t loam_odometry_input(loam_odometry* h, int32_t stream, const float* sharp, int32_t n_sharp,
                            const float* less_sharp, int32_t n_less_sharp, const float* flat, int32_t n_flat,
                            const float* less_flat, int32_t n_less_flat);
/* same, device pointers read in place during the next solve (e.g. loam_scanreg_device_ptr) */
int32_t loam_odometry_input_device(loam_odometry* h, int32_t stream, const float* sharp, int32_t n_sharp,
                                   const float* less_sharp, int32_t n_less_sharp, const float* flat,
                                   int32_t n_flat, const float* less_flat, int32_t n_less_flat);
/* the VO prior of the next solve, vloam_tf->velo_last_VOT_velo_curr (q xyzw, t), with
 * detach_vo_lo = 0 (laser_odometry.cpp:237-250): both outer rounds start from it.  Required for
 * every stream with an input when detach_vo_lo = 0 (solve returns LOAM_ERR_STATE otherwise),
 * rejected (LOAM_ERR_STATE) when detach_vo_lo = 1; consumed by the solve; NULLs clear it. */
int32_t loam_odometry_set_prior(loam_odometry* h, int32_t stream, const double* q_xyzw, const double* t_xyz);
/* LaserOdometry::solveLO (laser_odometry.cpp:199-584) */
int32_t loam_odometry_solve(loam_odometry* h);
/* LaserOdometry::output (laser_odometry.cpp:660-679): q_w_curr, t_w_curr, q_last_curr,
 * t_last_curr (each may be NULL), skip_frame = frameCount % mapping_skip_frame != 0 */
int32_t loam_odometry_output(loam_odometry* h, int32_t stream, double* q_w, double* t_w, double* q_lc,
                             double* t_lc, int32_t* skip_frame);
/* laserCloudCornerLast (which 0) / laserCloudSurfLast (1): device pointer valid until the
 * next solve (feeds loam_mapper_input_device); returns the count */
int32_t loam_odometry_last_cloud(loam_odometry* h, int32_t stream, int32_t which, const float** d_ptr);
int32_t loam_odometry_copy_last(loam_odometry* h, int32_t stream, int32_t which, float* out, int32_t cap);
int32_t loam_odometry_stats(loam_odometry* h, int32_t stream, loam_odom_stats* st);

/* --------------------------------------------------------------------------------------
 * LaserMapping (laser_mapping.h:85-100) — a handle holds n_streams independent mappers
 * (independent sequences / vehicles) processed together by every launch.  n_streams = 1 is
 * exactly the reference's single LaserMapping object.
 * ------------------------------------------------------------------------------------ */
typedef struct loam_mapper loam_mapper;

/* LaserMapping::LaserMapping + init (laser_mapping.cpp:40-129) */
int32_t loam_mapper_create(const loam_params* p, int32_t device, int32_t n_streams,
                           loam_mapper** out);
int32_t loam_mapper_destroy(loam_mapper* h);
/* re-init all streams: empty maps, identity poses (laser_mapping.cpp:47-97) */
int32_t loam_mapper_reset(loam_mapper* h);

/* LaserMapping::input (laser_mapping.cpp:178-209): host clouds, deep-copied to HBM.
 * corner = laserCloudCornerLast, surf = laserCloudSurfLast (4 floats / point). */
int32_t loam_mapper_input(loam_mapper* h, int32_t stream, const float* corner, int32_t n_corner,
                          const float* surf, int32_t n_surf, const double* q_wodom,
                          const double* t_wodom, int32_t skip_frame);
/* same, clouds already resident in HBM on the handle's device (device pointers, read in place:
 * they must stay valid until loam_mapper_solve returns) */
int32_t loam_mapper_input_device(loam_mapper* h, int32_t stream, const float* d_corner,
                                 int32_t n_corner, const float* d_surf, int32_t n_surf,
                                 const double* q_wodom, const double* t_wodom,
                                 int32_t skip_frame);
/* loam_mapper_input_device for n streams at once: streams[i], device pointers (as integers),
 * sizes, q_wodom (n x 4), t_wodom (n x 3); skip_frame = 0 */
int32_t loam_mapper_input_device_batch(loam_mapper* h, int32_t n, const int32_t* streams,
                                       const uint64_t* d_corner, const int32_t* n_corner,
                                       const uint64_t* d_surf, const int32_t* n_surf,
                                       const double* q_wodom, const double* t_wodom);
/* LaserMapping::solveMapping (laser_mapping.cpp:212-814) for every stream that received an
 * input since the last call (skip_frame inputs only update the high-frequency pose).
 * A negative status (LOAM_ERR_CAPACITY: a device buffer overflowed; LOAM_ERR_SYNC: an LM hand-off
 * timed out; loam_last_error names the stream and the cause) still leaves the frame committed
 * as computed (pose, insertion, re-VoxelGrid): reset the failed stream before relying on it. */
int32_t loam_mapper_solve(loam_mapper* h);
/* loam_mapper_solve in two halves: _async enqueues the frame on the handle's HIP streams and
 * returns; _wait blocks until the OLDEST frame not yet waited for is done and then does its host
 * side (transformUpdate, laser_mapping.cpp:147-151, stats, status).
 * Up to two frames can be in the queue: while frame f is in flight, frame f + 1's inputs may be
 * given (loam_mapper_input*) and _async called again.  On a handle that runs frames as one
 * hipGraph (<= 4 streams, not sharded, profiling off) frame f + 1 is then queued behind f on the
 * device: its stream records (the initial guess :206-207 from f's transformUpdate, the cube
 * window :228-251) are prepared by the device, so the GPU goes from f to f + 1 without a host
 * round trip.  A frame the host foresees recentering (:252-444) waits, pending, for f to be
 * waited for; one the device finds recentering or due for an arena compaction is deferred and
 * run again on the host-prepared path (loam_map_stats.queued / .rerun say which happened).
 * Otherwise (other handles) frame f + 1's stack VoxelGrids (:492-500) run beside f and the rest
 * is enqueued by the _wait that finishes f, before it returns.  loam_mapper_prefetch queues the
 * stack VoxelGrids of given inputs early.
 * The results are those of the sequential loam_mapper_solve, bit for bit; only the order in time
 * changes.  loam_mapper_pose / _stats / _stats_all / _total_iterations / _get_state report the
 * newest frame waited for (a frame enqueued with nothing before it in the queue is waited for by
 * them first); every other call waits for every frame in the queue.  Device inputs must stay
 * valid until the frame that takes them is waited for.
 * Status: _async returns LOAM_OK exactly when it enqueued the new frame; any other status means
 * nothing was enqueued (give the same input again or drop it).  _async called with two frames in
 * the queue first finishes the oldest (its pose and stats are readable as after _wait); if that
 * frame failed (LOAM_ERR_CAPACITY / LOAM_ERR_SYNC) its status is held and the next _wait or
 * loam_mapper_solve returns LOAM_ERR_EARLIER (unless the frame that call finishes fails itself,
 * which is returned first; the held status then waits for the call after).  _wait returns the
 * status of the frame it finishes.  A queued frame that could not be enqueued when its turn came
 * is dropped, and the call that tried returns that error with "dropped" in loam_last_error. */
int32_t loam_mapper_solve_async(loam_mapper* h);
int32_t loam_mapper_wait(loam_mapper* h);
/* loam_mapper_solve for a caller that needs the pose before the map update: it returns once the
 * frame's optimisation is done (laser_mapping.cpp:516-736: the pose the node publishes as
 * /aft_mapped_to_init, and the frame's stats), while the insertion and re-VoxelGrid of the cubes
 * (:741-808) are still running on the device.  They finish beside the next frame's stack
 * VoxelGrid (the next call queues that frame behind this one, as loam_mapper_solve_async does)
 * or before any call that reads or changes the map (every call but _pose / _stats / _stats_all /
 * _total_iterations / _get_state, which report this frame).  Same results as loam_mapper_solve,
 * bit for bit.  Status: a failure found by the optimisation (or a deferred frame, run again on
 * the host path) is returned by this call, after the whole frame; one of the map update
 * (LOAM_ERR_CAPACITY) is returned as LOAM_ERR_EARLIER by the next solve / wait.  Frames that
 * do not run as the handle's hipGraph (handles of more than 4 streams, sharded, profiling, a
 * recentering or compaction ahead) are finished whole.  The first call switches the handle's
 * frame sequence to one that also writes the records after the optimisation. */
int32_t loam_mapper_solve_pose(loam_mapper* h);
/* queue the stack VoxelGrids of every stream's pending input now */
int32_t loam_mapper_prefetch(loam_mapper* h);
/* pose after solveMapping: q_w_curr (xyzw), t_w_curr (laser_mapping.cpp:826-832) */
int32_t loam_mapper_pose(loam_mapper* h, int32_t stream, double* q_w, double* t_w);
int32_t loam_mapper_stats(loam_mapper* h, int32_t stream, loam_map_stats* st);
/* device phase counters (diagnostics, n <= LOAM_DEBUG_COUNTERS): [0..2] re-VoxelGrid cycles
 * merge / full / append, [3] new points of merged cubes, [4..6] items of each, [7] merges with
 * more than 1024 new points, [8] cell-index build cycles, [9] points indexed, [10] old points,
 * [11..14] merge phases (bounding box, hash + pass A, new-voxel sort, pass B), [15] LM step
 * alone (lane 0), [16] cell-index hash phase, [17..21] LM round: leader eval, leader wait,
 * reduce + step, passes, member wait, [22..23] the leader's share-0 evaluation: record loop,
 * block reduction,
 * [24..31] re-VoxelGrid items by output size (< 1k, 2k, 4k, 8k, 16k, 32k, 64k, more),
 * [32..39] their cycles (filter + index), [40] sharded: pose values that differed from rank 0's
 * after the LM (0 when the all-reduce is bit-identical on every rank), [41] arena compactions
 * ((stream, map) pairs), [42..45] stack VoxelGrid cycles: bounding box, hash, sort + scan,
 * member lists + centroids, [46..47] of the latter: member lists, per-voxel sort + sums,
 * [48..49] arena compactions of the corner / surf maps (summed over streams), [50..52] exact
 * order (exact_voxel_order = 1) cube re-filters with a voxel of 3+ members: cycles of the pruned
 * sort emulation (libstdc++ introsort), of those voxels' centroids, filters (voxel_hot.h), [54..56] the same for
 * the stack VoxelGrids, [72..76] the cube emulation's elements heap-sorted literally, then cycles
 * of its setup, workgroup partitions, wave subtrees, positions, [77..81] the same for stacks,
 * [82..90] the cube emulation's wave partitions by length (<= 65, 129, 257, 513, 1025), wave
 * cycles in subtrees (sum, longest drain), heap-sort cycles, subtrees,
 * [58..61] k_frame_prep cycles: FrameIn load, device preparation, stack sizes, submap offsets,
 * [62] its launches, [63] of them frames prepared on the device, [64..65] PCL-order VoxelGrid
 * (exact_voxel_order = 1) sorts in global memory: cycles of their own levels, cubes / stacks
 * ([11..14] / [42..45] hold the rest), [66..67] cube sorts' depth-limit segments and their
 * elements, [68..69] the same for stack sorts, [91] the few-stream stack VoxelGrid's (k_stack_part)
 * histogram and range cuts ([42..45] then hold its bounding box, hash, sort + scan, member lists +
 * centroids, summed over its parts).
 * The cycle counters (all but [40], [41], [48], [49]; [52], [56], [66..69], [72], [77], [82..86], [90] count) run only in a handle created with the
 * environment variable LOAM_PHASE_COUNTERS=1 (they cost atomics in the kernels); else they stay 0. */
#define LOAM_DEBUG_COUNTERS 96
int32_t loam_mapper_debug_counters(loam_mapper* h, uint64_t* out, int32_t n, int32_t reset);
/* sum over the streams solved by the last loam_mapper_solve of their LM iterations (both rounds) */
int64_t loam_mapper_total_iterations(loam_mapper* h);
/* the LM schedule the handle runs (decided at create; laser_mapping.cpp:709-717 either way):
 * 0 two launches per Ceres iteration (k_lm_eval, then k_lm_step; sharded over several ranks the
 *   normal equations are all-reduced between them), 1 one persistent launch per outer round
 *   (k_lm_round), 2 the in-process group's round (k_lm_group: every rank of a
 *   loam_comm_create_local group in one launch), 3 the persistent round of ranks in separate
 *   processes, their per-iteration sums meeting in IPC-mapped peer buffers (RCCL / callback comms;
 *   LOAM_PEER_LM=0 at create keeps 0) */
int32_t loam_mapper_lm_path(loam_mapper* h);
/* stats of streams 0..n-1 */
int32_t loam_mapper_stats_all(loam_mapper* h, loam_map_stats* out, int32_t n);

/* kernel-level timing: with profiling on, every launch of loam_mapper_solve is bracketed by
 * HIP events on the handle's stream; times, launches and algorithmic bytes (DESIGN.md,
 * "Kernels") accumulate per kernel family until reset.  Families: 0 stack VoxelGrid,
 * 1 submap hash build, 2 correspondences (kNN + PCA/plane fit), 3 fused LM pass,
 * 4 insertion, 5 window-cube re-VoxelGrid, 6 other (prep / finish / shift / compaction). */
#define LOAM_KFAM_COUNT 8
typedef struct loam_kernel_times {
  double ms[LOAM_KFAM_COUNT];
  int64_t launches[LOAM_KFAM_COUNT];
  double bytes[LOAM_KFAM_COUNT];
} loam_kernel_times;
int32_t loam_mapper_set_profiling(loam_mapper* h, int32_t enable);
int32_t loam_mapper_kernel_times(loam_mapper* h, loam_kernel_times* out);
int32_t loam_mapper_reset_kernel_times(loam_mapper* h);

/* map state (for teacher-forced parity and for the /laser_cloud_map publisher,
 * laser_mapping.cpp:884-899).  cube = i + 21*j + 441*k; which: 0 corner, 1 surf. */
int32_t loam_mapper_get_state(loam_mapper* h, int32_t stream, int32_t* cen,
                              double* q_wmap_wodom, double* t_wmap_wodom);
int32_t loam_mapper_set_state(loam_mapper* h, int32_t stream, const int32_t* cen,
                              const double* q_wmap_wodom, const double* t_wmap_wodom);
int32_t loam_mapper_cube_count(loam_mapper* h, int32_t stream, int32_t which, int32_t cube);
/* laserCloudCornerStack (which 0) / laserCloudSurfStack (1) of the last solve
 * (laser_mapping.cpp:492-500): copies when cap >= the count; returns the count */
int32_t loam_mapper_stack_copy(loam_mapper* h, int32_t stream, int32_t which, float* out, int32_t cap);
int32_t loam_mapper_cube_copy(loam_mapper* h, int32_t stream, int32_t which, int32_t cube,
                              float* out);
int32_t loam_mapper_cube_set(loam_mapper* h, int32_t stream, int32_t which, int32_t cube,
                             const float* pts, int32_t n);
/* /laser_cloud_map (laser_mapping.cpp:884-899): corner cube 0, surf cube 0, corner cube 1, ...
 * gathered on the device; copies when cap >= the count (4 floats / point); returns the count.
 * On a sharded handle: this rank's points. */
int32_t loam_mapper_map_copy(loam_mapper* h, int32_t stream, float* out, int64_t cap);
/* /velodyne_cloud_registered (:901-911): laserCloudFullRes transformed with the pose that
 * loam_mapper_pose returns (pointAssociateToMap, :154-164); n points of 4 floats; host
 * buffers, or device buffers (in place allowed) for the _device form; returns n */
int32_t loam_mapper_register_cloud(loam_mapper* h, int32_t stream, const float* in, int32_t n, float* out);
int32_t loam_mapper_register_cloud_device(loam_mapper* h, int32_t stream, const float* d_in, int32_t n,
                                          float* d_out);

/* --------------------------------------------------------------------------------------
 * Sharded LaserMapping: one mapping stream split over `size` GPUs (ranks).
 * The reference is a single CPU thread and has no counterpart; the semantics are those of
 * LaserMapping::solveMapping (laser_mapping.cpp:212-814) unchanged.  Each rank stores the map
 * points of the 4 m voxel-aligned blocks it owns (owner = hash(block) mod size), so the
 * insertion (:741-788) and the per-cube VoxelGrid (:795-808) are rank-local and exact.  Per
 * outer round every rank runs the 5-NN (:554, :633) of every query over its own points; one
 * all-gather merges the per-rank candidate lists into the exact 5-NN.  Every LM pass (Ceres
 * iteration, :709-729) evaluates a 1/size share of the factors and all-reduces the 29 fp64
 * normal-equation sums (J^T J upper, J^T r, cost, rows); all ranks then take the identical
 * trust-region step.  Per frame: one all-reduce of the window cube counts (the submap
 * sizes of :475-489 and the skip test of :514).
 *
 * Transport: a loam_comm is either RCCL (built in, loaded at run time from librccl.so.1; the
 * collectives are enqueued on the mapper's HIP stream, no host synchronisation) or caller
 * callbacks.  All ranks call loam_mapper_solve with identical inputs (the feature clouds are
 * broadcast by the caller, like the reference's single input() call).
 * ------------------------------------------------------------------------------------ */
typedef struct loam_comm loam_comm;

#define LOAM_DT_F64 0
#define LOAM_DT_I32 1
#define LOAM_RCCL_ID_BYTES 128

typedef struct loam_comm_ops {
  void* user;
  /* 1: the library synchronises its stream and passes host (pinned) copies of the buffers;
     0: device pointers, and hip_stream is the mapper's HIP stream handle to order the work on */
  int32_t host_buffers;
  /* in-place sum over all ranks of count elements of dtype (LOAM_DT_*); returns 0 on success */
  int32_t (*allreduce_sum)(void* user, void* buf, int64_t count, int32_t dtype, void* hip_stream);
  /* recv[r * bytes .. (r + 1) * bytes) = rank r's send, for every rank r; returns 0 on success */
  int32_t (*allgather)(void* user, const void* send, void* recv, int64_t bytes, void* hip_stream);
} loam_comm_ops;

int32_t loam_comm_create(int32_t rank, int32_t size, const loam_comm_ops* ops, loam_comm** out);
/* RCCL: rank 0 makes the id (ncclGetUniqueId), the caller distributes it to every rank */
int32_t loam_comm_rccl_unique_id(uint8_t* id);
int32_t loam_comm_create_rccl(int32_t rank, int32_t size, const uint8_t* id, int32_t device,
                              loam_comm** out);
/* `size` ranks of ONE process sharing one device (threads, one sharded handle each): out[r] is
 * rank r's comm.  The collectives are ordered on the ranks' HIP streams by events (device-side
 * staging, an on-stream sum in rank order); the host threads meet once per collective when they
 * enqueue it and never wait for the device.  For running and measuring the multi-rank schedule
 * on one GPU; each comm is destroyed on its own (the shared state goes with the last). */
#define LOAM_LOCAL_MAX_RANKS 8
int32_t loam_comm_create_local(int32_t size, int32_t device, loam_comm** out);
int32_t loam_comm_destroy(loam_comm* c);
/* collectives through a comm on a device buffer (for tests and callers' own exchanges) */
int32_t loam_comm_allreduce_sum(loam_comm* c, void* d_buf, int64_t count, int32_t dtype,
                                void* hip_stream);
int32_t loam_comm_allgather(loam_comm* c, const void* d_send, void* d_recv, int64_t bytes,
                            void* hip_stream);

/* a mapper whose streams are each sharded over the comm's ranks (one handle per rank, every
 * rank with the same n_streams and params); the comm must outlive the mapper */
int32_t loam_mapper_create_sharded(const loam_params* p, int32_t device, int32_t n_streams,
                                   loam_comm* comm, loam_mapper** out);
/* the rank (of nrank) that stores map point xyz of a map with VoxelGrid leaf `leaf`
 * (mapping_line_resolution for corners, mapping_plane_resolution for surfs); host only */
int32_t loam_shard_owner(const float* xyz, float leaf, int32_t nrank);

/* --------------------------------------------------------------------------------------
 * Visual-odometry depth association — vloam::PointCloudUtil
 * (src/visual_odometry/include/visual_odometry/point_cloud_util.h:25-75), n_streams
 * independent instances per handle (the reference keeps two, point_cloud_utils[0/1]).
 * ------------------------------------------------------------------------------------ */
typedef struct loam_depth loam_depth;

typedef struct loam_depth_params {
  float cam_T_velo[16];   /* 4x4 row-major (visual_odometry.cpp:162-163) */
  float rect0_T_cam[16];  /* 4x4 row-major, R_rect_00 (point_cloud_util.cpp:113-125) */
  float P_rect0[12];      /* 3x4 row-major (visual_odometry.cpp:178-181) */
  int32_t grid;           /* downsample_grid_size, 5 */
  int32_t img_width;      /* IMG_WIDTH 1242 (point_cloud_util.h:50) */
  int32_t img_height;     /* IMG_HEIGHT 375 (point_cloud_util.h:49) */
  int32_t max_points;     /* per input cloud (default 262144) */
} loam_depth_params;

/* matrices zero (set them from the calibration), KITTI image, grid 5 */
void loam_depth_params_default(loam_depth_params* p);
int32_t loam_depth_create(const loam_depth_params* p, int32_t device, int32_t n_streams, loam_depth** out);
int32_t loam_depth_destroy(loam_depth* h);
/* point_cloud_3d_tilde of stream s (visual_odometry.cpp:201-208): n points, `stride` floats
 * each (x, y, z first); host memory (copied) or device memory (read in place) */
int32_t loam_depth_input(loam_depth* h, int32_t stream, const float* xyz, int32_t n, int32_t stride);
int32_t loam_depth_input_device(loam_depth* h, int32_t stream, const float* d_xyz, int32_t n, int32_t stride);
/* projectPointCloud + downsamplePointCloud (point_cloud_util.cpp:183-324) of every stream
 * with an input */
int32_t loam_depth_process(loam_depth* h);
/* sizes of point_cloud_2d (points in front) and point_cloud_2d_dnsp */
int32_t loam_depth_counts(loam_depth* h, int32_t stream, int32_t* n_front, int32_t* n_dnsp);
/* which 0: point_cloud_2d, 1: point_cloud_2d_dnsp, 3 floats (u, v, depth) per row; copies
 * when cap >= the count; returns the count */
int32_t loam_depth_copy(loam_depth* h, int32_t stream, int32_t which, float* out, int32_t cap);
/* bucket_x / bucket_y / bucket_depth / bucket_count, [i * new_height + j] */
int32_t loam_depth_buckets(loam_depth* h, int32_t stream, float* bx, float* by, float* bd, int32_t* bc);
/* queryDepth (point_cloud_util.cpp:381-487): depth of n image points xy (2 floats each) in
 * streams[i]'s buckets; -1 where fewer than 10 buckets are occupied (searching_radius 2) */
int32_t loam_depth_query(loam_depth* h, int32_t n, const int32_t* streams, const float* xy, int32_t radius,
                         float* depth);
int32_t loam_depth_query_device(loam_depth* h, int32_t n, const int32_t* d_streams, const float* d_xy,
                                int32_t radius, float* d_depth);
/* device time of the last loam_depth_process (ms) */
double loam_depth_ms(loam_depth* h);

/* --------------------------------------------------------------------------------------
 * Visual-odometry pose solve — VisualOdometry::solveNlsAll
 * (src/visual_odometry/src/visual_odometry.cpp:304-509): n_problems independent problems,
 * factor records of 10 doubles, problem p = records offsets[p] .. offsets[p + 1]:
 *   type 4 CostFunctor32 (ceres_cost_function.h:58-102): p = X0 (point_3d_rect0_0),
 *          a[0..1] = (x1_bar, y1_bar)
 *   type 5 CostFunctor22 (:151-189): a[0..1] = (x0_bar, y0_bar), b[0..1] = (x1_bar, y1_bar)
 * x: n_problems x 6 = angles_0to1 (angle-axis), t_0to1; in: initial values (zeros, or the
 * LiDAR-odometry prior, :311-331), out: the solution.  HuberLoss(0.1), Ceres TR-LM, DENSE_QR,
 * max_iterations (the reference: 100).  st: n_problems stats (may be NULL).
 * ------------------------------------------------------------------------------------ */
int32_t loam_vo_solve(int32_t device, int32_t n_problems, const int32_t* offsets, const double* factors,
                      double* x, int32_t max_iterations, loam_lm_stats* st);

/* --------------------------------------------------------------------------------------
 * Device LM engine on an explicit factor list (lidarFactor.hpp + Ceres TR-LM).  Factor
 * record = 10 doubles: type (1 LidarEdgeFactor, 2 LidarPlaneFactor, 3 LidarPlaneNormFactor),
 * curr_point[3], a[3], b[3] (edge: last_point_a/b; plane: j, unit normal ljm; plane-norm:
 * unit normal, negative_OA_dot_norm in b[0]).  x = q(xyzw) + t, in/out.
 * ------------------------------------------------------------------------------------ */
int32_t loam_lm_solve(int32_t device, const double* factors, int32_t n_factors, double* x,
                      int32_t max_iterations, loam_lm_stats* st);
/* cost, J^T J (6x6 row-major) and J^T r of the Huber-corrected residuals at x, in the
 * 6-dof local space of EigenQuaternionParameterization (unscaled) */
int32_t loam_lm_normal_equations(int32_t device, const double* factors, int32_t n_factors,
                                 const double* x, double* cost, double* jtj, double* jtr);

/* --------------------------------------------------------------------------------------
 * Primitives exposed for parity tests of the kernels behind the stages.
 * ------------------------------------------------------------------------------------ */
/* pcl::VoxelGrid<PointXYZI> (leaf metres) on one cloud; returns count in *n_out */
int32_t loam_voxel_grid(int32_t device, const float* in, int32_t n, float leaf, float* out,
                        int32_t* n_out);
/* pcl::VoxelGrid<PointXYZI> with PCL's own within-voxel summation order (the libstdc++
 * sort permutation of voxel_grid.hpp's (idx, point) pairs) — the order ScanRegistration's
 * per-ring filter uses (scan_registration.cpp:497-501).  loam_voxel_grid sums in input order
 * (the mapper's filters). */
int32_t loam_voxel_grid_pcl(int32_t device, const float* in, int32_t n, float leaf, float* out, int32_t* n_out);
/* the permutation libstdc++'s introsort gives the elements (keys[i], i) compared by key only
 * (the sector sort of scan_registration.cpp:365-366 and PCL's VoxelGrid sort), computed on the
 * device by n_waves (1..16) cooperating waves */
int32_t loam_sort_perm(int32_t device, const uint32_t* keys, int32_t n, int32_t n_waves, int32_t* perm);
/* VoxelGrid of fixed ++ added where `fixed` is already a VoxelGrid output of the same leaf
 * whose centroids stayed in their voxels (the per-cube map update, laser_mapping.cpp:795-808):
 * same result as loam_voxel_grid on the concatenation.  *merged = 1 if the merge path ran
 * (n1 <= 4096), 0 if the full filter did.  out holds n0 + n1 points. */
int32_t loam_voxel_merge(int32_t device, const float* fixed, int32_t n0, const float* added, int32_t n1,
                         float leaf, float* out, int32_t* n_out, int32_t* merged);
/* exact kNN (k <= 5) of queries against pts restricted to d2 < radius2 (1 m cells):
 * idx/d2 sorted ascending; missing entries idx = -1 */
int32_t loam_knn_radius(int32_t device, const float* pts, int32_t n, const float* queries,
                        int32_t nq, int32_t k, float radius2, int32_t* idx, float* d2);

#ifdef __cplusplus
}
#endif
#endif /* LOAM_CORE_H */
