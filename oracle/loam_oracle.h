/*
 * loam_oracle.h — C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a single-threaded C++17 restatement of the reference LOAM hot path
 * (liuzm-slam/VLOAM-NOTED, src/lidar_odometry_mapping) and of the third-party
 * arithmetic it calls (Ceres 2.0 trust-region LM / DENSE_QR / HuberLoss /
 * EigenQuaternionParameterization, PCL VoxelGrid + KdTreeFLANN, Eigen 3.3).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the CPU baseline — never as the product path.
 *
 * PARITY UNPINNED: the reference ships no tests or golden vectors, and it cannot be
 * built here (ROS1, PCL, Ceres, Eigen are absent).  The restatement is
 * cross-checked against independent implementations (scipy cKDTree, numpy eigh /
 * lstsq, finite differences) in tests/test_oracle_*.py.
 */
#ifndef LOAM_ORACLE_H
#define LOAM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- standalone primitives (4 floats per point: x, y, z, intensity) ---- */

/* PCL VoxelGrid<PointXYZI>::filter semantics (leaf in metres); returns output count.
 * out must hold n points.  Within-voxel summation order: PCL's (std::sort of (idx, point)
 * comparing idx only), or input order after oracle_set_voxel_order(1).  Used by every
 * VoxelGrid of the oracle pipeline (ScanRegistration, LaserMapping). */
int32_t oracle_voxel_grid(const float* in, int32_t n, float leaf, float* out);
/* 0: PCL order (default), 1: input order (the mapper kernels' documented order); returns the
 * previous setting */
int32_t oracle_set_voxel_order(int32_t order);
/* the permutation libstdc++ std::sort produces on (keys[i], i) compared by key only */
int32_t oracle_std_sort_perm(const uint32_t* keys, int32_t n, int32_t* perm);

/* exact kNN (FLANN L2_Simple<float> distances, ties broken by index). */
int32_t oracle_knn(const float* pts, int32_t n, const float* q, int32_t nq, int32_t k,
                   int32_t* idx, float* d2);

/* mapping correspondence geometry (laser_mapping.cpp:557-603 / :642-680).
 * nbr: 5 points (x,y,z,i).  edge: returns 1 and a,b if line-like.  plane: returns 1
 * and n (unit), d if the plane check passes. */
int32_t oracle_edge_from_nbrs(const float* nbr, double* a, double* b);
int32_t oracle_plane_from_nbrs(const float* nbr, double* n, double* d);

/* factor record: type (1 edge, 2 plane(odometry), 3 plane-norm (mapping)),
 * p[3], a[3], b[3]  (plane: a=j, b=n;  plane-norm: a=n, b[0]=d) — 10 doubles each. */
typedef struct oracle_lm_stats {
  int32_t iterations;       /* trust-region steps taken (Ceres summary.iterations.size()-1) */
  int32_t successful;       /* accepted steps (excluding iteration 0) */
  int32_t invalid;          /* steps with model_cost_change <= 0 */
  int32_t termination;      /* 0 max-iter, 1 function tol, 2 parameter tol, 3 gradient tol, 4 no residuals, 5 failure */
  double initial_cost;
  double final_cost;
} oracle_lm_stats;

/* Ceres 2.0 TrustRegionMinimizer(LM, DENSE_QR, Huber 0.1, EigenQuaternion) on the factors.
 * x: q(x,y,z,w), t(x,y,z) in/out. */
int32_t oracle_lm_solve(const double* factors, int32_t nf, double* x, int32_t max_iter,
                        oracle_lm_stats* st);
/* cost / J^T J / J^T r (unscaled, Huber-corrected, local 6-dof) at x — for kernel checks */
int32_t oracle_lm_normal_eq(const double* factors, int32_t nf, const double* x,
                            double* cost, double* jtj36, double* jtr6);

/* ---- ScanRegistration (scan_registration.cpp:144-513) ---- */
typedef struct oracle_scanreg oracle_scanreg;
oracle_scanreg* oracle_scanreg_create(int32_t n_scans, double minimum_range);
void oracle_scanreg_destroy(oracle_scanreg* h);
/* xyz: n points with stride (floats) */
int32_t oracle_scanreg_input(oracle_scanreg* h, const float* xyz, int32_t n, int32_t stride);
/* which: 0 laserCloud, 1 sharp, 2 lessSharp, 3 flat, 4 lessFlat */
int32_t oracle_scanreg_count(oracle_scanreg* h, int32_t which);
int32_t oracle_scanreg_copy(oracle_scanreg* h, int32_t which, float* out);
/* per-point debug arrays of the concatenated cloud: curvature, label */
int32_t oracle_scanreg_curvature(oracle_scanreg* h, float* curv, int32_t* label);
double oracle_scanreg_ms(oracle_scanreg* h);

/* ---- LaserOdometry (laser_odometry.cpp:137-584) ---- */
typedef struct oracle_odom oracle_odom;
oracle_odom* oracle_odom_create(int32_t mapping_skip_frame);
void oracle_odom_destroy(oracle_odom* h);
/* clouds: full, sharp, lessSharp, flat, lessFlat (4 floats per point) */
int32_t oracle_odom_input(oracle_odom* h, const float* full, int32_t nfull, const float* sharp,
                          int32_t nsharp, const float* less_sharp, int32_t nless_sharp,
                          const float* flat, int32_t nflat, const float* less_flat,
                          int32_t nless_flat);
int32_t oracle_odom_solve(oracle_odom* h);
/* the VO prior velo_last_VOT_velo_curr (!detach_VO_LO, laser_odometry.cpp:237-250): q xyzw, t;
 * used by every following solve until cleared with NULLs */
int32_t oracle_odom_set_prior(oracle_odom* h, const double* q, const double* t);
/* q_w[4] xyzw, t_w[3], q_lc[4], t_lc[3]; returns skip_frame */
int32_t oracle_odom_output(oracle_odom* h, double* q_w, double* t_w, double* q_lc, double* t_lc);
/* which: 0 cornerLast, 1 surfLast, 2 fullRes */
int32_t oracle_odom_count(oracle_odom* h, int32_t which);
int32_t oracle_odom_copy(oracle_odom* h, int32_t which, float* out);
/* per-round stats: corner/plane correspondences + LM stats of the last solve (2 rounds) */
int32_t oracle_odom_stats(oracle_odom* h, int32_t* corr /*[4]*/, oracle_lm_stats* lm /*[2]*/);
double oracle_odom_ms(oracle_odom* h);

/* ---- LaserMapping (laser_mapping.cpp:147-814) ---- */
typedef struct oracle_map oracle_map;
typedef struct oracle_map_stats {
  int32_t optimized;            /* 0 if map too small (laser_mapping.cpp:514) */
  int32_t corner_stack, surf_stack;
  int32_t corner_map, surf_map; /* submap sizes used for the KD trees */
  int32_t corner_num[2], surf_num[2];
  oracle_lm_stats lm[2];
  int32_t center[3];            /* centerCube I,J,K after recentering */
  int32_t valid_num;
  double ms_total, ms_opt;      /* whole solveMapping, optimisation block (:516-729) */
} oracle_map_stats;

oracle_map* oracle_map_create(float line_res, float plane_res);
void oracle_map_destroy(oracle_map* h);
/* corner/surf/full: 4 floats per point; q_wodom xyzw, t_wodom xyz */
int32_t oracle_map_input(oracle_map* h, const float* corner, int32_t nc, const float* surf,
                         int32_t ns, const float* full, int32_t nf, const double* q_wodom,
                         const double* t_wodom, int32_t skip_frame);
int32_t oracle_map_solve(oracle_map* h);
int32_t oracle_map_pose(oracle_map* h, double* q_w, double* t_w);
int32_t oracle_map_get_stats(oracle_map* h, oracle_map_stats* st);
/* state for teacher forcing: cen[3], q_wmap_wodom[4], t_wmap_wodom[3] */
int32_t oracle_map_get_state(oracle_map* h, int32_t* cen, double* q_wmap_wodom, double* t_wmap_wodom);
int32_t oracle_map_set_state(oracle_map* h, const int32_t* cen, const double* q_wmap_wodom,
                             const double* t_wmap_wodom);
/* cube contents: which 0 corner, 1 surf; cube = i + 21*j + 441*k */
int32_t oracle_map_cube_count(oracle_map* h, int32_t which, int32_t cube);
int32_t oracle_map_cube_copy(oracle_map* h, int32_t which, int32_t cube, float* out);
int32_t oracle_map_cube_set(oracle_map* h, int32_t which, int32_t cube, const float* pts, int32_t n);
/* factor list of the last solved round r (0/1) — 10 doubles per factor */
int32_t oracle_map_factor_count(oracle_map* h, int32_t round);
int32_t oracle_map_factors(oracle_map* h, int32_t round, double* out);
/* pose at the start of round r (0/1) */
int32_t oracle_map_round_pose(oracle_map* h, int32_t round, double* x7);

/* ---- visual-odometry depth association (depth_oracle.cpp; point_cloud_util.cpp:183-487) ----
 * matrices row-major: cam_T_velo 4x4, rect0_T_cam 4x4, P_rect0 3x4 */
void* oracle_depth_create(const float* cam_T_velo, const float* rect0_T_cam, const float* P_rect0, int32_t grid,
                          int32_t img_w, int32_t img_h);
void oracle_depth_destroy(void* h);
/* projectPointCloud + downsamplePointCloud; returns the point_cloud_2d_dnsp count */
int32_t oracle_depth_process(void* h, const float* xyz, int32_t n, int32_t stride);
/* which 0: point_cloud_2d (n x 3), 1: point_cloud_2d_dnsp */
int32_t oracle_depth_count(void* h, int32_t which);
void oracle_depth_copy(void* h, int32_t which, float* out);
/* bucket_x / _y / _depth / _count, [i * new_height + j] */
void oracle_depth_buckets(void* h, float* bx, float* by, float* bd, int32_t* bc);
/* queryDepth of n image points (x, y); returns the milliseconds taken */
double oracle_depth_query(void* h, const float* xy, int32_t n, int32_t radius, float* depth);
double oracle_depth_ms(void* h);

/* ---- visual-odometry LM (visual_odometry.cpp:304-509): factor records of 10 doubles,
 * type 4 CostFunctor32 (p = X0, a[0..1] = x1_bar, y1_bar), type 5 CostFunctor22
 * (a[0..1] = x0_bar, y0_bar, b[0..1] = x1_bar, y1_bar); x6 = angles_0to1 (angle-axis), t_0to1.
 * Jet autodiff of the functors, HuberLoss(0.1), Ceres TR-LM / DENSE_QR on Euclidean params. */
int32_t oracle_vo_solve(const double* factors, int32_t nf, double* x6, int32_t max_iter, oracle_lm_stats* st);
/* cost, J^T J (6x6 row-major), J^T r (Huber-corrected); returns the residual rows */
int32_t oracle_vo_normal_eq(const double* factors, int32_t nf, const double* x6, double* cost, double* jtj,
                            double* jtr);

#ifdef __cplusplus
}
#endif
#endif
