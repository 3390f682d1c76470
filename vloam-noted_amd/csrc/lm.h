// lm.h — device Levenberg-Marquardt engine for the 6-dof LiDAR pose problem.
//
// Residual blocks (lidarFactor.hpp):
//   type 1 LidarEdgeFactor (3 rows)       r = (p' - a) x e,   e = (a - b)/|a - b|
//            (== ((p'-a) x (p'-b))/|a-b| of lidarFactor.hpp:41-46, rearranged)
//   type 2 LidarPlaneFactor (1 row)       r = (p' - j) . n    (lidarFactor.hpp:95)
//   type 3 LidarPlaneNormFactor (1 row)   r = n . p' + d      (lidarFactor.hpp:130)
// with p' = R(q) p + t (s = 1: DISTORTION = false, laser_odometry.h:90), analytic Jacobians in
// the local space of EigenQuaternionParameterization: dp'/d(dtheta) = -2 [R p]_x, dp'/dt = I.
// HuberLoss(0.1) + Ceres Corrector (rho'' <= 0 branch): rows scale by sqrt(rho'), so the
// normal equations accumulate rho' J^T J and rho' J^T r, cost 1/2 sum rho(|r|^2).
//
// Solver: Ceres 2.0 TrustRegionMinimizer + LevenbergMarquardtStrategy with the reference's
// options (laser_mapping.cpp:709-717, laser_odometry.cpp:500-509): radius0 1e4, Jacobi
// scaling fixed at iteration 0, LM diagonal clamp [1e-6, 1e32], min_relative_decrease 1e-3,
// function/parameter/gradient tolerances 1e-6/1e-8/1e-10, max 5 consecutive invalid steps,
// max_num_iterations 4.  Ceres factorises [J_s; D] with Householder QR (DENSE_QR); here the
// same least-squares step comes from the 6x6 normal equations (Cholesky in fp64), which is
// what a device reduction produces.  Everything the step needs is a function of
// (J^T J, J^T r, cost): one fused pass per trust-region iteration evaluates the candidate's
// cost AND its normal equations (used only if the step is accepted), so an iteration costs
// exactly one pass over the correspondences.
#pragma once
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include "common.h"
#include "device_math.h"

namespace loam {

constexpr int LM_NACC = 29;  // 21 J^T J (upper, row-major) + 6 J^T r + cost + rows

enum : int { LM_EVAL_X = 0, LM_EVAL_CAND = 1, LM_DONE = 2 };

struct LmState {
  double x[7], cand[7], best[7];
  double jtj[21], g[6];
  double cost, initial_cost, min_cost, mcc;
  double scaling[6], diag[6];
  double radius, decrease, x_norm, gmax;
  int status, iteration, reuse_diag, consec_invalid;
  int term, successful, invalid, max_iter;
  int passes;  // evaluation passes consumed (iteration 0 + candidates)
  int euclid;  // 1: x[0..5] = (angle-axis, t) with plain x + delta (the VO problem), x[6] = 0
};

__host__ __device__ inline int ut_index(int r, int c) {  // r <= c, upper triangle of 6x6
  return r * 6 - (r * (r - 1)) / 2 + (c - r);
}

__host__ __device__ inline void lm_init(LmState& S, const double* x7, int max_iter, bool active) {
  for (int i = 0; i < 7; ++i) {
    S.x[i] = x7[i];
    S.cand[i] = x7[i];
    S.best[i] = x7[i];
  }
  for (int i = 0; i < 21; ++i) S.jtj[i] = 0;
  for (int i = 0; i < 6; ++i) {
    S.g[i] = 0;
    S.scaling[i] = 1;
    S.diag[i] = 0;
  }
  S.cost = S.initial_cost = S.mcc = 0;
  S.min_cost = 1.7976931348623157e308;
  S.radius = 1e4;
  S.decrease = 2.0;
  S.x_norm = S.gmax = 0;
  S.status = active ? LM_EVAL_X : LM_DONE;
  S.iteration = 0;
  S.reuse_diag = 0;
  S.consec_invalid = 0;
  S.term = active ? 0 : 4;
  S.successful = 0;
  S.invalid = 0;
  S.max_iter = max_iter;
  S.passes = 0;
  S.euclid = 0;
}

// one residual block at X: accumulates rho' J^T J, rho' J^T r, 1/2 rho, rows.  The library
// is built with -ffp-contract=off (bit-exact VoxelGrid / kNN); here FMA contraction is allowed:
// the LM sums are matched to a tolerance (their order already differs from the reference's),
// and contraction halves the fp64 instructions of the accumulation, the bound of this loop.
// The rotation enters as the matrix of the pose's quaternion (lm_rotmat, once per pass):
// 9 multiply-adds per point instead of Eigen's two cross products.
__device__ inline void lm_rotmat(const double* X, double* Rm) {
  const double x = X[0], y = X[1], z = X[2], w = X[3];
  Rm[0] = 1.0 - 2.0 * (y * y + z * z); Rm[1] = 2.0 * (x * y - w * z); Rm[2] = 2.0 * (x * z + w * y);
  Rm[3] = 2.0 * (x * y + w * z); Rm[4] = 1.0 - 2.0 * (x * x + z * z); Rm[5] = 2.0 * (y * z - w * x);
  Rm[6] = 2.0 * (x * z - w * y); Rm[7] = 2.0 * (y * z + w * x); Rm[8] = 1.0 - 2.0 * (x * x + y * y);
}

__device__ inline void lm_accum(int type, float px, float py, float pz, double a0, double a1,
                                double a2, double b0, double b1, double b2, const double* Rm,
                                const double* X, double* acc) {
#pragma clang fp contract(fast)
  const double dx = px, dy = py, dz = pz;
  d3 Rp{Rm[0] * dx + Rm[1] * dy + Rm[2] * dz, Rm[3] * dx + Rm[4] * dy + Rm[5] * dz,
        Rm[6] * dx + Rm[7] * dy + Rm[8] * dz};
  d3 lp{Rp.x + X[4], Rp.y + X[5], Rp.z + X[6]};
  double J[3][6];
  double r[3];
  int m;
  if (type == 1) {
    // r = u x e ; dr/dlp = -[e]x ; J_rot = 2 [e]x [Rp]x ; J_t = -[e]x
    d3 u{lp.x - a0, lp.y - a1, lp.z - a2};
    r[0] = u.y * b2 - u.z * b1;
    r[1] = u.z * b0 - u.x * b2;
    r[2] = u.x * b1 - u.y * b0;
    const double E[3][3] = {{0, -b2, b1}, {b2, 0, -b0}, {-b1, b0, 0}};
    const double K[3][3] = {{0, -Rp.z, Rp.y}, {Rp.z, 0, -Rp.x}, {-Rp.y, Rp.x, 0}};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        J[i][c] = 2.0 * (E[i][0] * K[0][c] + E[i][1] * K[1][c] + E[i][2] * K[2][c]);
        J[i][3 + c] = -E[i][c];
      }
    }
    m = 3;
  } else {
    if (type == 2)
      r[0] = ((lp.x - a0) * b0 + (lp.y - a1) * b1) + (lp.z - a2) * b2;  // n = b
    else
      r[0] = ((a0 * lp.x + a1 * lp.y) + a2 * lp.z) + b0;  // n = a, d = b0
    const double nx = type == 2 ? b0 : a0, ny = type == 2 ? b1 : a1, nz = type == 2 ? b2 : a2;
    // J_rot = 2 (Rp x n)^T, J_t = n^T
    J[0][0] = 2.0 * (Rp.y * nz - Rp.z * ny);
    J[0][1] = 2.0 * (Rp.z * nx - Rp.x * nz);
    J[0][2] = 2.0 * (Rp.x * ny - Rp.y * nx);
    J[0][3] = nx;
    J[0][4] = ny;
    J[0][5] = nz;
    m = 1;
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < m) s += r[i] * r[i];
  double rho0, rho1;
  if (s > 0.01) {
    const double sq = sqrt(s);
    rho0 = 2.0 * 0.1 * sq - 0.01;
    rho1 = fmax(2.2250738585072014e-308, 0.1 / sq);
  } else {
    rho0 = s;
    rho1 = 1.0;
  }
  acc[27] += 0.5 * rho0;
  acc[28] += (double)m;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= m) break;
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const double wa = rho1 * J[i][a];
#pragma unroll
      for (int b = a; b < 6; ++b) acc[k++] += wa * J[i][b];
      acc[21 + a] += wa * r[i];
    }
  }
}

// EigenQuaternionParameterization::Plus + Euclidean t; euclid: x + d on all 6 parameters
__host__ __device__ inline void lm_plus(const double* x, const double* d, double* out, int euclid = 0) {
  if (euclid) {
    for (int i = 0; i < 6; ++i) out[i] = x[i] + d[i];
    out[6] = x[6];
    return;
  }
  double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    double sn, cs;
    sincos(nd, &sn, &cs);
    double s = sn / nd;
    dq dqq{s * d[0], s * d[1], s * d[2], cs};
    dq r = qmul(dqq, dq{x[0], x[1], x[2], x[3]});
    out[0] = r.x;
    out[1] = r.y;
    out[2] = r.z;
    out[3] = r.w;
  } else {
    out[0] = x[0];
    out[1] = x[1];
    out[2] = x[2];
    out[3] = x[3];
  }
  out[4] = x[4] + d[3];
  out[5] = x[5] + d[4];
  out[6] = x[6] + d[5];
}

// max_i |x_i - Plus(x, -g)_i| (Ceres' gradient max norm).  Its only use is the test
// gmax <= gradient_tolerance (1e-10): the translation terms are computed exactly as in the
// full expression, so when one of them already exceeds the tolerance the rotation terms
// (two transcendentals) cannot change the outcome and are skipped.
__host__ __device__ inline double lm_gradmax(const double* x, const double* g, int euclid = 0) {
  if (euclid) {
    double m = 0.0;
    for (int c = 0; c < 6; ++c) m = fmax(m, fabs(x[c] - (x[c] + -g[c])));
    return m;
  }
  double mt = 0.0;
  for (int c = 0; c < 3; ++c) mt = fmax(mt, fabs(x[4 + c] - (x[4 + c] + -g[3 + c])));
  if (mt > 1e-10) return mt;
  double ng[6], pg[7];
  for (int c = 0; c < 6; ++c) ng[c] = -g[c];
  lm_plus(x, ng, pg);
  double mx = 0.0;
  for (int i = 0; i < 7; ++i) mx = fmax(mx, fabs(x[i] - pg[i]));
  return mx;
}

__host__ __device__ inline double lm_norm7(const double* x) {
  double s = 0;
  for (int i = 0; i < 7; ++i) s += x[i] * x[i];
  return sqrt(s);
}

// LM step: (S J^T J S + diag(D^2)) y = S J^T r, step = -y.  Returns false if not solvable.
// LDL^T of the 6x6 system: one reciprocal per column on the dependent chain and no square roots
// (a Cholesky took 6 square roots and 27 divisions in sequence, 5.7k cycles on one lane of
// gfx950; this ~2k).  D^2 = diag / radius enters directly (Ceres' D = sqrt(diag / radius)
// appears only squared in the normal equations of [J S; D]).
__host__ __device__ inline bool lm_solve_step(LmState& S, double* step) {
  double A[6][6], b[6];
  for (int i = 0; i < 6; ++i) {
    if (!S.reuse_diag) {
      double d = S.scaling[i] * S.scaling[i] * S.jtj[ut_index(i, i)];
      S.diag[i] = fmin(fmax(d, 1e-6), 1e32);
    }
  }
  const double rinv = 1.0 / S.radius;
  for (int i = 0; i < 6; ++i) {
    for (int j = 0; j <= i; ++j) A[i][j] = S.scaling[i] * S.jtj[ut_index(j, i)] * S.scaling[j];
    A[i][i] += S.diag[i] * rinv;
    b[i] = S.scaling[i] * S.g[i];
  }
  S.reuse_diag = 1;
  // A = L diag(dv) L^T: unit L in the strict lower triangle, w = L[i][j] dv[j] in the upper
  // (A[j][i]) for the rows below
  double rd[6];
  for (int j = 0; j < 6; ++j) {
    double d = A[j][j];
    for (int k = 0; k < j; ++k) d -= A[j][k] * A[k][j];
    if (!(d > 0.0)) return false;
    rd[j] = 1.0 / d;
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i][j];
      for (int k = 0; k < j; ++k) t -= A[i][k] * A[k][j];
      A[j][i] = t;
      A[i][j] = t * rd[j];
    }
  }
  double z[6], y[6];
  for (int i = 0; i < 6; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= A[i][k] * z[k];
    z[i] = t;
  }
  for (int i = 5; i >= 0; --i) {
    double t = z[i] * rd[i];
    for (int k = i + 1; k < 6; ++k) t -= A[k][i] * y[k];
    y[i] = t;
  }
  for (int i = 0; i < 6; ++i) {
    step[i] = -y[i];
    if (!isfinite(step[i])) return false;
  }
  return true;
}

// Consume one reduced pass (red[LM_NACC]) and advance the trust-region state machine until
// it needs another pass (status LM_EVAL_CAND) or terminates (LM_DONE, best in S.best).
__host__ __device__ inline void lm_step(LmState& S, const double* red) {
  if (S.status == LM_DONE) return;
  S.passes++;
  bool step_ok;
  if (S.status == LM_EVAL_X) {
    for (int i = 0; i < 21; ++i) S.jtj[i] = red[i];
    for (int i = 0; i < 6; ++i) S.g[i] = red[21 + i];
    S.cost = red[27];
    S.initial_cost = S.cost;
    if (red[28] == 0.0) {  // no residual blocks: parameters untouched
      S.term = 4;
      S.min_cost = S.cost;
      S.status = LM_DONE;
      return;
    }
    for (int i = 0; i < 6; ++i) S.scaling[i] = 1.0 / (1.0 + sqrt(S.jtj[ut_index(i, i)]));
    S.gmax = lm_gradmax(S.x, S.g, S.euclid);
    S.x_norm = lm_norm7(S.x);
    step_ok = true;
  } else {
    const double cand_cost = red[27];
    const double cost_change = S.cost - cand_cost;
    if (fabs(cost_change) <= 1e-6 * S.cost) {  // FunctionToleranceReached
      S.term = 1;
      S.status = LM_DONE;
      return;
    }
    const double rel = cost_change / S.mcc;
    if (rel > 1e-3) {  // HandleSuccessfulStep
      for (int i = 0; i < 7; ++i) S.x[i] = S.cand[i];
      for (int i = 0; i < 21; ++i) S.jtj[i] = red[i];
      for (int i = 0; i < 6; ++i) S.g[i] = red[21 + i];
      S.cost = cand_cost;
      S.x_norm = lm_norm7(S.x);
      S.gmax = lm_gradmax(S.x, S.g, S.euclid);
      S.successful++;
      double f = 2.0 * rel - 1.0;
      S.radius = S.radius / fmax(1.0 / 3.0, 1.0 - f * f * f);
      S.radius = fmin(1e16, S.radius);
      S.decrease = 2.0;
      S.reuse_diag = 0;
      step_ok = true;
    } else {  // HandleUnsuccessfulStep
      S.radius = S.radius / S.decrease;
      S.decrease *= 2.0;
      S.reuse_diag = 1;
      step_ok = false;
    }
  }
  while (true) {  // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (step_ok && S.cost < S.min_cost) {
      S.min_cost = S.cost;
      for (int i = 0; i < 7; ++i) S.best[i] = S.x[i];
    }
    if (S.iteration >= S.max_iter) { S.term = 0; break; }
    if (step_ok && S.gmax <= 1e-10) { S.term = 3; break; }
    if (S.radius <= 1e-32) { S.term = 5; break; }
    S.iteration++;
    step_ok = false;
    double step[6];
    bool valid = lm_solve_step(S, step);
    if (valid) {
      // model_cost_change = -(step^T S g + 1/2 step^T (S JtJ S) step)
      // (six independent row sums, then one of six: a short dependent chain)
      double v[6], lin = 0, quad = 0;
      for (int i = 0; i < 6; ++i) v[i] = step[i] * S.scaling[i];
      for (int i = 0; i < 6; ++i) {
        double w = 0;
        for (int j = 0; j < 6; ++j) w += S.jtj[ut_index(i < j ? i : j, i < j ? j : i)] * v[j];
        lin += v[i] * S.g[i];
        quad += v[i] * w;
      }
      S.mcc = -(lin + 0.5 * quad);
      valid = S.mcc > 0.0;
    }
    if (!valid) {  // HandleInvalidStep
      S.invalid++;
      if (++S.consec_invalid >= 5) { S.term = 5; break; }
      S.radius = S.radius / S.decrease;
      S.decrease *= 2.0;
      S.reuse_diag = 1;
      continue;
    }
    S.consec_invalid = 0;
    double delta[6];
    for (int i = 0; i < 6; ++i) delta[i] = step[i] * S.scaling[i];
    lm_plus(S.x, delta, S.cand, S.euclid);
    double sn = 0;
    for (int i = 0; i < 7; ++i) sn += (S.x[i] - S.cand[i]) * (S.x[i] - S.cand[i]);
    sn = sqrt(sn);
    if (sn <= 1e-8 * (S.x_norm + 1e-8)) { S.term = 2; break; }  // ParameterToleranceReached
    S.status = LM_EVAL_CAND;
    return;
  }
  S.status = LM_DONE;
}

// ---------------------------------------------------------------------------------------
// LM pass, split in two launches per trust-region iteration:
//   lm_eval_block  (many workgroups per stream)  evaluate every residual block at the state's
//                  evaluation point, grid-stride over the records, one partial
//                  (J^T J, J^T r, cost, rows) per workgroup in a fixed slot;
//   lm_step_wave   (one wave per stream)  sum the partials in a fixed order (lane-strided,
//                  then a shuffle tree: deterministic), run lm_step on lane 0.
// Keeping the trust-region logic out of the evaluation kernel keeps its register budget (and
// occupancy) that of the residual arithmetic alone.
// ---------------------------------------------------------------------------------------
// Block sum of LM_NACC per-thread accumulators -> sum[0 .. LM_NACC) (LDS, valid after the
// trailing barrier; all kThreads threads call it).  The four lanes of each quad combine in
// registers first (DPP quad permutes: lane pairs, then pairs of pairs), a quarter of the rows go
// through an LDS transpose, thread 8a + q sums segment q of accumulator a in row order, and the
// 8 segment sums combine in a fixed butterfly: a fixed summation order.  (29 wave butterflies
// of 6 dependent fp64 shuffles took ~15k cycles per 256-thread block, this ~3k.)
template <int kThreads>
__device__ inline void lm_block_sum(const double* acc, double* sum) {
  static_assert(kThreads % 64 == 0 && LM_NACC * 8 <= kThreads, "transpose reduction layout");
  constexpr int SEG = 8, ROWS = kThreads / 4, PER = ROWS / SEG;
  __shared__ double tr[LM_NACC][ROWS + 1];
  const int tid = threadIdx.x;
  auto dpp_add = [](double v, auto ctrl) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, decltype(ctrl)::value, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), decltype(ctrl)::value, 0xF, 0xF, false);
    return v + __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  };
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) {
    double v = dpp_add(acc[i], std::integral_constant<int, 0xB1>{});  // quad_perm [1, 0, 3, 2]
    v = dpp_add(v, std::integral_constant<int, 0x4E>{});              // quad_perm [2, 3, 0, 1]
    if ((tid & 3) == 0) tr[i][tid >> 2] = v;
  }
  __syncthreads();
  double part = 0.0;
  if (tid < LM_NACC * SEG) {
    const int a = tid / SEG, q = tid % SEG;
#pragma unroll 8
    for (int k = 0; k < PER; ++k) part += tr[a][q * PER + k];
  }
  part += __shfl_xor(part, 4, 64);
  part += __shfl_xor(part, 2, 64);
  part += __shfl_xor(part, 1, 64);
  if (tid < LM_NACC * SEG && (tid % SEG) == 0) sum[tid / SEG] = part;
  __syncthreads();
}

struct LmRecView {
  const int* type;
  const float *px, *py, *pz;
  const double *a0, *a1, *a2, *b0, *b1, *b2;
};

// residual sums of records r = blk*kThreads + tid + k*nblk*kThreads at X; the block total
// is left in sum[LM_NACC] (LDS) for tid < LM_NACC after the trailing barrier.  Two records per
// thread are loaded before either is evaluated, so their loads are in flight together.
template <int kThreads>
__device__ inline void lm_eval_sum(const LmRecView& R, int nrec, const double* X, int blk, int nblk,
                                   double* sum, unsigned long long* prof = nullptr) {
  const int tid = threadIdx.x;
  double acc[LM_NACC];
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) acc[i] = 0.0;
  const int stride = nblk * kThreads;
  // software pipeline: the next two records are loaded while the current two are evaluated
  struct Rec {
    int t;
    float px, py, pz;
    double a0, a1, a2, b0, b1, b2;
  };
  auto load = [&](Rec* q, int r) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = r + u * stride;
      q[u].t = 0;
      if (rr < nrec) {
        q[u].t = R.type[rr];
        q[u].px = R.px[rr]; q[u].py = R.py[rr]; q[u].pz = R.pz[rr];
        q[u].a0 = R.a0[rr]; q[u].a1 = R.a1[rr]; q[u].a2 = R.a2[rr];
        q[u].b0 = R.b0[rr]; q[u].b1 = R.b1[rr]; q[u].b2 = R.b2[rr];
      }
    }
  };
  const unsigned long long tp0 = prof ? __builtin_readcyclecounter() : 0ull;
  double Rm[9];
  lm_rotmat(X, Rm);
  const int r0 = blk * kThreads + tid;
  Rec cur[2], nxt[2];
  load(cur, r0);
  for (int r = r0; r < nrec; r += 2 * stride) {
    load(nxt, r + 2 * stride);
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (cur[u].t != 0)
        lm_accum(cur[u].t, cur[u].px, cur[u].py, cur[u].pz, cur[u].a0, cur[u].a1, cur[u].a2, cur[u].b0, cur[u].b1,
                 cur[u].b2, Rm, X, acc);
#pragma unroll
    for (int u = 0; u < 2; ++u) cur[u] = nxt[u];
  }
  unsigned long long tp1 = 0;
  if (prof) {
    __syncthreads();
    tp1 = __builtin_readcyclecounter();
    if (tid == 0) atomicAdd(&prof[0], tp1 - tp0);
  }
  lm_block_sum<kThreads>(acc, sum);
  if (prof && tid == 0) atomicAdd(&prof[1], __builtin_readcyclecounter() - tp1);
}

template <int kThreads>
__device__ inline void lm_eval_block(const LmRecView& R, int nrec, const LmState& S, int blk,
                                     int nblk, double* partial_out) {
  __shared__ double bsum[LM_NACC];
  const int status = S.status;
  if (status == LM_DONE) return;  // uniform for every workgroup of the stream
  double X[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) X[i] = status == LM_EVAL_X ? S.x[i] : S.cand[i];
  lm_eval_sum<kThreads>(R, nrec, X, blk, nblk, bsum);
  if (threadIdx.x < LM_NACC) partial_out[threadIdx.x] = bsum[threadIdx.x];
}

// one wave: reduce nblk partials, advance the state; returns true (lane 0) if the state
// terminated in this step
__device__ inline bool lm_step_wave(const double* partials, int nblk, LmState& S,
                                    double* best_out = nullptr) {
  const int lane = threadIdx.x & 63;
  if (S.status == LM_DONE) return false;
  __shared__ double sred[LM_NACC];
  // the state is staged in LDS: lm_step is a long dependent chain, and every access to the
  // global copy would pay a memory round trip
  __shared__ LmState ls;
  static_assert(sizeof(LmState) % 8 == 0, "LmState copy granularity");
  constexpr int NW = sizeof(LmState) / 8;
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&S);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(&ls);
  for (int w = lane; w < NW; w += 64) dst[w] = src[w];
  double v[LM_NACC];
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) v[i] = 0.0;
  for (int c = lane; c < nblk; c += 64) {  // all loads of a block row in flight together
#pragma unroll
    for (int i = 0; i < LM_NACC; ++i) v[i] += partials[(size_t)c * LM_NACC + i];
  }
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) {
    const double t = wave_sum_d(v[i]);
    if (lane == 0) sred[i] = t;
  }
  __syncthreads();
  if (lane == 0) {
    LmState L = ls;  // registers for the dependent chain
    lm_step(L, sred);
    ls = L;
  }
  __syncthreads();
  unsigned long long* back = reinterpret_cast<unsigned long long*>(&S);
  for (int w = lane; w < NW; w += 64) back[w] = dst[w];
  const bool done = ls.status == LM_DONE;
  if (done && best_out && lane < 7) best_out[lane] = ls.best[lane];
  return done;
}

// ---------------------------------------------------------------------------------------
// Persistent LM round: all <= 5 passes of one solve in one launch.  The records are cut into
// G fixed shares; the partial sums of share c go to part[c] and the leader (g = 0) adds them in
// share order, so the arithmetic depends on G alone, not on who evaluates a share.  Shares
// are claimed per pass with an atomic ticket by whichever of the stream's workgroups is
// running: the leader keeps claiming until every share is taken, then waits only for shares
// that running workgroups hold.  No workgroup waits for one that may not be resident, so
// handles sharing the GPU cannot deadlock (the leaders are the first blocks of every grid; a
// member that starts after the round ended sees DONE and leaves).  The leader keeps the
// trust-region state in its LDS and runs the step.  Every word handed between workgroups is an
// agent-scope atomic (sc1: written through / read past the XCD's L2): partials are stored so,
// drained, then counted with a relaxed ticket; the eval point is published with sc1 stores +
// drain + a relaxed generation; consumers poll relaxed and read the words with sc1 loads.  No
// fence: on gfx950 an agent-scope release fence writes back the whole L2 of the XCD and an
// acquire invalidates it (buffer_wbl2 / buffer_inv), whatever is dirty or cached from other
// kernels (LM_HANDOFF_FENCES=1 builds the fence recipe of cdna_hip_programming.md §6 Guideline
// 16 instead).  Every spin is bounded (err_code).
// ---------------------------------------------------------------------------------------
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
#ifndef LM_HANDOFF_FENCES
#define LM_HANDOFF_FENCES 0
#endif

__device__ inline void lm_part_store(double* p, double v) {
#if LM_HANDOFF_FENCES
  *p = v;
#else
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v), RLX_AGENT);
#endif
}

__device__ inline double lm_part_load(const double* p) {
#if LM_HANDOFF_FENCES
  return *p;
#else
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), RLX_AGENT));
#endif
}

// the producer side of a hand-off: this thread's stores are complete before what follows
__device__ inline void lm_release() {
#if LM_HANDOFF_FENCES
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the consumer side, after the polled word showed the hand-off
__device__ inline void lm_acquire() {
#if LM_HANDOFF_FENCES
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

#ifndef LM_RED_BATCH
#define LM_RED_BATCH 16  // the leader's partial loads in flight per batch
#endif
constexpr int LM_MAX_PASSES = 8;          // a round needs <= 1 + max_num_iterations = 5
constexpr uint32_t LM_SPIN_LIMIT = 1u << 21;
constexpr uint32_t LM_PEER_SPIN_LIMIT = 1u << 24;  // the cross-rank wait: other ranks' kernels
                                                   // start after their own earlier kernels
// the cross-rank wait's bound as the kernels read it: LOAM_PEER_SPIN_LIMIT (environment, written
// per device when a mapper is created there) lowers it, so that tests can show an exhausted wait
// reaching the caller as LOAM_ERR_SYNC (tests/test_gpu_shard_mp.py)
static __device__ uint32_t lm_peer_spin_limit_g = LM_PEER_SPIN_LIMIT;
static inline void lm_peer_spin_limit_from_env(int device) {
  const char* e = getenv("LOAM_PEER_SPIN_LIMIT");
  if (!e || device < 0 || device >= 64) return;
  static std::mutex mu;
  static uint64_t done = 0;
  std::lock_guard<std::mutex> lk(mu);
  if ((done >> device) & 1ull) return;
  const uint32_t v = (uint32_t)strtoul(e, nullptr, 10);
  if (hipMemcpyToSymbol(HIP_SYMBOL(lm_peer_spin_limit_g), &v, sizeof(v)) == hipSuccess) done |= 1ull << device;
}
// sync words per solve, zeroed before the launch: [1] generation (pass + 1 of the published
// evaluation point; past LM_MAX_PASSES once the round has ended), [4 + p] claims of pass p's
// shares 1.. (share 0 is the leader's), [4 + LM_MAX_PASSES + p] shares 1.. of pass p completed
constexpr int LM_SYNC_WORDS = 4 + 2 * LM_MAX_PASSES;

// the polled word once it reaches target (>= 1), or 0 when the wait runs out
__device__ inline uint32_t lm_spin_val(uint32_t* w, uint32_t target, uint32_t limit = LM_SPIN_LIMIT) {
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t v = __hip_atomic_load(w, RLX_AGENT);
    if (v >= target) return v;
    if (spins >= limit) return 0u;
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ inline bool lm_spin_ge(uint32_t* w, uint32_t target, uint32_t limit = LM_SPIN_LIMIT) {
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(w, RLX_AGENT) >= target) return true;
    if (spins >= limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// the cross-process exchange (LmJob::ipc): peer buffers another process (perhaps another GPU over
// xGMI) reads, so every access is a system-scope atomic (written through / read past every cache
// on the way), data and flags alike, in either build
#define RLX_SYS __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM
__device__ inline void lm_sys_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v), RLX_SYS);
}
__device__ inline double lm_sys_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), RLX_SYS));
}
__device__ inline bool lm_spin_ge_sys(uint32_t* w, uint32_t target, uint32_t limit) {
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(w, RLX_SYS) >= target) return true;
    if (spins >= limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// streams padded to a multiple of the 8 XCDs: block g * Bp + s of a persistent LM launch runs
// on XCD s % 8 for every member g (workgroups are dealt to the XCDs round-robin)
__host__ __device__ inline int lm_padded(int B) { return (B + 7) & ~7; }

// one LM solve (one outer round of one stream) spread over G workgroups
struct LmJob {
  LmState* S;         // state, initialised by lm_init in an earlier launch
  LmRecView R;        // factor records
  int nrec;
  double* part;       // [G][LM_NACC] share partials
  uint32_t* sync;     // [LM_SYNC_WORDS] zeroed in an earlier launch
  double* xpub;       // [8] published evaluation point
  double* best_out;   // [7] pose written when the solve terminates
  int* err;
  int err_code;
  unsigned long long* prof = nullptr;  // optional cycles: [0] leader eval, [1] leader wait,
                                       // [2] reduce + step, [3] passes, [4] member wait for x
  // one solve sharded over nrank ranks whose kernels run at once (loam_comm_create_local): this
  // rank evaluates shares rank * G .. of nrank * G; per pass its leader stores the rank's sums in
  // its slot of peer ([nrank][LM_MAX_PASSES][LM_NACC], shared by the ranks), raises its flag
  // peer_flag[rank] to flag_base + pass + 1 and, once every rank's flag is there, sums the slots
  // in rank order: the same bits, hence the same step, on every rank
  int rank = 0, nrank = 1;
  double* peer = nullptr;
  uint32_t* peer_flag = nullptr;
  uint32_t flag_base = 0;
  // ranks in separate processes (loam_comm kinds 0 / 1, each rank's launch on its own stream): each
  // rank owns a buffer the others map through IPC handles; ipc[r] is rank r's slot base (double*),
  // ipc[nrank + r] its flag base (uint32_t*), as this process maps them; this solve's slots start
  // ipc_slot_off doubles in ([LM_MAX_PASSES][LM_NACC]), its flag ipc_flag_off words in
  const unsigned long long* ipc = nullptr;
  size_t ipc_slot_off = 0, ipc_flag_off = 0;
};

// share c of pass `pass` at X -> part[c], then counted complete (release)
template <int kThreads>
__device__ inline void lm_share(const LmJob& J, const double* X, int c, int G, int pass, double* bsum) {
  const int tid = threadIdx.x;
  lm_eval_sum<kThreads>(J.R, J.nrec, X, J.rank * G + c, J.nrank * G, bsum);
  if (tid < LM_NACC) lm_part_store(&J.part[(size_t)c * LM_NACC + tid], bsum[tid]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    lm_release();
    __hip_atomic_fetch_add(&J.sync[4 + LM_MAX_PASSES + pass], 1u, RLX_AGENT);
  }
}

template <int kThreads>
__device__ inline void lm_round_device(const LmJob& J, int g, int G) {
  __shared__ LmState ls;
  __shared__ double sx[7];
  __shared__ double bsum[LM_NACC];
  __shared__ double bsum0[LM_NACC];  // the leader's share 0, kept in LDS
  __shared__ double sred[LM_NACC];
  __shared__ int sstat, sshare, spass;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  LmState& S = *J.S;
  uint32_t* sync = J.sync;
  double* xpub = J.xpub;
  const double* part = J.part;
  unsigned long long t0 = 0;
  if (g != 0) {  // member: join the pass in progress, evaluate the shares it can claim
    uint32_t want = 1;
    while (true) {
      if (tid == 0) {
        t0 = __builtin_readcyclecounter();
        int st = LM_DONE, c = G, p = 0;
        // the generation as polled (0: the wait ran out, a member that waits too long just
        // leaves); above LM_MAX_PASSES the round has ended
        const uint32_t gen = lm_spin_val(&sync[1], want);
        if (gen != 0u && gen <= (uint32_t)LM_MAX_PASSES) {
          lm_acquire();
          p = (int)gen - 1;
          // the point's loads and the claim in flight together (one memory round trip): they are
          // issued after the generation was seen, so the point is at least pass p's, and a claimed
          // share holds the leader in pass p, so it is not yet a later one; with no share left
          // the values are not used
          double xv[7];
#pragma unroll
          for (int i = 0; i < 7; ++i) xv[i] = __hip_atomic_load(&xpub[i], RLX_AGENT);
          c = 1 + (int)__hip_atomic_fetch_add(&sync[4 + p], 1u, RLX_AGENT);
          if (c < G)
            for (int i = 0; i < 7; ++i) sx[i] = xv[i];
          st = LM_EVAL_CAND;  // (any status but LM_DONE)
        }
        sstat = st;
        sshare = c;
        spass = p;
        if (J.prof) atomicAdd(&J.prof[4], __builtin_readcyclecounter() - t0);
      }
      __syncthreads();
      // LDS broadcasts read as scalars: the branches around barriers must be uniform to the
      // compiler (a divergent loop here is structured so that some lanes never leave it)
      if (__builtin_amdgcn_readfirstlane(sstat) == LM_DONE) return;
      const int c = __builtin_amdgcn_readfirstlane(sshare), p = __builtin_amdgcn_readfirstlane(spass);
      if (c >= G) {  // pass p fully claimed: wait for the next evaluation point
        want = (uint32_t)p + 2;
        __syncthreads();
        continue;
      }
      double X[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) X[i] = sx[i];
      lm_share<kThreads>(J, X, c, G, p, bsum);
      want = (uint32_t)p + 1;  // more shares of pass p, if any are left
      __syncthreads();
    }
  }
  {  // leader: state written by an earlier launch, plain loads
    constexpr int NW = sizeof(LmState) / 8;
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&S);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(&ls);
    for (int w = tid; w < NW; w += kThreads) dst[w] = src[w];
  }
  __syncthreads();
  bool aborted = false;
  for (int pass = 0; pass < LM_MAX_PASSES; ++pass) {
    // ---- evaluation point of this pass
    if (tid == 0) {
      sstat = ls.status;
      for (int i = 0; i < 7; ++i) sx[i] = ls.status == LM_EVAL_X ? ls.x[i] : ls.cand[i];
    }
    __syncthreads();
    if (G > 1 && wid == 0) {  // publish: sc1 stores, drain, relaxed generation (pass + 1, or
                              // past LM_MAX_PASSES when the round has ended: the members leave)
      if (lane < 7) __hip_atomic_store(&xpub[lane], sx[lane], RLX_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_store(&sync[1], sstat == LM_DONE ? (uint32_t)LM_MAX_PASSES + 1u : (uint32_t)(pass + 1), RLX_AGENT);
    }
    if (__builtin_amdgcn_readfirstlane(sstat) == LM_DONE) break;
    if (tid == 0) t0 = __builtin_readcyclecounter();
    double X[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) X[i] = sx[i];
    // ---- share 0, then the shares nobody else took.  Structure (member loop too): every
    // thread-0 region is bracketed by barriers, and every branch that skips a barrier tests an
    // LDS word written in such a region and read through readfirstlane, so the control flow
    // around barriers is uniform whatever the compiler does with the regions.  A share's
    // completion (release) and the next claim are one thread-0 region.
    lm_eval_sum<kThreads>(J.R, J.nrec, X, J.rank * G, J.nrank * G, bsum0, J.prof ? J.prof + 5 : nullptr);
    if (G > 1) {
      if (tid == 0) sshare = 1 + (int)__hip_atomic_fetch_add(&sync[4 + pass], 1u, RLX_AGENT);
      __syncthreads();
      while (true) {
        const int c = __builtin_amdgcn_readfirstlane(sshare);
        if (c >= G) break;
        lm_eval_sum<kThreads>(J.R, J.nrec, X, J.rank * G + c, J.nrank * G, bsum);
        if (tid < LM_NACC) lm_part_store(&J.part[(size_t)c * LM_NACC + tid], bsum[tid]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every thread has read sshare and stored its part
        if (tid == 0) {
          lm_release();
          __hip_atomic_fetch_add(&sync[4 + LM_MAX_PASSES + pass], 1u, RLX_AGENT);
          sshare = 1 + (int)__hip_atomic_fetch_add(&sync[4 + pass], 1u, RLX_AGENT);
        }
        __syncthreads();
      }
    }
    if (tid == 0 && J.prof) {
      const unsigned long long t1 = __builtin_readcyclecounter();
      atomicAdd(&J.prof[0], t1 - t0);
      atomicAdd(&J.prof[3], 1ull);
      t0 = t1;
    }
    // ---- every share complete (the others are held by running workgroups)
    if (tid == 0 && G > 1) {
      if (lm_spin_ge(&sync[4 + LM_MAX_PASSES + pass], (uint32_t)(G - 1))) {
        lm_acquire();
      } else {
        atomicOr(J.err, J.err_code);
        sstat = -1;
      }
    }
    if (tid == 0 && J.prof) {
      const unsigned long long t1 = __builtin_readcyclecounter();
      atomicAdd(&J.prof[1], t1 - t0);
      t0 = t1;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(sstat) == -1) {
      aborted = true;
      break;
    }
    if (wid == 0) {
      // lane i sums accumulator i over the shares in order (G <= 32: one lane per
      // accumulator beats a shuffle tree per accumulator)
      if (lane < LM_NACC) {  // loads LM_RED_BATCH at a time in flight (one batch up to G = 17),
                             // added in share order
        double v = bsum0[lane];
        for (int c = 1; c < G; c += LM_RED_BATCH) {
          double q[LM_RED_BATCH];
#pragma unroll
          for (int u = 0; u < LM_RED_BATCH; ++u)
            q[u] = c + u < G ? lm_part_load(&part[(size_t)(c + u) * LM_NACC + lane]) : 0.0;
#pragma unroll
          for (int u = 0; u < LM_RED_BATCH; ++u)
            if (c + u < G) v += q[u];
        }
        sred[lane] = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (J.nrank > 1 && J.ipc) {  // ranks of other processes: their IPC-mapped buffers
        const uint32_t want = J.flag_base + (uint32_t)pass + 1u;
        const size_t so = J.ipc_slot_off + (size_t)pass * LM_NACC;
        double* mine = reinterpret_cast<double*>(J.ipc[J.rank]) + so;
        if (lane < LM_NACC) lm_sys_store(&mine[lane], sred[lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
#if LM_HANDOFF_FENCES
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the memory model's recipe
#endif
          __hip_atomic_store(reinterpret_cast<uint32_t*>(J.ipc[J.nrank + J.rank]) + J.ipc_flag_off, want, RLX_SYS);
        }
        const bool ok = lane >= J.nrank ||
                        lm_spin_ge_sys(reinterpret_cast<uint32_t*>(J.ipc[J.nrank + lane]) + J.ipc_flag_off, want,
                                       lm_peer_spin_limit_g);
        if (__ballot(!ok) != 0ull) {
          if (lane == 0) {
            atomicOr(J.err, J.err_code);
            sstat = -1;
          }
        } else if (lane < LM_NACC) {
#if LM_HANDOFF_FENCES
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
          double v = lm_sys_load(reinterpret_cast<const double*>(J.ipc[0]) + so + lane);
          for (int r = 1; r < J.nrank; ++r) v += lm_sys_load(reinterpret_cast<const double*>(J.ipc[r]) + so + lane);
          sred[lane] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else if (J.nrank > 1) {  // this rank's sums to its slot, then every rank's, in rank order
        const uint32_t want = J.flag_base + (uint32_t)pass + 1u;
        double* mine = J.peer + ((size_t)J.rank * LM_MAX_PASSES + pass) * LM_NACC;
        if (lane < LM_NACC) lm_part_store(&mine[lane], sred[lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          lm_release();
          __hip_atomic_store(&J.peer_flag[J.rank], want, RLX_AGENT);
        }
        const bool ok = lane >= J.nrank || lm_spin_ge(&J.peer_flag[lane], want, lm_peer_spin_limit_g);
        if (__ballot(!ok) != 0ull) {  // a rank did not come: this rank's LM stops here
          if (lane == 0) {
            atomicOr(J.err, J.err_code);
            sstat = -1;
          }
        } else {
          lm_acquire();
          if (lane < LM_NACC) {
            double v = lm_part_load(&J.peer[(size_t)pass * LM_NACC + lane]);
            for (int r = 1; r < J.nrank; ++r) v += lm_part_load(&J.peer[((size_t)r * LM_MAX_PASSES + pass) * LM_NACC + lane]);
            sred[lane] = v;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      if (lane == 0 && __builtin_amdgcn_readfirstlane(sstat) != -1) {
        const unsigned long long ts = J.prof ? __builtin_readcyclecounter() : 0ull;
        // the step works on the LDS state in place: a register copy of the whole state (~140
        // VGPRs) spilled into AGPRs beside the solve's temporaries (tools/mb_lmstep2.hip: 5.7k ->
        // 4.8k cycles per step; in the kernel 7.4k against 9.9k for a copy of the fields a step
        // touches, taken once and written back once, profiles/r6_lm_step_regs.txt)
        lm_step(ls, sred);
        if (J.prof) atomicAdd(&J.prof[-2], __builtin_readcyclecounter() - ts);  // [15]: the step alone
      }
    }
    __syncthreads();
    if (tid == 0 && J.prof) atomicAdd(&J.prof[2], __builtin_readcyclecounter() - t0);
    if (__builtin_amdgcn_readfirstlane(sstat) == -1) {  // (the cross-rank wait ran out)
      aborted = true;
      break;
    }
  }
  if (aborted && tid == 0) {  // stop this stream's LM where it is (best so far)
    ls.term = 6;
    ls.status = LM_DONE;
    if (G > 1)  // members waiting for a next pass leave now
      __hip_atomic_store(&sync[1], (uint32_t)LM_MAX_PASSES + 1u, RLX_AGENT);
  }
  __syncthreads();
  if (ls.status == LM_DONE && tid < 7 && J.best_out) J.best_out[tid] = ls.best[tid];
  constexpr int NW = sizeof(LmState) / 8;
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&ls);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(&S);
  for (int w = tid; w < NW; w += kThreads) dst[w] = src[w];
}


}  // namespace loam
