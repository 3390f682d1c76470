// vo.hip — visual-odometry pose solve on MI355X.
//
// Reference: VisualOdometry::solveNlsAll (src/visual_odometry/src/visual_odometry.cpp:304-509):
// one residual block per feature match, CostFunctor32 (3D-2D, the previous point has a depth
// from queryDepth) or CostFunctor22 (2D-2D epipolar) of ceres_cost_function.h:58-189, on the
// parameter blocks angles_0to1 (angle-axis) and t_0to1, HuberLoss(0.1), Ceres TR-LM with
// DENSE_QR and max_num_iterations = 100 (visual_odometry.cpp:70-74), no parameterization.
//
// Device form: the same Ceres trust-region state machine as the LiDAR stages (lm.h) with
// Euclidean parameters, and analytic Jacobians in place of the Jets:
//   P = R(w) X + t, R(w) = exp([w]x) (ceres::AngleAxisRotatePoint, same Rodrigues value
//   formula, first-order branch below epsilon), dP/dw = -[R X]x A with A = R(w) J_r(w) per pass
//   (J_r the right Jacobian of SO(3); A = I in the first-order branch, where dP/dw = -[X]x).
//   type 4 (CostFunctor32): r = (P.x - P.z x1, P.y - P.z y1)
//   type 5 (CostFunctor22): r = X1 . (t x q), q = R(w) X0: dr/dt = (q x X1)^T,
//                           dr/dw = (X1 x t)^T dq/dw
// One workgroup per problem runs all passes (evaluation -> block reduction -> step on one
// lane), so a batch of B problems is one launch with no host round trip.
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.h"
#include "lm.h"

namespace loam {

constexpr int VO_THREADS = 256;
constexpr int VO_MAX_PASSES = 256;  // >= max_num_iterations + 1 (invalid steps need no pass)

struct VoRot {
  double w[3];         // the rotation as Ceres' value path: unit axis, cos, sin, or first order
  double cs, sn;
  int small;           // theta^2 <= DBL_EPSILON: result = p + w x p
  double A[9];         // R(w) J_r(w) (identity in the first-order branch)
};

__device__ inline void vo_rot(const double* x, VoRot& V) {
  const double th2 = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
  V.small = !(th2 > 2.220446049250313e-16);
  if (V.small) {
    for (int i = 0; i < 3; ++i) V.w[i] = x[i];
    V.cs = 1.0;
    V.sn = 0.0;
    for (int i = 0; i < 9; ++i) V.A[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double th = sqrt(th2), ti = 1.0 / th;
  sincos(th, &V.sn, &V.cs);
  for (int i = 0; i < 3; ++i) V.w[i] = x[i] * ti;
  // R = cos I + sin [u]x + (1 - cos) u u^T ; J_r = I - a [x]x + b [x]x^2 with
  // a = (1 - cos) / th^2, b = (th - sin) / th^3 (series below 1e-4)
  const double* u = V.w;
  double R[9];
  const double c1 = 1.0 - V.cs;
  R[0] = V.cs + c1 * u[0] * u[0];        R[1] = c1 * u[0] * u[1] - V.sn * u[2]; R[2] = c1 * u[0] * u[2] + V.sn * u[1];
  R[3] = c1 * u[1] * u[0] + V.sn * u[2]; R[4] = V.cs + c1 * u[1] * u[1];        R[5] = c1 * u[1] * u[2] - V.sn * u[0];
  R[6] = c1 * u[2] * u[0] - V.sn * u[1]; R[7] = c1 * u[2] * u[1] + V.sn * u[0]; R[8] = V.cs + c1 * u[2] * u[2];
  double a, b;
  if (th < 1e-4) {
    a = 0.5 - th2 / 24.0;
    b = 1.0 / 6.0 - th2 / 120.0;
  } else {
    a = c1 / th2;
    b = (th - V.sn) / (th2 * th);
  }
  const double K[9] = {0, -x[2], x[1], x[2], 0, -x[0], -x[1], x[0], 0};
  double K2[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) K2[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  double Jr[9];
  for (int i = 0; i < 9; ++i) Jr[i] = ((i % 4 == 0) ? 1.0 : 0.0) - a * K[i] + b * K2[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) V.A[3 * i + j] = R[3 * i] * Jr[j] + R[3 * i + 1] * Jr[3 + j] + R[3 * i + 2] * Jr[6 + j];
}

// ceres::AngleAxisRotatePoint value (rotation.h)
__device__ inline void vo_rotate(const VoRot& V, const double p[3], double out[3]) {
  const double* w = V.w;
  const double wc[3] = {w[1] * p[2] - w[2] * p[1], w[2] * p[0] - w[0] * p[2], w[0] * p[1] - w[1] * p[0]};
  if (V.small) {
    for (int i = 0; i < 3; ++i) out[i] = p[i] + wc[i];
    return;
  }
  const double tmp = ((w[0] * p[0] + w[1] * p[1]) + w[2] * p[2]) * (1.0 - V.cs);
  for (int i = 0; i < 3; ++i) out[i] = (p[i] * V.cs + wc[i] * V.sn) + w[i] * tmp;
}

// dP/dw = -[v]x A (v = R X, or X in the first-order branch)
__device__ inline void vo_dpdw(const VoRot& V, const double v[3], double D[9]) {
  const double K[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      D[3 * i + j] = -(K[3 * i] * V.A[j] + K[3 * i + 1] * V.A[3 + j] + K[3 * i + 2] * V.A[6 + j]);
}

__device__ inline void vo_accum(int type, const double* rec, const VoRot& V, const double* x, double* acc) {
  double r[2], J[2][6];
  int m;
  if (type == 4) {  // CostFunctor32
    const double X0[3] = {rec[1], rec[2], rec[3]};
    double q[3];
    vo_rotate(V, X0, q);
    const double P[3] = {q[0] + x[3], q[1] + x[4], q[2] + x[5]};
    const double x1 = rec[4], y1 = rec[5];
    r[0] = P[0] - P[2] * x1;
    r[1] = P[1] - P[2] * y1;
    double D[9];
    vo_dpdw(V, V.small ? X0 : q, D);
    for (int c = 0; c < 3; ++c) {
      J[0][c] = D[c] - x1 * D[6 + c];
      J[1][c] = D[3 + c] - y1 * D[6 + c];
    }
    J[0][3] = 1.0; J[0][4] = 0.0; J[0][5] = -x1;
    J[1][3] = 0.0; J[1][4] = 1.0; J[1][5] = -y1;
    m = 2;
  } else {  // CostFunctor22
    const double X0[3] = {rec[4], rec[5], 1.0}, X1[3] = {rec[7], rec[8], 1.0};
    const double* t = x + 3;
    double q[3];
    vo_rotate(V, X0, q);
    const double c[3] = {t[1] * q[2] - t[2] * q[1], t[2] * q[0] - t[0] * q[2], t[0] * q[1] - t[1] * q[0]};
    r[0] = (X1[0] * c[0] + X1[1] * c[1]) + X1[2] * c[2];
    const double g[3] = {X1[1] * t[2] - X1[2] * t[1], X1[2] * t[0] - X1[0] * t[2], X1[0] * t[1] - X1[1] * t[0]};
    double D[9];
    vo_dpdw(V, V.small ? X0 : q, D);
    for (int k = 0; k < 3; ++k) J[0][k] = g[0] * D[k] + g[1] * D[3 + k] + g[2] * D[6 + k];
    J[0][3] = q[1] * X1[2] - q[2] * X1[1];
    J[0][4] = q[2] * X1[0] - q[0] * X1[2];
    J[0][5] = q[0] * X1[1] - q[1] * X1[0];
    m = 1;
  }
  double s = 0.0;
  for (int i = 0; i < m; ++i) s += r[i] * r[i];
  double rho0, rho1;  // HuberLoss(0.1) + Corrector (lm.h)
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
  for (int i = 0; i < m; ++i) {
    int k = 0;
    for (int a = 0; a < 6; ++a) {
      const double wa = rho1 * J[i][a];
      for (int b = a; b < 6; ++b) acc[k++] += wa * J[i][b];
      acc[21 + a] += wa * r[i];
    }
  }
}

// one workgroup per problem: every pass of the solve
__global__ void __launch_bounds__(VO_THREADS) k_vo_solve(const double* factors, const int* off, double* xs,
                                                          int max_iter, LmState* states) {
  __shared__ LmState S;
  __shared__ double sum[LM_NACC];
  __shared__ double X[7];
  const int p = blockIdx.x, tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r0 = off[p], nrec = off[p + 1] - r0;
  const double* F = factors + (size_t)r0 * 10;
  if (tid == 0) {
    double x7[7] = {xs[6 * p], xs[6 * p + 1], xs[6 * p + 2], xs[6 * p + 3], xs[6 * p + 4], xs[6 * p + 5], 0.0};
    lm_init(S, x7, max_iter, true);
    S.euclid = 1;
  }
  __syncthreads();
  for (int pass = 0; pass < VO_MAX_PASSES && S.status != LM_DONE; ++pass) {
    if (tid < 7) X[tid] = S.status == LM_EVAL_X ? S.x[tid] : S.cand[tid];
    __syncthreads();
    double x[7];
    for (int i = 0; i < 7; ++i) x[i] = X[i];
    VoRot V;
    vo_rot(x, V);
    double acc[LM_NACC];
    for (int i = 0; i < LM_NACC; ++i) acc[i] = 0.0;
    for (int i = tid; i < nrec; i += VO_THREADS) {
      const double* rec = F + (size_t)i * 10;
      const int type = (int)rec[0];
      if (type == 4 || type == 5) vo_accum(type, rec, V, x, acc);
    }
    lm_block_sum<VO_THREADS>(acc, sum);
    if (tid == 0) {
      LmState L = S;
      lm_step(L, sum);
      S = L;
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (S.status != LM_DONE) S.term = 5;  // pass budget exhausted (not reached with <= 100 iterations)
    for (int i = 0; i < 6; ++i) xs[6 * p + i] = S.best[i];
    states[p] = S;
  }
}

}  // namespace loam

using namespace loam;

extern "C" {

int32_t loam_vo_solve(int32_t device, int32_t n_problems, const int32_t* offsets, const double* factors,
                      double* x, int32_t max_iterations, loam_lm_stats* st) {
  if (n_problems < 0 || (n_problems > 0 && (!offsets || !x)) || max_iterations < 0 ||
      max_iterations > VO_MAX_PASSES - 1) {
    set_error("loam_vo_solve: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (n_problems == 0) return LOAM_OK;
  for (int p = 0; p < n_problems; ++p)
    if (offsets[p + 1] < offsets[p] || offsets[0] != 0) {
      set_error("loam_vo_solve: offsets must start at 0 and not decrease");
      return LOAM_ERR_ARG;
    }
  const int nf = offsets[n_problems];
  if (nf > 0 && !factors) return LOAM_ERR_ARG;
  TRY(ensure_device(device));
  LOAM_HIP(hipSetDevice(device));
  double* d_f = nullptr;
  double* d_x = nullptr;
  int* d_off = nullptr;
  LmState* d_s = nullptr;
  auto cleanup = [&]() {
    if (d_f) (void)hipFree(d_f);
    if (d_x) (void)hipFree(d_x);
    if (d_off) (void)hipFree(d_off);
    if (d_s) (void)hipFree(d_s);
  };
  hipError_t e = hipMalloc(&d_f, sizeof(double) * 10 * std::max(nf, 1));
  if (e == hipSuccess) e = hipMalloc(&d_x, sizeof(double) * 6 * n_problems);
  if (e == hipSuccess) e = hipMalloc(&d_off, sizeof(int) * (n_problems + 1));
  if (e == hipSuccess) e = hipMalloc(&d_s, sizeof(LmState) * n_problems);
  if (e == hipSuccess && nf) e = hipMemcpy(d_f, factors, sizeof(double) * 10 * nf, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_x, x, sizeof(double) * 6 * n_problems, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_off, offsets, sizeof(int) * (n_problems + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    k_vo_solve<<<n_problems, VO_THREADS>>>(d_f, d_off, d_x, max_iterations, d_s);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(x, d_x, sizeof(double) * 6 * n_problems, hipMemcpyDeviceToHost);
  std::vector<LmState> hs(n_problems);
  if (e == hipSuccess) e = hipMemcpy(hs.data(), d_s, sizeof(LmState) * n_problems, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) {
    set_error(std::string("loam_vo_solve: ") + hipGetErrorString(e));
    return LOAM_ERR_HIP;
  }
  if (st)
    for (int p = 0; p < n_problems; ++p) {
      st[p].iterations = hs[p].iteration;
      st[p].successful = hs[p].successful;
      st[p].invalid = hs[p].invalid;
      st[p].termination = hs[p].term;
      st[p].initial_cost = hs[p].initial_cost;
      st[p].final_cost = hs[p].min_cost;
    }
  return LOAM_OK;
}

}  // extern "C"
