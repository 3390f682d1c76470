// Microbenchmark: cycles of the LM trust-region step on one lane (lm_step and its parts), the
// serial tail of every pass of k_lm_round.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Ivloam-noted_amd/csrc \
//   tools/mb_lmstep.hip -o gpurun_out/mb_lmstep
#include <hip/hip_runtime.h>

#include <cstdio>

#include "lm.h"

using namespace loam;


// the previous solve (Cholesky + divisions), for the numerical comparison only
__device__ bool solve_ref(LmState S, double* step) {
  double A[6][6], b[6];
  for (int i = 0; i < 6; ++i) {
    for (int j = 0; j < 6; ++j) {
      int r = i < j ? i : j, c = i < j ? j : i;
      A[i][j] = S.scaling[i] * S.jtj[ut_index(r, c)] * S.scaling[j];
    }
    double D = sqrt(S.diag[i] / S.radius);
    A[i][i] += D * D;
    b[i] = S.scaling[i] * S.g[i];
  }
  for (int j = 0; j < 6; ++j) {
    double s = A[j][j];
    for (int k = 0; k < j; ++k) s -= A[j][k] * A[j][k];
    if (!(s > 0.0)) return false;
    double d = sqrt(s);
    A[j][j] = d;
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i][j];
      for (int k = 0; k < j; ++k) t -= A[i][k] * A[j][k];
      A[i][j] = t / d;
    }
  }
  double z[6], y[6];
  for (int i = 0; i < 6; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= A[i][k] * z[k];
    z[i] = t / A[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double t = z[i];
    for (int k = i + 1; k < 6; ++k) t -= A[k][i] * y[k];
    y[i] = t / A[i][i];
  }
  for (int i = 0; i < 6; ++i) step[i] = -y[i];
  return true;
}

struct Out {
  unsigned long long cyc[8];
  unsigned long long rt[8];
  double step_new[6], step_ref[6];
  double sink;
};

__global__ void k_mb(const double* red0, Out* out) {
  if (threadIdx.x != 0) return;
  __shared__ LmState ls;
  double x7[7] = {0.01, -0.02, 0.03, 0.999, 12.0, -3.0, 0.5};
  double nrm = sqrt(x7[0] * x7[0] + x7[1] * x7[1] + x7[2] * x7[2] + x7[3] * x7[3]);
  for (int i = 0; i < 4; ++i) x7[i] /= nrm;
  LmState S;
  lm_init(S, x7, 4, true);
  double red[LM_NACC];
  for (int i = 0; i < LM_NACC; ++i) red[i] = red0[i];
  double sink = 0;
  // [0] first step (EVAL_X), [1..3] candidate steps, successful / unsuccessful alternately
  for (int k = 0; k < 4; ++k) {
    const unsigned long long t0 = __builtin_readcyclecounter();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    ls = S;
    LmState L = ls;
    lm_step(L, red);
    ls = L;
    S = ls;
    const unsigned long long t1 = __builtin_readcyclecounter();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out->cyc[k] = t1 - t0;
    out->rt[k] = r1 - r0;
    sink += S.cand[0] + S.radius;
    red[27] = k & 1 ? red[27] * 1.5 : red[27] * 0.5;  // success, then failure, ...
    if (S.status == LM_DONE) lm_init(S, x7, 4, true);
  }
  // [4] lm_solve_step alone, [5] lm_plus alone, [6] lm_gradmax (rotation branch), [7] LDS
  // state copy in + out (as lm_round_device does)
  {
    double step[6];
    const unsigned long long t0 = __builtin_readcyclecounter();
    S.reuse_diag = 0;
    bool ok = lm_solve_step(S, step);
    const unsigned long long t1 = __builtin_readcyclecounter();
    out->cyc[4] = t1 - t0;
    double sr[6];
    solve_ref(S, sr);
    for (int i = 0; i < 6; ++i) {
      out->step_new[i] = step[i];
      out->step_ref[i] = sr[i];
    }
    sink += ok ? step[0] : 0.0;
    double c[7];
    const unsigned long long t2 = __builtin_readcyclecounter();
    lm_plus(S.x, step, c);
    const unsigned long long t3 = __builtin_readcyclecounter();
    out->cyc[5] = t3 - t2;
    sink += c[1];
    double g[6] = {1e-12, 2e-12, 3e-12, 1e-13, 1e-13, 1e-13};
    const unsigned long long t4 = __builtin_readcyclecounter();
    double gm = lm_gradmax(S.x, g);
    const unsigned long long t5 = __builtin_readcyclecounter();
    out->cyc[6] = t5 - t4;
    sink += gm;
    ls = S;
    const unsigned long long t6 = __builtin_readcyclecounter();
    LmState L = ls;
    L.radius += 1.0;
    ls = L;
    const unsigned long long t7 = __builtin_readcyclecounter();
    out->cyc[7] = t7 - t6;
    sink += ls.radius;
  }
  out->sink = sink;
}

int main() {
  // a well-conditioned 6x6 J^T J of the magnitude of a mapping pass (~5k rows)
  double h[LM_NACC];
  const double M[6] = {9000, 8000, 7000, 3000, 2500, 5000};
  int k = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) h[k++] = a == b ? M[a] : 0.05 * (a + 1) * (b + 2) * 10;
  for (int a = 0; a < 6; ++a) h[21 + a] = 3.0 * (a - 2.5);
  h[27] = 40.0;
  h[28] = 5000;
  double* dred;
  Out* dout;
  hipMalloc(&dred, sizeof(h));
  hipMalloc(&dout, sizeof(Out));
  hipMemcpy(dred, h, sizeof(h), hipMemcpyHostToDevice);
  Out o{};
  for (int rep = 0; rep < 3; ++rep) {
    k_mb<<<1, 64>>>(dred, dout);
    hipMemcpy(&o, dout, sizeof(Out), hipMemcpyDeviceToHost);
  }
  const char* names[8] = {"lm_step EVAL_X", "lm_step cand (success)", "lm_step cand (fail)", "lm_step cand (success)",
                          "lm_solve_step", "lm_plus", "lm_gradmax (rotation)", "LDS state copy in/out"};
  for (int i = 0; i < 8; ++i)
    std::printf("%-26s %8llu cycles%s", names[i], o.cyc[i], i < 4 ? "" : "\n"), i < 4 ? std::printf("  %6.2f us\n", o.rt[i] / 100.0) : 0;
  for (int i = 0; i < 6; ++i)
    std::printf("step[%d] LDL %.17g Cholesky %.17g rel %.2e\n", i, o.step_new[i], o.step_ref[i],
                (o.step_new[i] - o.step_ref[i]) / o.step_ref[i]);
  std::printf("sink %g\n", o.sink);
  return 0;
}
