// Microbenchmark: what one lane's LM trust-region step (lm.h lm_step, the serial tail of every
// pass of k_lm_round) spends its cycles on.  Each piece runs R times in a dependent loop on lane 0
// (the next input depends on the last output), timed with s_memrealtime (100 MHz) and the cycle
// counter; printed per call.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Ivloam-noted_amd/csrc tools/mb_lmstep2.hip -o tools/bin/mb_lmstep2
#include <hip/hip_runtime.h>

#include <cstdio>

#include "lm.h"

using namespace loam;

constexpr int R = 512;

struct Out {
  unsigned long long cyc[10], rt[10];
  double sink;
};

__device__ __noinline__ void keep(double* s, double v) { *s += v; }

__global__ void k_mb(const double* red0, Out* out) {
  if (threadIdx.x != 0) return;
  __shared__ LmState ls;
  double sink = 0;
  double x7[7] = {0.01, -0.02, 0.03, 0.999, 12.0, -3.0, 0.5};
  double nrm = sqrt(x7[0] * x7[0] + x7[1] * x7[1] + x7[2] * x7[2] + x7[3] * x7[3]);
  for (int i = 0; i < 4; ++i) x7[i] /= nrm;
  double red[LM_NACC];
  for (int i = 0; i < LM_NACC; ++i) red[i] = red0[i];
  int slot = 0;
  auto t = [&](int k, unsigned long long c0, unsigned long long r0) {
    out->cyc[k] = (__builtin_readcyclecounter() - c0) / R;
    out->rt[k] = (__builtin_amdgcn_s_memrealtime() - r0);
  };
  // [0] lm_step over passes (EVAL_X, then candidates alternately accepted / rejected), state in
  // registers
  {
    LmState S;
    lm_init(S, x7, 1 << 30, true);
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      red[27] = (it & 1) ? red[27] * 0.25 : red[27] * 3.0;
      lm_step(S, red);
      if (S.status == LM_DONE) lm_init(S, S.x, 1 << 30, true);
    }
    t(slot++, c0, r0);
    sink += S.x[0] + S.radius;
  }
  // [1] the same with the state staged in LDS (copy in, step, copy out: as k_lm_round does)
  {
    LmState S;
    lm_init(S, x7, 1 << 30, true);
    ls = S;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      red[27] = (it & 1) ? red[27] * 0.25 : red[27] * 3.0;
      LmState L = ls;
      lm_step(L, red);
      if (L.status == LM_DONE) lm_init(L, L.x, 1 << 30, true);
      ls = L;
    }
    t(slot++, c0, r0);
    sink += ls.x[1];
  }
  // [2] lm_solve_step
  {
    LmState S;
    lm_init(S, x7, 4, true);
    for (int i = 0; i < 21; ++i) S.jtj[i] = red[i];
    for (int i = 0; i < 6; ++i) S.g[i] = red[21 + i], S.scaling[i] = 1.0 / (1.0 + sqrt(S.jtj[ut_index(i, i)]));
    double step[6] = {0, 0, 0, 0, 0, 0};
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      S.reuse_diag = 0;
      S.radius = 1e4 + step[0] * 1e-20;
      lm_solve_step(S, step);
    }
    t(slot++, c0, r0);
    sink += step[2];
  }
  // [3] lm_plus (quaternion: sincos + sqrt)
  {
    double x[7], d[6] = {1e-3, -2e-3, 5e-4, 0.01, 0.02, -0.01}, o[7];
    for (int i = 0; i < 7; ++i) x[i] = x7[i];
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      lm_plus(x, d, o);
      d[0] = 1e-3 + o[0] * 1e-20;
    }
    t(slot++, c0, r0);
    sink += o[3];
  }
  // [4] sincos alone
  {
    double a = 1e-3, sn = 0, cs = 0;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      sincos(a, &sn, &cs);
      a = 1e-3 + sn * 1e-20;
    }
    t(slot++, c0, r0);
    sink += cs;
  }
  // [5] sqrt alone
  {
    double a = 2.0;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) a = sqrt(a) + 1.0;
    t(slot++, c0, r0);
    sink += a;
  }
  // [6] division alone
  {
    double a = 2.0;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) a = 1.0 / a + 1.0;
    t(slot++, c0, r0);
    sink += a;
  }
  // [7] dependent fp64 FMA
  {
    double a = 1.0;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) a = fma(a, 0.999999, 1e-7);
    t(slot++, c0, r0);
    sink += a;
  }
  // [8] LDS state copy in + out
  {
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      LmState L = ls;
      L.radius += 1.0;
      ls = L;
    }
    t(slot++, c0, r0);
    sink += ls.radius;
  }
  // [9] lm_gradmax (rotation branch: small gradient)
  {
    double g[6] = {1e-12, 2e-12, 3e-12, 1e-13, 1e-13, 1e-13}, m = 0;
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      m = lm_gradmax(x7, g);
      g[0] = 1e-12 + m * 1e-30;
    }
    t(slot++, c0, r0);
    sink += m;
  }
  out->sink = sink;
}

// [10] as k_lm_round runs it: a 256-thread workgroup, the state in LDS, lane 0 steps a register copy
__global__ void __launch_bounds__(256) k_round_like(const double* red0, Out* out) {
  __shared__ LmState ls;
  __shared__ double sred[LM_NACC];
  if (threadIdx.x < LM_NACC) sred[threadIdx.x] = red0[threadIdx.x];
  if (threadIdx.x == 0) {
    double x7[7] = {0.01, -0.02, 0.03, 0.99925, 12.0, -3.0, 0.5};
    LmState S;
    lm_init(S, x7, 1 << 30, true);
    ls = S;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      sred[27] = (it & 1) ? sred[27] * 0.25 : sred[27] * 3.0;
      LmState L = ls;
      lm_step(L, sred);
      if (L.status == LM_DONE) lm_init(L, L.x, 1 << 30, true);
      ls = L;
    }
    out->cyc[0] = (__builtin_readcyclecounter() - c0) / R;
    out->rt[0] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// [11] the step straight on the LDS state (no register copy of the whole state)
__global__ void __launch_bounds__(256) k_round_lds(const double* red0, Out* out) {
  __shared__ LmState ls;
  __shared__ double sred[LM_NACC];
  if (threadIdx.x < LM_NACC) sred[threadIdx.x] = red0[threadIdx.x];
  if (threadIdx.x == 0) {
    double x7[7] = {0.01, -0.02, 0.03, 0.99925, 12.0, -3.0, 0.5};
    lm_init(ls, x7, 1 << 30, true);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
      sred[27] = (it & 1) ? sred[27] * 0.25 : sred[27] * 3.0;
      lm_step(ls, sred);
      if (ls.status == LM_DONE) {
        double x7[7];
        for (int i = 0; i < 7; ++i) x7[i] = ls.x[i];
        lm_init(ls, x7, 1 << 30, true);
      }
    }
    out->cyc[0] = (__builtin_readcyclecounter() - c0) / R;
    out->rt[0] = __builtin_amdgcn_s_memrealtime() - r0;
    out->sink = ls.x[0];
  }
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
  if (hipMalloc(&dred, sizeof(h)) != hipSuccess || hipMalloc(&dout, sizeof(Out)) != hipSuccess) return 1;
  if (hipMemcpy(dred, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  Out o{};
  for (int rep = 0; rep < 3; ++rep) {
    k_mb<<<1, 64>>>(dred, dout);
    if (hipMemcpy(&o, dout, sizeof(Out), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  Out o2{};
  for (int rep = 0; rep < 3; ++rep) {
    k_round_like<<<1, 256>>>(dred, dout);
    if (hipMemcpy(&o2, dout, sizeof(Out), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  std::printf("%-32s %7llu cycles per call  (%.3f us per call)\n", "lm_step as in k_lm_round", o2.cyc[0],
              o2.rt[0] / 100.0 / R);
  double xa = o2.sink;
  for (int rep = 0; rep < 3; ++rep) {
    k_round_lds<<<1, 256>>>(dred, dout);
    if (hipMemcpy(&o2, dout, sizeof(Out), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  std::printf("%-32s %7llu cycles per call  (%.3f us per call)  (x0 %.17g)\n", "lm_step on the LDS state", o2.cyc[0],
              o2.rt[0] / 100.0 / R, o2.sink);
  (void)xa;
  const char* names[10] = {"lm_step (state in registers)", "lm_step (state staged in LDS)", "lm_solve_step",
                           "lm_plus", "sincos f64", "sqrt f64", "1/x f64", "fma f64 (dependent)",
                           "LDS state copy in + out", "lm_gradmax (rotation branch)"};
  for (int i = 0; i < 10; ++i)
    std::printf("%-32s %7llu cycles per call  (%.3f us per call)\n", names[i], o.cyc[i], o.rt[i] / 100.0 / R);
  std::printf("sink %g\n", o.sink);
  return 0;
}
