// common.h — HIP plumbing shared by the LOAM core translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "loam_core.h"

namespace loam {

void set_error(const std::string& msg);

#define LOAM_HIP(call)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                \
      ::loam::set_error(std::string(#call) + ": " + hipGetErrorString(e_) + " (" +          \
                        __FILE__ + ":" + std::to_string(__LINE__) + ")");                  \
      return LOAM_ERR_HIP;                                                                 \
    }                                                                                      \
  } while (0)

// one-time check that a gfx950 device is present and usable
int32_t ensure_device(int32_t device);

#define TRY(x)                      \
  do {                              \
    int32_t rc_ = (x);              \
    if (rc_ != LOAM_OK) return rc_; \
  } while (0)

// Wave-wide inclusive scan / reductions on 64-lane waves
__device__ inline int wave_lane() { return threadIdx.x & 63; }

__device__ inline uint64_t lanemask_lt() {
  int l = wave_lane();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

__device__ inline double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ inline float wave_min_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline uint32_t wave_sum_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
// DPP (GFX9 data-parallel primitives, no LDS round trip): inclusive prefix sum of a u32 across the
// wave (row_shr 1/2/4/8 within each row of 16, then row_bcast 15 / 31 across the rows; lanes whose
// source is outside keep the 0 given as the old value), the wave total, and whole-wave shifts
__device__ inline uint32_t dpp_incl_scan_u(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return (uint32_t)x;
}
__device__ inline uint32_t dpp_wave_sum_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dpp_incl_scan_u(v), 63);
}
// lane i <- lane i + 1 (lane 63 <- 0) / lane i <- lane i - 1 (lane 0 <- 0)
__device__ inline uint32_t dpp_from_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);  // wave_shl:1
}
__device__ inline uint32_t dpp_from_prev(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

// inclusive prefix sum across the wave
__device__ inline uint32_t wave_incl_scan_u(uint32_t v) {
  int l = wave_lane();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

}  // namespace loam
