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
