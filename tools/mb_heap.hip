// Microbenchmark: libstdc++ heap sort (__make_heap + __sort_heap) of one LDS segment per wave, in
// the two device formulations of stdsort.h / voxel_hot.h: one lane (ss_heap_sort) and the wave
// (vh_heap_sort_wave: scalar path codes over 5-level look-aheads).  Checks the permutations
// agree; prints cycles per element.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../vloam-noted_amd/csrc tools/mb_heap.hip -o /tmp/mb_heap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "voxel_hot.h"

using namespace loam;

template <int MODE>
__global__ void __launch_bounds__(1024) k_heap(const uint32_t* in, uint32_t* out, int len, unsigned long long* cyc) {
  __shared__ uint32_t E[16 * 2048];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* S = E + wid * 2048;
  const uint32_t* src = in + (size_t)(blockIdx.x * (blockDim.x >> 6) + wid) * len;
  for (int i = lane; i < len; i += 64) S[i] = src[i];
  ss_wave_fence();
  const unsigned long long t0 = __builtin_readcyclecounter();
  if (MODE == 0) {
    if (lane == 0) ss_heap_sort(S, 0, len, VhLess{});
    ss_wave_fence();
  } else {
    vh_heap_sort_wave(S, 0, len);
    ss_wave_fence();
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (lane == 0) atomicAdd(cyc, t1 - t0);
  uint32_t* dst = out + (size_t)(blockIdx.x * (blockDim.x >> 6) + wid) * len;
  for (int i = lane; i < len; i += 64) dst[i] = S[i];
}

int main() {
  const int lens[] = {20, 128, 512, 1024, 2048};
  for (int waves : {1, 16}) {
    for (int len : lens) {
      const int blocks = 256, segs = blocks * waves;
      std::vector<uint32_t> h((size_t)segs * len);
      srand(7);
      for (int s = 0; s < segs; ++s)
        for (int i = 0; i < len; ++i) h[(size_t)s * len + i] = ((uint32_t)(rand() % (len / 3 + 1)) << 16) | (uint32_t)i;
      uint32_t *din, *dout;
      unsigned long long* dc;
      hipMalloc(&din, h.size() * 4);
      hipMalloc(&dout, h.size() * 4 * 3);
      hipMalloc(&dc, 8 * 3);
      hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
      hipMemset(dc, 0, 24);
      k_heap<0><<<blocks, 64 * waves>>>(din, dout, len, dc);
      k_heap<1><<<blocks, 64 * waves>>>(din, dout + h.size(), len, dc + 1);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel error\n");
        return 1;
      }
      std::vector<uint32_t> o(h.size() * 2);
      unsigned long long c[2];
      hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
      hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
      const bool ok = std::equal(o.begin(), o.begin() + h.size(), o.begin() + h.size());
      printf("waves/CU %2d len %5d: cycles/element one-lane %.0f wave %.0f  (%s)\n", waves, len,
             (double)c[0] / segs / len, (double)c[1] / segs / len, ok ? "same permutation" : "DIFFERS");
      if (!ok) return 1;
      hipFree(din);
      hipFree(dout);
      hipFree(dc);
    }
  }
  return 0;
}
