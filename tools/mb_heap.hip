// Microbenchmark: libstdc++ heap sort (__make_heap + __sort_heap) of one LDS segment per wave, in
// the two device formulations of stdsort.h / voxel_hot.h: one lane (ss_heap_sort) and the wave
// (vh_heap_sort_wave: scalar path codes over 5-level look-aheads), and the pipelined pops
// (vh_sort_heap_pipe).  Checks the permutations
// agree; prints cycles per element.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../vloam-noted_amd/csrc tools/mb_heap.hip -o /tmp/mb_heap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "voxel_hot.h"

using namespace loam;


// variant under test: vh_sort_heap_wave with compiler-only ordering (no lgkmcnt(0) waits): the
// LDS executes one wave's instructions in order
__device__ inline void mb_order() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ inline void mb_make_heap_wave(uint32_t* E, int lo, int hi) {
  const int lane = threadIdx.x & 63;
  const VhLess less;
  const int len = hi - lo;
  const int pmax = (len - 2) / 2;
  for (int d = 31 - __clz(pmax + 1); d >= 0; --d) {
    const int a = (1 << d) - 1, b = min(pmax, (1 << (d + 1)) - 2);
    for (int p = b - lane; p >= a; p -= 64) ss_adjust_heap(E, lo, p, len, E[lo + p], less);
    ss_wave_fence();
  }
}
__device__ inline void mb_sort_heap_wave(uint32_t* E, int lo, int hi) {
  const int lane = threadIdx.x & 63;
  const VhLess less;
  const int lj = 31 - __clz(lane + 2), lt = lane + 2 - (1 << lj);
  for (int last = hi - 1; last > lo; --last) {
    const int n = last - lo;
    const uint32_t v = E[last], top = E[lo];
    const int lim = (n - 1) / 2;
    int h = 0, k = 0;
    uint32_t code = 0;
    while (h < lim) {
      const int node = ((h + 1) << lj) - 1 + lt;
      const uint32_t x = (lane < 62 && node < n) ? E[lo + node] : 0u;
      const uint32_t xr = dpp_from_next(x);
      const uint64_t rw = __ballot(!less(xr, x));
      int tt = 0;
#pragma unroll
      for (int jj = 0; jj < 5; ++jj) {
        if (h >= lim) break;
        const int dir = (int)((rw >> ((1 << (jj + 1)) - 2 + 2 * tt)) & 1ull);
        h = 2 * h + 1 + dir;
        tt = 2 * tt + dir;
        code = 2 * code + (uint32_t)dir;
        ++k;
      }
    }
    if ((n & 1) == 0 && h == (n - 2) / 2) {
      h = 2 * h + 1;
      code = 2 * code;
      ++k;
    }
    const int j1 = lane + 1;
    const int hj = lane == 0 || lane > k ? 0 : (1 << lane) - 1 + (int)(code >> (k - lane));
    const int cj = j1 <= k ? (1 << j1) - 1 + (int)(code >> (k - j1)) : 0;
    const uint32_t pv = lane < k ? E[lo + cj] : 0u;
    const int q = k - __popcll(__ballot(lane < k && less(pv, v)));
    mb_order();
    if (lane < q) E[lo + hj] = pv;
    if (lane == q) E[lo + hj] = v;
    if (lane == 0) E[last] = top;
    mb_order();
  }
}

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
  } else if (MODE == 1) {
    vh_heap_sort_wave(S, 0, len, len);
    ss_wave_fence();
  } else if (MODE == 2) {
    if (len >= 2) {
      mb_make_heap_wave(S, 0, len);
      mb_sort_heap_wave(S, 0, len);
    }
    ss_wave_fence();
  } else if (MODE == 3) {  // the pipelined pops (vh_sort_heap_pipe)
    if (len >= 2) {
      vh_make_heap_wave(S, 0, len);
      ss_wave_fence();
      vh_sort_heap_pipe(S, 0, len, len);
    }
    ss_wave_fence();
  } else {  // __make_heap alone
    if (len >= 2) vh_make_heap_wave(S, 0, len);
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
      hipMalloc(&dout, h.size() * 4 * 5);
      hipMalloc(&dc, 8 * 5);
      hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
      hipMemset(dc, 0, 40);
      k_heap<0><<<blocks, 64 * waves>>>(din, dout, len, dc);
      k_heap<1><<<blocks, 64 * waves>>>(din, dout + h.size(), len, dc + 1);
      k_heap<2><<<blocks, 64 * waves>>>(din, dout + 2 * h.size(), len, dc + 2);
      k_heap<3><<<blocks, 64 * waves>>>(din, dout + 3 * h.size(), len, dc + 3);
      k_heap<4><<<blocks, 64 * waves>>>(din, dout + 4 * h.size(), len, dc + 4);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel error\n");
        return 1;
      }
      std::vector<uint32_t> o(h.size() * 5);
      unsigned long long c[5];
      hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
      hipMemcpy(c, dc, 40, hipMemcpyDeviceToHost);
      const bool ok = std::equal(o.begin(), o.begin() + h.size(), o.begin() + h.size()) &&
                      std::equal(o.begin(), o.begin() + h.size(), o.begin() + 2 * h.size()) &&
                      std::equal(o.begin(), o.begin() + h.size(), o.begin() + 3 * h.size());
      printf("waves/CU %2d len %5d: cycles/element one-lane %.0f wave %.0f variant %.0f pipelined %.0f"
             " (make_heap alone %.0f)  (%s)\n", waves, len,
             (double)c[0] / segs / len, (double)c[1] / segs / len, (double)c[2] / segs / len,
             (double)c[3] / segs / len, (double)c[4] / segs / len, ok ? "same permutation" : "DIFFERS");
      if (!ok) return 1;
      hipFree(din);
      hipFree(dout);
      hipFree(dc);
    }
  }
  return 0;
}
