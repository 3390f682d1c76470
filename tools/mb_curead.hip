// Microbenchmark: how long one 1024-thread workgroup takes to read a freshly written cube (16 B
// points, just written by another kernel, possibly on another XCD), against the same bytes read by
// K workgroups (1/K each) -- the first pass of the re-VoxelGrid merge of a large cube.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mb_curead.hip -o /tmp/mb_curead
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_write(float4* p, int n, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    p[i] = make_float4(v + i, v - i, v * 0.5f + i, 1.f);
}

// K workgroups; workgroup b reads points [b n / K, (b + 1) n / K), U loads in flight per round
template <int U>
__global__ void __launch_bounds__(1024) k_read(const float4* p, int n, int K, float* out, unsigned long long* cyc) {
  const int b = blockIdx.x;
  const int lo = (int)((long long)n * b / K), hi = (int)((long long)n * (b + 1) / K);
  const unsigned long long t0 = __builtin_readcyclecounter();
  float mn = 3e38f, mx = -3e38f;
  for (int i0 = lo + threadIdx.x; i0 < hi; i0 += U * 1024) {
    float4 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * 1024 < hi) q[u] = p[i0 + u * 1024];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * 1024 < hi) {
        mn = fminf(mn, fminf(q[u].x, fminf(q[u].y, q[u].z)));
        mx = fmaxf(mx, fmaxf(q[u].x, fmaxf(q[u].y, q[u].z)));
      }
  }
  __shared__ float s[2];
  if (threadIdx.x == 0) s[0] = s[1] = 0.f;
  __syncthreads();
  atomicAdd(&s[0], mn);
  atomicAdd(&s[1], mx);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[b] = s[0] + s[1];
    atomicMax(cyc, __builtin_readcyclecounter() - t0);
  }
}

int main() {
  const int n = 14000;  // a large map cube
  float4* p;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&p, sizeof(float4) * n * 64);
  hipMalloc(&out, sizeof(float) * 64);
  hipMalloc(&cyc, 8 * 64);
  for (int K : {1, 2, 4, 8}) {
    for (int U : {4, 16}) {
      unsigned long long tot = 0;
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        float4* q = p + (size_t)(r % 64) * n;  // a fresh location every time, written by 7 blocks
        k_write<<<7, 256>>>(q, n, (float)r);
        hipMemset(cyc, 0, 8);
        if (U == 4) k_read<4><<<K, 1024>>>(q, n, K, out, cyc);
        else k_read<16><<<K, 1024>>>(q, n, K, out, cyc);
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        if (r >= 2) tot += c;
      }
      printf("n %d points, %d workgroups, %2d loads in flight per lane: %.0f cycles (slowest workgroup)\n", n, K, U,
             (double)tot / (reps - 2));
    }
  }
  return 0;
}
