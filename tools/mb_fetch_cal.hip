// FETCH_SIZE calibration for the access widths of the correspondence kernels (MI355X_MICROARCH.md
// HBM section: "On gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
// streaming read ... Other access widths are uncalibrated: calibrate on a known byte count in
// your own access pattern").  Each kernel touches a known number of distinct 128-B lines of a
// 2 GiB buffer (far past the 256 MiB Infinity Cache), one access per line:
//   k_stream16   coalesced 16 B / lane stream            (known bytes = lines x 128)
//   k_rand8      one 8 B load at a random line           (the cell-table probe of k_knn)
//   k_rand16     one 16 B load at a random line          (a float4 map point)
//   k_rand64     four consecutive 16 B loads of one line by 4 lanes (a cell's first points)
// Run under rocprofv3 --pmc FETCH_SIZE --kernel-trace; FETCH_SIZE / (lines x 128 B) is the factor
// for that pattern (tools/pmc_traffic.py applies it per kernel).
// hipcc --offload-arch=gfx950 -O3 tools/mb_fetch_cal.hip -o gpurun_out/mb_fetch_cal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr size_t BUF = 2ull << 30;  // bytes
constexpr size_t LINES = BUF / 128;
constexpr int N = 1 << 22;  // accesses (4 Mi lines = 512 MiB of distinct lines)

__global__ void k_stream16(const float4* __restrict__ a, int n, float* out) {
  float acc = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) acc += a[i].x;
  if (acc == 12345.f) out[0] = acc;
}

__global__ void k_rand8(const uint2* __restrict__ a, const uint32_t* __restrict__ line, int n, uint32_t* out) {
  uint32_t acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    acc += a[(size_t)line[i] * 16].x;  // 16 x 8 B = 128 B per line
  if (acc == 12345u) out[0] = acc;
}

__global__ void k_rand16(const float4* __restrict__ a, const uint32_t* __restrict__ line, int n, float* out) {
  float acc = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    acc += a[(size_t)line[i] * 8].x;  // 8 x 16 B = 128 B per line
  if (acc == 12345.f) out[0] = acc;
}

__global__ void k_rand64(const float4* __restrict__ a, const uint32_t* __restrict__ line, int n, float* out) {
  float acc = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 4 * n; i += gridDim.x * blockDim.x)
    acc += a[(size_t)line[i >> 2] * 8 + (i & 3)].x;  // 4 lanes x 16 B of one line
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  void* buf = nullptr;
  uint32_t* d_line = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, BUF) != hipSuccess || hipMalloc(&d_line, sizeof(uint32_t) * N) != hipSuccess ||
      hipMalloc(&out, 64) != hipSuccess)
    return 1;
  (void)hipMemset(buf, 1, BUF);
  // N distinct random lines (a stride permutation of the line space)
  std::vector<uint32_t> line(N);
  const uint64_t stride = 2654435761ull % LINES | 1ull;
  for (int i = 0; i < N; ++i) line[i] = (uint32_t)(((uint64_t)i * stride) % LINES);
  (void)hipMemcpy(d_line, line.data(), sizeof(uint32_t) * N, hipMemcpyHostToDevice);
  const int grid = 4096, block = 256;
  // warm-up (code, TLB), then one measured launch each; an Infinity-Cache flush between them
  // (a 1 GiB stream of the other half) keeps the random lines cold
  k_stream16<<<grid, block>>>((const float4*)buf, (int)(BUF / 2 / 16), out);
  (void)hipDeviceSynchronize();
  k_stream16<<<grid, block>>>((const float4*)buf, (int)(BUF / 2 / 16), out);  // 1 GiB known
  k_stream16<<<grid, block>>>((const float4*)((char*)buf + BUF / 2), (int)(BUF / 2 / 16), out);
  k_rand8<<<grid, block>>>((const uint2*)buf, d_line, N, (uint32_t*)out);
  k_stream16<<<grid, block>>>((const float4*)((char*)buf + BUF / 2), (int)(BUF / 2 / 16), out);
  k_rand16<<<grid, block>>>((const float4*)buf, d_line, N, out);
  k_stream16<<<grid, block>>>((const float4*)((char*)buf + BUF / 2), (int)(BUF / 2 / 16), out);
  k_rand64<<<grid, block>>>((const float4*)buf, d_line, N, out);
  (void)hipDeviceSynchronize();
  std::printf("known bytes: stream16 %zu (1 GiB), random patterns %zu distinct 128-B lines = %zu B\n",
              (size_t)(BUF / 2), (size_t)N, (size_t)N * 128);
  (void)hipFree(buf);
  (void)hipFree(d_line);
  (void)hipFree(out);
  return 0;
}
