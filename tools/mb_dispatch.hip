// Microbenchmark: cost of launching many workgroups that exit at once, by block size and LDS
// footprint (the k_revox launch shape: B * 2 * INS_SLOTS workgroups, most with nothing to do).
// hipcc --offload-arch=gfx950 -O3 tools/mb_dispatch.hip -o gpurun_out/mb_dispatch
#include <hip/hip_runtime.h>

#include <cstdio>

template <int NT, int LW>
__global__ void __launch_bounds__(NT) k_exit(const int* flag, int* out) {
  __shared__ int lds[LW];
  if (flag[blockIdx.x] == 0) return;
  lds[threadIdx.x] = (int)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[NT - 1 - threadIdx.x];
}

template <int NT, int LW>
static void run(const char* name, int grid, const int* flag, int* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) k_exit<NT, LW><<<grid, NT>>>(flag, out);
  hipEventRecord(a);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) k_exit<NT, LW><<<grid, NT>>>(flag, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  std::printf("%-28s grid %6d: %8.1f us / launch\n", name, grid, 1000.f * ms / reps);
}

int main() {
  const int grid = 128 * 2 * 139;
  int *flag, *out;
  hipMalloc(&flag, grid * sizeof(int));
  hipMalloc(&out, grid * sizeof(int));
  hipMemset(flag, 0, grid * sizeof(int));
  run<1024, 40960>("1024 thr, 160 KiB LDS", grid, flag, out);
  run<1024, 1024>("1024 thr, 4 KiB LDS", grid, flag, out);
  run<512, 16896>("512 thr, 66 KiB LDS", grid, flag, out);
  run<256, 256>("256 thr, 1 KiB LDS", grid, flag, out);
  run<64, 64>("64 thr", grid, flag, out);
  run<1024, 40960>("1024 thr, 160 KiB, grid/8", grid / 8, flag, out);
  hipFree(flag);
  hipFree(out);
  return 0;
}
