// Microbenchmark: per-kernel cost of short kernels in a hipGraph vs plain stream launches
// (the one-stream mapper frame is ~16 dependent launches).
// hipcc --offload-arch=gfx950 -O3 tools/mb_graph.hip -o tools/bin/mb_graph
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_tiny(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += v;
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::printf("%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

int main() {
  int* p;
  check(hipMalloc(&p, 4096), "malloc");
  hipStream_t st;
  check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int blocks : {1, 64, 512}) {
    for (int n : {1, 16}) {
      // plain launches
      for (int w = 0; w < 10; ++w) k_tiny<<<blocks, 64, 0, st>>>(p, 1);
      hipStreamSynchronize(st);
      const int reps = 200;
      hipEventRecord(a, st);
      for (int r = 0; r < reps; ++r)
        for (int k = 0; k < n; ++k) k_tiny<<<blocks, 64, 0, st>>>(p, 1);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const float plain = 1000.f * ms / (reps * n);
      // the same as one graph of n kernels
      hipGraph_t g;
      hipGraphExec_t ge;
      check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "capture");
      for (int k = 0; k < n; ++k) k_tiny<<<blocks, 64, 0, st>>>(p, 1);
      check(hipStreamEndCapture(st, &g), "end capture");
      check(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "instantiate");
      for (int w = 0; w < 10; ++w) hipGraphLaunch(ge, st);
      hipStreamSynchronize(st);
      hipEventRecord(a, st);
      for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      const float graph = 1000.f * ms / (reps * n);
      // one graph launch + host sync per iteration (a frame's launch -> wait round trip)
      hipEventRecord(a, st);
      for (int r = 0; r < 50; ++r) {
        hipGraphLaunch(ge, st);
        hipStreamSynchronize(st);
      }
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      const float rt = 1000.f * ms / 50;
      std::printf("blocks %4d kernels %3d: plain %6.2f us/kernel, graph %6.2f us/kernel, graph launch+sync %7.2f us\n",
                  blocks, n, plain, graph, rt);
      hipGraphExecDestroy(ge);
      hipGraphDestroy(g);
    }
  }
  return 0;
}
