// Check: a kernel (plain launch and inside a graph) reads page-locked host memory that the host
// rewrote just before each launch, with system-scope atomic loads and with plain loads.
// hipcc --offload-arch=gfx950 -O3 tools/mb_hostread.hip -o tools/bin/mb_hostread
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_read(const unsigned long long* h, unsigned long long* out) {
  const int w = threadIdx.x;
  if (w < 12) {
    out[w] = __hip_atomic_load(h + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    out[16 + w] = h[w];
  }
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::printf("%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

int main() {
  const unsigned flags[3] = {hipHostMallocDefault, hipHostMallocMapped | hipHostMallocCoherent,
                             hipHostMallocMapped | hipHostMallocNonCoherent};
  const char* names[3] = {"default", "mapped|coherent", "mapped|noncoherent"};
  hipStream_t st;
  check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  unsigned long long* out;
  check(hipMalloc(&out, 256), "out");
  for (int f = 0; f < 3; ++f) {
    unsigned long long* h;
    check(hipHostMalloc(reinterpret_cast<void**>(&h), 4096, flags[f]), "host");
    void* dp = nullptr;
    check(hipHostGetDevicePointer(&dp, h, 0), "devptr");
    hipGraph_t gr;
    hipGraphExec_t ge;
    check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "cap");
    k_read<<<1, 64, 0, st>>>(reinterpret_cast<const unsigned long long*>(dp), out);
    check(hipStreamEndCapture(st, &gr), "end");
    check(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0), "inst");
    int bad_atomic[2] = {0, 0}, bad_plain[2] = {0, 0};
    for (int graph = 0; graph < 2; ++graph)
      for (int r = 0; r < 50; ++r) {
        for (int w = 0; w < 12; ++w) h[w] = 1000ull * r + w + 7;
        if (graph) check(hipGraphLaunch(ge, st), "launch");
        else k_read<<<1, 64, 0, st>>>(reinterpret_cast<const unsigned long long*>(dp), out);
        unsigned long long o[32];
        check(hipMemcpyAsync(o, out, 256, hipMemcpyDeviceToHost, st), "copy");
        check(hipStreamSynchronize(st), "sync");
        for (int w = 0; w < 12; ++w) {
          bad_atomic[graph] += o[w] != 1000ull * r + w + 7;
          bad_plain[graph] += o[16 + w] != 1000ull * r + w + 7;
        }
      }
    std::printf("%-20s dev ptr %s host ptr: wrong words, plain launch: atomic %d plain %d; graph: atomic %d plain %d (of 600)\n",
                names[f], dp == (void*)h ? "==" : "!=", bad_atomic[0], bad_plain[0], bad_atomic[1], bad_plain[1]);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(gr);
    hipHostFree(h);
  }
  return 0;
}
