// Microbenchmark: the device-side gap between a kernel that leaves much of L2 dirty and the next
// kernel, across the boundaries a frame of the mapper has (plain stream order, a D2H copy to
// page-locked memory, an event record, a graph-to-graph boundary).  Wall clock from
// s_memrealtime (100 MHz) written by the kernels themselves.
// hipcc --offload-arch=gfx950 -O3 tools/mb_flush.hip -o tools/bin/mb_flush
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

// writes `words` dwords (dirty lines in L2), then every block stamps its end time
__global__ void k_dirty(uint32_t* buf, size_t words, unsigned long long* stamp) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
    buf[i] = (uint32_t)i;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&stamp[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

__global__ void k_stamp(unsigned long long* stamp) {
  if (threadIdx.x == 0 && blockIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::printf("%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

int main() {
  const size_t words = (size_t)16 << 20;  // 64 MiB written
  uint32_t* buf;
  unsigned long long* stamp;
  char* host;
  char* dsmall;
  check(hipMalloc(&buf, words * 4), "buf");
  check(hipMalloc(&stamp, 64), "stamp");
  check(hipMalloc(&dsmall, 8192), "small");
  check(hipHostMalloc(reinterpret_cast<void**>(&host), 8192, hipHostMallocDefault), "host");
  hipStream_t st;
  check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  hipEvent_t ev, evt;
  check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "ev");
  check(hipEventCreate(&evt), "evt");
  // graphs: [dirty] and [stamp]
  hipGraphExec_t g_dirty, g_stamp, g_dirty_copy;
  for (int k = 0; k < 3; ++k) {
    hipGraph_t gr;
    check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "cap");
    if (k == 1) k_stamp<<<1, 64, 0, st>>>(stamp);
    else k_dirty<<<1024, 256, 0, st>>>(buf, words, stamp);
    if (k == 2) hipMemcpyAsync(host, dsmall, 4096, hipMemcpyDeviceToHost, st);
    check(hipStreamEndCapture(st, &gr), "end");
    check(hipGraphInstantiate(k == 0 ? &g_dirty : (k == 1 ? &g_stamp : &g_dirty_copy), gr, nullptr, nullptr, 0), "inst");
    hipGraphDestroy(gr);
  }
  const char* names[] = {"plain stream order", "D2H copy (4 KiB, page-locked) between", "untimed event record between",
                         "timed event record between", "graph -> graph", "graph with D2H node -> graph",
                         "graph with D2H node + untimed event -> graph",
                         "graph -> wait (event of a 2nd stream, done) -> graph",
                         "graph -> wait (2nd stream event, pending at enqueue) -> graph"};
  hipStream_t st2;
  check(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking), "stream2");
  hipEvent_t ev2;
  check(hipEventCreateWithFlags(&ev2, hipEventDisableTiming), "ev2");
  for (int clean = 0; clean < 2; ++clean) {
    for (int v = 0; v < 9; ++v) {
      double tot = 0;
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        check(hipMemsetAsync(stamp, 0, 64, st), "memset");
        check(hipStreamSynchronize(st), "sync0");
        const size_t w = clean ? 1024 : words;
        if (v < 4) {
          k_dirty<<<1024, 256, 0, st>>>(buf, w, stamp);
          if (v == 1) hipMemcpyAsync(host, dsmall, 4096, hipMemcpyDeviceToHost, st);
          if (v == 2) hipEventRecord(ev, st);
          if (v == 3) hipEventRecord(evt, st);
          k_stamp<<<1, 64, 0, st>>>(stamp);
        } else {
          if (clean) {  // (graphs hold the full size; the clean rows use the plain forms only)
            k_dirty<<<1024, 256, 0, st>>>(buf, w, stamp);
          } else {
            if (v == 7) {  // an event of stream 2, complete before anything is enqueued here
              k_stamp<<<1, 64, 0, st2>>>(stamp + 4);
              hipEventRecord(ev2, st2);
              hipStreamSynchronize(st2);
            }
            if (v == 8) {  // pending at enqueue, done while the first graph runs
              k_stamp<<<1, 64, 0, st2>>>(stamp + 4);
              hipEventRecord(ev2, st2);
            }
            hipGraphLaunch(v == 4 || v >= 7 ? g_dirty : g_dirty_copy, st);
            if (v == 6) hipEventRecord(ev, st);
            if (v >= 7) hipStreamWaitEvent(st, ev2, 0);
          }
          hipGraphLaunch(g_stamp, st);
        }
        check(hipStreamSynchronize(st), "sync");
        unsigned long long h[2];
        check(hipMemcpy(h, stamp, 16, hipMemcpyDeviceToHost), "read");
        tot += (double)(h[1] - h[0]) / 100.0;
      }
      std::printf("%-6s L2: %-46s next kernel starts %7.2f us after the last block\n", clean ? "clean" : "dirty",
                  names[v], tot / reps);
    }
  }
  return 0;
}
