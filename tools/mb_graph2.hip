// Microbenchmark: host time of hipGraphLaunch while the stream is busy (a frame in flight),
// for graphs of short kernels with / without a D2H memcpy node and a cross-stream event wait
// before the launch.
// hipcc --offload-arch=gfx950 -O3 tools/mb_graph2.hip -o tools/bin/mb_graph2
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void k_tiny(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += v;
}

struct Big {
  int* p;
  long long pad[100];  // ~800 bytes of kernel arguments, as the mapper's by-value MapperDev
};
__global__ void k_big(Big b, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) b.p[0] += v + (int)b.pad[v & 63];
}
// reads a few words of page-locked host memory with system-scope loads (k_frame_prep's FrameIn)
__global__ void k_hostread(const unsigned long long* h, int* p) {
  if (threadIdx.x < 12) {
    unsigned long long v = __hip_atomic_load(h + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == 12345) p[1] = 1;
  }
}

// spins about `us` microseconds (s_memrealtime: 100 MHz)
__global__ void k_spin(int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(8);
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::printf("%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int* p;
  int* hbuf;
  check(hipMalloc(&p, 1 << 20), "malloc");
  check(hipHostMalloc(reinterpret_cast<void**>(&hbuf), 1 << 20, hipHostMallocDefault), "host malloc");
  hipStream_t st, st2;
  check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  check(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking), "stream2");
  hipEvent_t ev;
  check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
  unsigned long long* hin;
  check(hipHostMalloc(reinterpret_cast<void**>(&hin), 4096, hipHostMallocMapped | hipHostMallocCoherent), "host in");
  void* hin_dev = nullptr;
  check(hipHostGetDevicePointer(&hin_dev, hin, 0), "dev ptr");
  Big big{};
  big.p = p;
  for (int variant = 0; variant < 16; ++variant) {
    const bool copy = variant & 1, two = variant & 2, bigargs = variant & 4, hostread = variant & 8;
    hipGraphExec_t ge[2];
    for (int g = 0; g < 2; ++g) {
      hipGraph_t gr;
      check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "capture");
      if (hostread) k_hostread<<<1, 64, 0, st>>>(reinterpret_cast<const unsigned long long*>(hin_dev), p);
      for (int k = 0; k < 16; ++k) {
        if (bigargs) k_big<<<64, 64, 0, st>>>(big, k);
        else k_tiny<<<64, 64, 0, st>>>(p, 1);
      }
      if (copy) check(hipMemcpyAsync(hbuf, p, 64 * 1024, hipMemcpyDeviceToHost, st), "copy node");
      check(hipStreamEndCapture(st, &gr), "end capture");
      check(hipGraphInstantiate(&ge[g], gr, nullptr, nullptr, 0), "instantiate");
      hipGraphDestroy(gr);
    }
    for (int wait = 0; wait < 2; ++wait) {
      double t_launch = 0, t_max = 0;
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        k_spin<<<1, 64, 0, st>>>(300);  // the stream is busy for ~300 us
        if (wait) {
          k_tiny<<<1, 64, 0, st2>>>(p + 4096, 1);
          check(hipEventRecord(ev, st2), "record");
          check(hipStreamWaitEvent(st, ev, 0), "wait event");
        }
        const double t0 = now_us();
        check(hipGraphLaunch(ge[two ? (r & 1) : 0], st), "launch");
        const double dt = now_us() - t0;
        t_launch += dt;
        t_max = dt > t_max ? dt : t_max;
        check(hipStreamSynchronize(st), "sync");
      }
      std::printf("graph 16 %skernels%s%s, %s exec%s%s: hipGraphLaunch host time avg %7.1f us, max %7.1f us\n",
                  bigargs ? "800-byte-argument " : "", hostread ? " after a host-memory read" : "",
                  copy ? " + D2H node" : "", two ? "two alternating" : "one", two ? "s" : "",
                  wait ? ", after a cross-stream event wait" : "", t_launch / reps, t_max);
    }
    {  // device time of one graph launch (stream idle before)
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      float tot = 0;
      for (int r = 0; r < 20; ++r) {
        hipEventRecord(a, st);
        hipGraphLaunch(ge[0], st);
        hipEventRecord(b, st);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        tot += ms;
      }
      std::printf("   device time per launch: %7.1f us\n", 1000.f * tot / 20);
      hipEventDestroy(a);
      hipEventDestroy(b);
    }
    // back to back: two graph launches in flight, the second's host time
    {
      double t_launch = 0;
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        check(hipGraphLaunch(ge[0], st), "launch a");
        k_spin<<<1, 64, 0, st>>>(300);
        const double t0 = now_us();
        check(hipGraphLaunch(ge[two ? 1 : 0], st), "launch b");
        t_launch += now_us() - t0;
        check(hipStreamSynchronize(st), "sync");
      }
      std::printf("   second launch behind a graph + 300 us kernel: %7.1f us\n", t_launch / reps);
    }
    for (auto& g : ge) hipGraphExecDestroy(g);
  }
  return 0;
}
