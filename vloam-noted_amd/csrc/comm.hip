// comm.hip — loam_comm: RCCL (run-time loaded) or caller callbacks (include/loam_core.h).
//
// RCCL is resolved with dlopen("librccl.so.1"): in a process that already loaded PyTorch's
// RCCL (same soname) that copy is reused, so the mapper's communicator and torch.distributed
// share one library.  The library links no RCCL at build time, and unsharded use never
// touches it.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "comm.h"

namespace {

struct RcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      api.err = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
      return;
    }
    api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(dlsym(h, "ncclAllReduce"));
    api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(h, "ncclAllGather"));
    api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
    api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_reduce && api.all_gather &&
             api.error_string;
    if (!api.ok) api.err = "librccl.so.1 lacks an expected symbol";
  });
  return api;
}

int32_t rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return LOAM_OK;
  loam::set_error(std::string(what) + ": " + rccl().error_string(r));
  return LOAM_ERR_HIP;
}

size_t dtype_size(int32_t dt) { return dt == LOAM_DT_F64 ? 8 : 4; }

int32_t ensure_staging(loam_comm* c, size_t send_bytes, size_t recv_bytes) {
  const size_t need = std::max(send_bytes, recv_bytes);
  if (need <= c->h_cap) return LOAM_OK;
  if (c->h_send) (void)hipHostFree(c->h_send);
  if (c->h_recv) (void)hipHostFree(c->h_recv);
  c->h_send = c->h_recv = nullptr;
  c->h_cap = 0;
  LOAM_HIP(hipHostMalloc(&c->h_send, need, hipHostMallocDefault));
  LOAM_HIP(hipHostMalloc(&c->h_recv, need, hipHostMallocDefault));
  c->h_cap = need;
  return LOAM_OK;
}

}  // namespace

namespace loam {

// Ranks of one process sharing one device (loam_comm_create_local): the collectives are ordered
// on the ranks' own HIP streams by events, and the host threads meet only when they enqueue (one
// barrier per collective), never waiting for the device.  Collective k of rank r, buffers of
// parity k & 1:
//   1. wait until every rank has finished reading this parity's staging (collective k - 2),
//      copy the input into its staging buffer, record evA[r];
//   2. host barrier: every rank has enqueued step 1 of collective k;
//   3. wait for every rank's evA, combine all ranks' staging buffers in rank order (a sum kernel
//      for the all-reduce: every rank adds the same values in the same order, so the results are
//      bit-identical; copies for the all-gather), record evB[r].
struct LocalGroup {
  int size = 1, device = 0;
  int alive = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  void* stage[2][LOAM_LOCAL_MAX_RANKS] = {};
  size_t cap[2][LOAM_LOCAL_MAX_RANKS] = {};
  hipEvent_t evA[2][LOAM_LOCAL_MAX_RANKS] = {};
  hipEvent_t evB[2][LOAM_LOCAL_MAX_RANKS] = {};
  bool usedB[2][LOAM_LOCAL_MAX_RANKS] = {};

  void* peer = nullptr;  // comm_peer_buffer
  size_t peer_bytes = 0;
  size_t peer_req[LOAM_LOCAL_MAX_RANKS] = {};     // this binding's requested size, per rank
  bool peer_bound[LOAM_LOCAL_MAX_RANKS] = {};     // a live mapper of rank r holds the buffer
  int32_t peer_rc = LOAM_OK;                      // rank 0's decision for the current binding
  int peer_leaders = 0;                           // LM leaders this binding reserved on the device
  const void* blobs[LOAM_LOCAL_MAX_RANKS] = {};  // comm_group_launch
  hipEvent_t ev_pre[LOAM_LOCAL_MAX_RANKS] = {};
  hipEvent_t ev_post = nullptr;
  bool broken = false;
  // false: a rank did not arrive within the timeout (it failed or stopped); the group is broken
  // and every later collective fails at once instead of hanging
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t g = generation;
    if (++arrived == size) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return true;
    }
    const bool woke = cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != g || broken; });
    // the barrier completed (every rank arrived) even if a rank broke the group just after it,
    // e.g. by leaving once its last collective was done: that collective succeeded
    if (generation != g) return true;
    (void)woke;  // timed out, or broken before every rank arrived
    broken = true;
    cv.notify_all();
    return false;
  }
  // a rank that fails between or inside collectives (or leaves the group) breaks it at once:
  // the other ranks' barriers return false now instead of after their 120 s timeout
  void break_group() {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
};

static void local_group_free_events(LocalGroup& G) {
  for (int p = 0; p < 2; ++p)
    for (int r = 0; r < LOAM_LOCAL_MAX_RANKS; ++r) {
      if (G.evA[p][r]) (void)hipEventDestroy(G.evA[p][r]);
      if (G.evB[p][r]) (void)hipEventDestroy(G.evB[p][r]);
      G.evA[p][r] = G.evB[p][r] = nullptr;
    }
  for (int r = 0; r < LOAM_LOCAL_MAX_RANKS; ++r) {
    if (G.ev_pre[r]) (void)hipEventDestroy(G.ev_pre[r]);
    G.ev_pre[r] = nullptr;
  }
  if (G.ev_post) (void)hipEventDestroy(G.ev_post);
  G.ev_post = nullptr;
}

struct LocalSum {
  const void* src[LOAM_LOCAL_MAX_RANKS];
};

template <typename T>
__global__ void k_local_sum(LocalSum in, int nsrc, T* out, int64_t count) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    T v = static_cast<const T*>(in.src[0])[i];
    for (int q = 1; q < nsrc; ++q) v += static_cast<const T*>(in.src[q])[i];
    out[i] = v;
  }
}

// steps 1 and 2; returns the parity.  A HIP failure before the barrier breaks the group (the
// other ranks would otherwise wait for this one until their timeout)
static int32_t local_stage_hip(LocalGroup& G, int r, int p, const void* d_in, size_t bytes, hipStream_t st) {
  for (int q = 0; q < G.size; ++q)
    if (G.usedB[p][q]) LOAM_HIP(hipStreamWaitEvent(st, G.evB[p][q], 0));
  if (G.cap[p][r] < bytes) {  // (grows rarely; hipFree waits for the device)
    if (G.stage[p][r]) LOAM_HIP(hipFree(G.stage[p][r]));
    G.stage[p][r] = nullptr;
    G.cap[p][r] = 0;
    LOAM_HIP(hipMalloc(&G.stage[p][r], bytes));
    G.cap[p][r] = bytes;
  }
  LOAM_HIP(hipMemcpyAsync(G.stage[p][r], d_in, bytes, hipMemcpyDeviceToDevice, st));
  LOAM_HIP(hipEventRecord(G.evA[p][r], st));
  return LOAM_OK;
}
static int32_t local_stage(loam_comm* c, const void* d_in, size_t bytes, hipStream_t st, int* par) {
  LocalGroup& G = *c->local;
  const int r = c->rank, p = (int)(c->seq++ & 1);
  *par = p;
  const int32_t rc = local_stage_hip(G, r, p, d_in, bytes, st);
  if (rc != LOAM_OK) {
    G.break_group();
    return rc;
  }
  if (!G.barrier()) {
    set_error("local comm: a rank did not reach the collective (group broken)");
    return LOAM_ERR_SYNC;
  }
  for (int q = 0; q < G.size; ++q)
    if (q != r) LOAM_HIP(hipStreamWaitEvent(st, G.evA[p][q], 0));
  return LOAM_OK;
}

static int32_t local_allreduce(loam_comm* c, void* d_buf, int64_t count, int32_t dtype, hipStream_t st) {
  LocalGroup& G = *c->local;
  const size_t bytes = (size_t)count * dtype_size(dtype);
  int p = 0;
  TRY(local_stage(c, d_buf, bytes, st, &p));
  LocalSum in{};
  for (int q = 0; q < G.size; ++q) in.src[q] = G.stage[p][q];
  const int blocks = (int)std::min<int64_t>(1024, (count + 255) / 256);
  if (dtype == LOAM_DT_F64)
    k_local_sum<double><<<blocks, 256, 0, st>>>(in, G.size, static_cast<double*>(d_buf), count);
  else
    k_local_sum<int32_t><<<blocks, 256, 0, st>>>(in, G.size, static_cast<int32_t*>(d_buf), count);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipEventRecord(G.evB[p][c->rank], st));
  G.usedB[p][c->rank] = true;
  return LOAM_OK;
}

static int32_t local_allgather(loam_comm* c, const void* d_send, void* d_recv, int64_t bytes, hipStream_t st) {
  LocalGroup& G = *c->local;
  int p = 0;
  TRY(local_stage(c, d_send, (size_t)bytes, st, &p));
  for (int q = 0; q < G.size; ++q)
    LOAM_HIP(hipMemcpyAsync(static_cast<char*>(d_recv) + (size_t)q * bytes, G.stage[p][q], (size_t)bytes,
                            hipMemcpyDeviceToDevice, st));
  LOAM_HIP(hipEventRecord(G.evB[p][c->rank], st));
  G.usedB[p][c->rank] = true;
  return LOAM_OK;
}

void comm_abort(loam_comm* c) {
  if (c && c->kind == 2 && c->local) c->local->break_group();
}

int32_t comm_group_launch(loam_comm* c, const void* blob, hipStream_t st, comm_group_launch_fn fn, void* user) {
  if (!c || c->kind != 2 || !c->local || !fn) return LOAM_ERR_STATE;
  LocalGroup& G = *c->local;
  const int r = c->rank;
  int32_t rc = LOAM_OK;
  if (hipEventRecord(G.ev_pre[r], st) != hipSuccess) rc = LOAM_ERR_HIP;
  G.blobs[r] = blob;  // (read by rank 0 before the second meeting; the caller's, valid until then)
  if (rc != LOAM_OK) {
    G.break_group();
    set_error("local comm: group launch: hipEventRecord failed");
    return rc;
  }
  if (!G.barrier()) {
    set_error("local comm: a rank did not reach the group launch (group broken)");
    return LOAM_ERR_SYNC;
  }
  if (r == 0) {
    for (int q = 1; q < G.size && rc == LOAM_OK; ++q)
      if (hipStreamWaitEvent(st, G.ev_pre[q], 0) != hipSuccess) rc = LOAM_ERR_HIP;
    if (rc == LOAM_OK) {
      fn(G.blobs, G.size, st, user);
      if (hipGetLastError() != hipSuccess || hipEventRecord(G.ev_post, st) != hipSuccess) rc = LOAM_ERR_HIP;
    }
    if (rc != LOAM_OK) {
      G.break_group();
      set_error("local comm: group launch failed");
      return rc;
    }
  }
  if (!G.barrier()) {  // rank 0 recorded ev_post
    set_error("local comm: the group launch's rank 0 failed (group broken)");
    return LOAM_ERR_SYNC;
  }
  if (r != 0) LOAM_HIP(hipStreamWaitEvent(st, G.ev_post, 0));
  return LOAM_OK;
}

// Leaders of the persistent group LM rounds (k_lm_group) reserved per device, process-wide: a
// leader waits for the other ranks' leaders of its launch, which are dispatched after it, so the
// leaders of every group bound at once in this process must fit the device together (one
// 256-thread LM workgroup per CU).  Kernels that end on their own (other handles' kernels, this
// handle's stack VoxelGrids) only delay a leader's dispatch; a binding whose leaders would not fit
// beside the groups already bound fails (LOAM_ERR_CAPACITY: the two-kernel LM path instead).
static std::mutex g_lead_mu;
static int g_lead_reserved[64] = {};

int32_t comm_peer_buffer(loam_comm* c, size_t bytes, int leaders, int capacity, void** dev) {
  if (!c || !dev || c->kind != 2 || !c->local) return LOAM_ERR_STATE;
  LocalGroup& G = *c->local;
  const int r = c->rank;
  {
    std::lock_guard<std::mutex> lk(G.mu);
    G.peer_req[r] = bytes;
  }
  // every rank binds (a sharded mapper is created on every rank); then rank 0 (re)allocates and
  // zeroes the buffer, flags and all, while no rank's kernels use it: the flags hold
  // epoch * LM_MAX_PASSES + pass + 1 of the mapper that used them last, and a new mapper counts
  // its epochs from 1 again.  A rank whose earlier mapper still holds the buffer makes
  // the binding fail on every rank alike (the mappers then take the two-kernel LM path)
  if (!G.barrier()) {
    set_error("local comm: a rank did not reach the peer-buffer binding (group broken)");
    return LOAM_ERR_SYNC;
  }
  if (r == 0) {
    std::lock_guard<std::mutex> lk(G.mu);
    int32_t rc = LOAM_OK;
    for (int q = 0; q < G.size; ++q) {
      if (G.peer_req[q] != bytes) rc = LOAM_ERR_ARG;
      if (G.peer_bound[q] && rc == LOAM_OK) rc = LOAM_ERR_STATE;
    }
    if (rc == LOAM_OK && G.peer && G.peer_bytes != bytes) {
      if (hipSetDevice(G.device) != hipSuccess || hipDeviceSynchronize() != hipSuccess || hipFree(G.peer) != hipSuccess)
        rc = LOAM_ERR_HIP;
      G.peer = nullptr;
      G.peer_bytes = 0;
    }
    if (rc == LOAM_OK && !G.peer) {
      if (hipSetDevice(G.device) != hipSuccess || hipMalloc(&G.peer, bytes) != hipSuccess) {
        G.peer = nullptr;
        rc = LOAM_ERR_HIP;
      } else {
        G.peer_bytes = bytes;
      }
    }
    // zeroed and finished before any rank's kernels (non-blocking streams are not ordered behind
    // the null stream); the device synchronize also waits out any kernel of an earlier mapper
    if (rc == LOAM_OK && (hipSetDevice(G.device) != hipSuccess || hipMemset(G.peer, 0, bytes) != hipSuccess ||
                          hipDeviceSynchronize() != hipSuccess))
      rc = LOAM_ERR_HIP;
    if (rc == LOAM_OK) {
      std::lock_guard<std::mutex> lk2(g_lead_mu);
      const int d = G.device & 63;
      if (leaders <= 0 || g_lead_reserved[d] + leaders > capacity) {
        rc = LOAM_ERR_CAPACITY;
      } else {
        g_lead_reserved[d] += leaders;
        G.peer_leaders = leaders;
      }
    }
    if (rc == LOAM_OK)
      for (int q = 0; q < G.size; ++q) G.peer_bound[q] = true;
    G.peer_rc = rc;
  }
  if (!G.barrier()) {
    set_error("local comm: the peer-buffer binding's rank 0 did not return (group broken)");
    return LOAM_ERR_SYNC;
  }
  int32_t rc;
  {
    std::lock_guard<std::mutex> lk(G.mu);
    rc = G.peer_rc;
  }
  if (rc != LOAM_OK) {
    set_error(rc == LOAM_ERR_STATE      ? "local comm: a rank's earlier mapper still holds the group's LM peer buffer"
              : rc == LOAM_ERR_ARG      ? "local comm: ranks asked for peer buffers of different sizes"
              : rc == LOAM_ERR_CAPACITY ? "local comm: the group LM's leaders do not fit the device beside the "
                                          "groups already bound"
                                        : "local comm: peer buffer allocation failed");
    return rc;
  }
  *dev = G.peer;
  return LOAM_OK;
}

void comm_peer_release(loam_comm* c) {
  if (!c || c->kind != 2 || !c->local) return;
  LocalGroup& G = *c->local;
  std::lock_guard<std::mutex> lk(G.mu);
  G.peer_bound[c->rank] = false;
  bool any = false;
  for (int q = 0; q < G.size; ++q) any |= G.peer_bound[q];
  if (!any && G.peer_leaders > 0) {  // the group's last mapper: its leaders leave the device budget
    std::lock_guard<std::mutex> lk2(g_lead_mu);
    g_lead_reserved[G.device & 63] -= G.peer_leaders;
    G.peer_leaders = 0;
  }
}

int32_t comm_allreduce(loam_comm* c, void* d_buf, int64_t count, int32_t dtype, hipStream_t st) {
  if (!c || count < 0 || (dtype != LOAM_DT_F64 && dtype != LOAM_DT_I32)) {
    set_error("comm allreduce: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (count == 0) return LOAM_OK;
  if (c->kind == 2) return c->size == 1 ? LOAM_OK : local_allreduce(c, d_buf, count, dtype, st);
  if (c->kind == 1)  // RCCL runs even at one rank (the transport is then exercised by tests)
    return rccl_check(rccl().all_reduce(d_buf, d_buf, (size_t)count, dtype == LOAM_DT_F64 ? ncclFloat64 : ncclInt32,
                                        ncclSum, static_cast<ncclComm_t>(c->nccl), st),
                      "ncclAllReduce");
  if (c->size == 1) return LOAM_OK;
  if (!c->ops.host_buffers) {
    if (c->ops.allreduce_sum(c->ops.user, d_buf, count, dtype, st) != 0) {
      set_error("comm allreduce callback failed");
      return LOAM_ERR_HIP;
    }
    return LOAM_OK;
  }
  const size_t bytes = (size_t)count * dtype_size(dtype);
  TRY(ensure_staging(c, bytes, bytes));
  LOAM_HIP(hipMemcpyAsync(c->h_send, d_buf, bytes, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipStreamSynchronize(st));
  if (c->ops.allreduce_sum(c->ops.user, c->h_send, count, dtype, nullptr) != 0) {
    set_error("comm allreduce callback failed");
    return LOAM_ERR_HIP;
  }
  LOAM_HIP(hipMemcpyAsync(d_buf, c->h_send, bytes, hipMemcpyHostToDevice, st));
  return LOAM_OK;
}

int32_t comm_allgather(loam_comm* c, const void* d_send, void* d_recv, int64_t bytes, hipStream_t st) {
  if (!c || bytes < 0) {
    set_error("comm allgather: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (bytes == 0) return LOAM_OK;
  if (c->kind == 2 && c->size > 1) return local_allgather(c, d_send, d_recv, bytes, st);
  if (c->kind == 1)
    return rccl_check(rccl().all_gather(d_send, d_recv, (size_t)bytes, ncclUint8, static_cast<ncclComm_t>(c->nccl), st),
                      "ncclAllGather");
  if (c->size == 1) {
    if (d_recv != d_send) LOAM_HIP(hipMemcpyAsync(d_recv, d_send, (size_t)bytes, hipMemcpyDeviceToDevice, st));
    return LOAM_OK;
  }
  if (!c->ops.host_buffers) {
    if (c->ops.allgather(c->ops.user, d_send, d_recv, bytes, st) != 0) {
      set_error("comm allgather callback failed");
      return LOAM_ERR_HIP;
    }
    return LOAM_OK;
  }
  const size_t total = (size_t)bytes * c->size;
  TRY(ensure_staging(c, (size_t)bytes, total));
  LOAM_HIP(hipMemcpyAsync(c->h_send, d_send, (size_t)bytes, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipStreamSynchronize(st));
  if (c->ops.allgather(c->ops.user, c->h_send, c->h_recv, bytes, nullptr) != 0) {
    set_error("comm allgather callback failed");
    return LOAM_ERR_HIP;
  }
  LOAM_HIP(hipMemcpyAsync(d_recv, c->h_recv, total, hipMemcpyHostToDevice, st));
  // the staging buffers are reused by the next call only after its own stream sync
  return LOAM_OK;
}

}  // namespace loam

extern "C" {

int32_t loam_comm_create(int32_t rank, int32_t size, const loam_comm_ops* ops, loam_comm** out) {
  if (!out || size < 1 || rank < 0 || rank >= size || (size > 1 && (!ops || !ops->allreduce_sum || !ops->allgather))) {
    loam::set_error("loam_comm_create: bad arguments");
    return LOAM_ERR_ARG;
  }
  auto* c = new loam_comm;
  c->rank = rank;
  c->size = size;
  c->kind = 0;
  if (ops) c->ops = *ops;
  *out = c;
  return LOAM_OK;
}

int32_t loam_comm_rccl_unique_id(uint8_t* id) {
  if (!id) return LOAM_ERR_ARG;
  if (!rccl().ok) {
    loam::set_error(rccl().err);
    return LOAM_ERR_NODEVICE;
  }
  ncclUniqueId u;
  TRY(rccl_check(rccl().get_unique_id(&u), "ncclGetUniqueId"));
  std::memcpy(id, u.internal, LOAM_RCCL_ID_BYTES);
  return LOAM_OK;
}

int32_t loam_comm_create_rccl(int32_t rank, int32_t size, const uint8_t* id, int32_t device, loam_comm** out) {
  if (!out || !id || size < 1 || rank < 0 || rank >= size) {
    loam::set_error("loam_comm_create_rccl: bad arguments");
    return LOAM_ERR_ARG;
  }
  *out = nullptr;
  TRY(loam::ensure_device(device));
  if (!rccl().ok) {
    loam::set_error(rccl().err);
    return LOAM_ERR_NODEVICE;
  }
  LOAM_HIP(hipSetDevice(device));
  ncclUniqueId u;
  std::memcpy(u.internal, id, LOAM_RCCL_ID_BYTES);
  ncclComm_t comm = nullptr;
  TRY(rccl_check(rccl().comm_init_rank(&comm, size, u, rank), "ncclCommInitRank"));
  auto* c = new loam_comm;
  c->rank = rank;
  c->size = size;
  c->kind = 1;
  c->nccl = comm;
  c->device = device;
  *out = c;
  return LOAM_OK;
}

int32_t loam_comm_create_local(int32_t size, int32_t device, loam_comm** out) {
  if (!out || size < 1 || size > LOAM_LOCAL_MAX_RANKS) {
    loam::set_error("loam_comm_create_local: bad arguments");
    return LOAM_ERR_ARG;
  }
  TRY(loam::ensure_device(device));
  LOAM_HIP(hipSetDevice(device));
  auto* G = new loam::LocalGroup;
  G->size = size;
  G->device = device;
  G->alive = size;
  bool ok = hipEventCreateWithFlags(&G->ev_post, hipEventDisableTiming) == hipSuccess;
  for (int r = 0; r < size && ok; ++r) ok = hipEventCreateWithFlags(&G->ev_pre[r], hipEventDisableTiming) == hipSuccess;
  for (int p = 0; p < 2 && ok; ++p)
    for (int r = 0; r < size && ok; ++r)
      ok = hipEventCreateWithFlags(&G->evA[p][r], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&G->evB[p][r], hipEventDisableTiming) == hipSuccess;
  if (!ok) {  // the events created so far, then the group
    loam::local_group_free_events(*G);
    delete G;
    loam::set_error("loam_comm_create_local: hipEventCreate failed");
    return LOAM_ERR_HIP;
  }
  for (int r = 0; r < size; ++r) {
    auto* c = new loam_comm;
    c->rank = r;
    c->size = size;
    c->kind = 2;
    c->local = G;
    c->device = device;
    out[r] = c;
  }
  return LOAM_OK;
}

int32_t loam_comm_destroy(loam_comm* c) {
  if (!c) return LOAM_ERR_ARG;
  if (c->kind == 2 && c->local) {
    loam::LocalGroup* G = c->local;
    bool last;
    {
      std::lock_guard<std::mutex> lk(G->mu);
      last = --G->alive == 0;
      // a rank leaving while others live ends the group: their next collective fails at once
      G->broken = true;
      G->cv.notify_all();
    }
    if (last) {
      (void)hipSetDevice(G->device);
      (void)hipDeviceSynchronize();
      for (int p = 0; p < 2; ++p)
        for (int r = 0; r < G->size; ++r)
          if (G->stage[p][r]) (void)hipFree(G->stage[p][r]);
      loam::local_group_free_events(*G);
      if (G->peer) (void)hipFree(G->peer);
      delete G;
    }
    delete c;
    return LOAM_OK;
  }
  if (c->kind == 1 && c->nccl) {
    (void)hipSetDevice(c->device);
    (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->nccl));
  }
  if (c->h_send) (void)hipHostFree(c->h_send);
  if (c->h_recv) (void)hipHostFree(c->h_recv);
  delete c;
  return LOAM_OK;
}

int32_t loam_comm_allreduce_sum(loam_comm* c, void* d_buf, int64_t count, int32_t dtype, void* hip_stream) {
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  TRY(loam::comm_allreduce(c, d_buf, count, dtype, st));
  LOAM_HIP(hipStreamSynchronize(st));
  return LOAM_OK;
}

int32_t loam_comm_allgather(loam_comm* c, const void* d_send, void* d_recv, int64_t bytes, void* hip_stream) {
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  TRY(loam::comm_allgather(c, d_send, d_recv, bytes, st));
  LOAM_HIP(hipStreamSynchronize(st));
  return LOAM_OK;
}

}  // extern "C"
