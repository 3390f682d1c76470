// comm.hip — loam_comm: RCCL (run-time loaded) or caller callbacks (include/loam_core.h).
//
// RCCL is resolved with dlopen("librccl.so.1"): in a process that already loaded PyTorch's
// RCCL (same soname) that copy is reused, so the mapper's communicator and torch.distributed
// share one library.  The library links no RCCL at build time, and unsharded use never
// touches it.
#include <dlfcn.h>

#include <cmath>
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

int32_t comm_allreduce(loam_comm* c, void* d_buf, int64_t count, int32_t dtype, hipStream_t st) {
  if (!c || count < 0 || (dtype != LOAM_DT_F64 && dtype != LOAM_DT_I32)) {
    set_error("comm allreduce: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (count == 0) return LOAM_OK;
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

int32_t loam_comm_destroy(loam_comm* c) {
  if (!c) return LOAM_ERR_ARG;
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
