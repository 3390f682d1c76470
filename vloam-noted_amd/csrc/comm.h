// comm.h — the collectives of a sharded mapper (include/loam_core.h, "Sharded LaserMapping").
//
// A loam_comm is RCCL (librccl.so.1 loaded at run time; collectives enqueued on the caller's
// HIP stream, nothing waits on the host) or caller callbacks (device pointers + stream, or
// host buffers: the library drains its stream into pinned staging, calls back, copies back).
#pragma once
#include "common.h"

namespace loam {
struct LocalGroup;
}

struct loam_comm {
  int rank = 0, size = 1;
  int kind = 0;  // 0 callbacks, 1 RCCL, 2 ranks of one process on one device (loam_comm_create_local)
  loam::LocalGroup* local = nullptr;
  uint64_t seq = 0;  // kind 2: collectives this rank has enqueued
  loam_comm_ops ops{};
  void* nccl = nullptr;  // ncclComm_t
  int device = 0;
  // pinned staging of the host-buffer callbacks
  void* h_send = nullptr;
  void* h_recv = nullptr;
  size_t h_cap = 0;
};

namespace loam {

int32_t comm_allreduce(loam_comm* c, void* d_buf, int64_t count, int32_t dtype, hipStream_t st);
int32_t comm_allgather(loam_comm* c, const void* d_send, void* d_recv, int64_t bytes, hipStream_t st);
// a rank's solve failed outside a collective: an in-process group (kind 2) is broken so the other
// ranks fail their next collective at once instead of waiting out the timeout (no-op otherwise:
// RCCL and callback transports own their failure handling)
void comm_abort(loam_comm* c);
// device memory every rank of the group sees at the same address (ranks of one process on one
// device, loam_comm_create_local), bound by every rank's mapper at once (its creation: the host
// threads meet twice, bounded): zeroed at each binding, every rank asks for the same size.
// LOAM_ERR_STATE for transports without one (RCCL, callbacks) and while a rank's earlier mapper
// still holds it (released by comm_peer_release when that mapper is destroyed).  `leaders`: the
// group LM's leader workgroups (one per rank and padded stream), reserved against `capacity` (LM
// workgroups the device holds at once) together with every group bound in this process:
// LOAM_ERR_CAPACITY when they would not all fit at once
int32_t comm_peer_buffer(loam_comm* c, size_t bytes, int leaders, int capacity, void** dev);
void comm_peer_release(loam_comm* c);
// ONE launch for every rank of an in-process group (ranks whose kernels must wait for each other
// on the device: separate launches could sit behind each other in one hardware queue, the HIP
// streams of a process sharing GPU_MAX_HW_QUEUES queues).  Each rank hands its argument blob and
// its stream; rank 0's stream waits for every rank's stream, rank 0 calls fn(blobs, nrank, its
// stream, user), and every other rank's stream then waits for that launch.  The host threads meet
// twice (bounded; LOAM_ERR_SYNC when the group is broken).
typedef void (*comm_group_launch_fn)(const void* const* blobs, int nrank, hipStream_t st, void* user);
int32_t comm_group_launch(loam_comm* c, const void* blob, hipStream_t st, comm_group_launch_fn fn, void* user);

// 4 m voxel-aligned ownership blocks: voxel v = floor(p / leaf) as PCL computes it
// (floorf(p * (1/leaf)), voxel.h); block = floor(v / bv) with bv voxels per block edge, so a
// voxel never straddles two owners and every rank's per-cube VoxelGrid is exact.
__host__ __device__ inline int shard_floor_div(int v, int d) { return v >= 0 ? v / d : -((-v + d - 1) / d); }
__host__ __device__ inline uint32_t shard_mix(uint32_t h) {  // murmur3 finaliser
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ inline int shard_owner(float x, float y, float z, float inv, int bv, int nrank) {
  if (nrank <= 1) return 0;
  const int bx = shard_floor_div((int)floorf(x * inv), bv);
  const int by = shard_floor_div((int)floorf(y * inv), bv);
  const int bz = shard_floor_div((int)floorf(z * inv), bv);
  const uint32_t h = shard_mix((uint32_t)bx * 73856093u ^ (uint32_t)by * 19349663u ^ (uint32_t)bz * 83492791u);
  return (int)(h % (uint32_t)nrank);
}
// voxels per block edge for a leaf (4 m blocks: 10 voxels of 0.4 m, 5 of 0.8 m)
inline int shard_block_voxels(float leaf) {
  const int bv = (int)lroundf(4.0f / leaf);
  return bv < 1 ? 1 : bv;
}

}  // namespace loam
