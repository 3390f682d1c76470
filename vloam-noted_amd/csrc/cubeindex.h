// cubeindex.h — persistent 1 m cell index of every map cube (replaces the per-frame KD-tree
// build of laser_mapping.cpp:519-520).
//
// A cube's content lives at arena[off .. off + n) in the reference order (VoxelGrid output
// order: the submap index of laser_mapping.cpp:448-489 is sub_off[window slot] + position).
// Its index is kept at the same offsets in two parallel arenas:
//   cpts[off + k]      the points sorted by 1 m cell, w = position in the cube (int bits)
//   ctab[4*off + h]    open-addressing table of the cube's cells, T = next_pow2(2n) <= 4n
//                      entries: x = local cell key | count << 18, y = start (in cpts)
// so moving content (compaction) moves its index verbatim and the table size needs no
// descriptor.  The index is rebuilt whenever a cube's content is rewritten (k_revox) or
// set through the API; unchanged cubes keep theirs across frames.
//
// Local cell coordinates are relative to the cube's lower corner, (cube - cen) * 50 - 25 m
// per axis.  The reference's cube rule (laser_mapping.cpp:747-756: int((v + 25) / 50), minus
// one when v + 25 < 0) files a point with v + 25 an exact negative multiple of 50 in the cube
// below, where its local coordinate is 50: 6 bits per axis hold 0..50.
#pragma once
#include "common.h"
#include "device_math.h"

namespace loam {

constexpr uint32_t CI_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t CI_KEY_MASK = (1u << 18) - 1;
constexpr int CI_LDS_MAX_T = 32768;  // table entries built in LDS (one packed word each)

__host__ __device__ inline uint32_t ci_table_size(uint32_t n) {
  uint32_t t = 1;
  while (t < 2 * n) t <<= 1;
  return t;
}
__device__ inline uint32_t ci_hash(uint32_t k, uint32_t mask) {
  uint32_t h = k * 0x9E3779B1u;
  h ^= h >> 15;
  return h & mask;
}
// lower corner (integer metres) of the cube whose grid index is c along an axis with centre cen
__device__ inline int ci_corner(int c, int cen) { return (c - cen) * 50 - 25; }
__device__ inline uint32_t ci_local_key(const float4& p, const int corner[3]) {
  const int lx = (int)floorf(p.x) - corner[0], ly = (int)floorf(p.y) - corner[1], lz = (int)floorf(p.z) - corner[2];
  return (uint32_t)(lx & 63) | ((uint32_t)(ly & 63) << 6) | ((uint32_t)(lz & 63) << 12);
}

// block-wide exclusive scan (nthreads threads); ws: nthreads / 64 + 1 LDS words
template <int nthreads>
__device__ inline uint32_t ci_block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  constexpr int W = nthreads / 64;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t inc = wave_incl_scan_u(v);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < W; ++w) {
      const uint32_t t = ws[w];
      ws[w] = acc;
      acc += t;
    }
    ws[W] = acc;
  }
  __syncthreads();
  const uint32_t r = ws[wid] + inc - v;
  *total = ws[W];
  __syncthreads();
  return r;
}

// Build the index of one cube (whole workgroup of nthreads, n points at pts).  lds: at least
// CI_LDS_MAX_T + nthreads / 64 + 1 words.  Cubes with 2n > CI_LDS_MAX_T build their
// table in global memory.  Returns false if a cell holds more points than the entry can
// count (2^14 - 1).
template <int nthreads, int MAXT = CI_LDS_MAX_T>
__device__ inline bool cube_index_build(const float4* pts, uint32_t n, const int corner[3], float4* cpts,
                                        uint2* ctab, uint32_t* lds, unsigned long long* prof = nullptr) {
  const int tid = threadIdx.x;
  if (n == 0) return true;
  const uint32_t T = ci_table_size(n), mask = T - 1;
  uint32_t* ws = lds + MAXT;
  bool ok = true;
  if (prof && tid == 0 && T <= (uint32_t)MAXT && n < (1u << 14)) atomicAdd(prof, 0ull - __builtin_readcyclecounter());
  if (T <= (uint32_t)MAXT && n < (1u << 14)) {  // counts fit the packed word
    uint32_t* lent = lds;  // key | count << 18 (count < n <= 2^14)
    for (uint32_t i = tid; i < T; i += nthreads) lent[i] = CI_EMPTY;
    __syncthreads();
    // 1. cells + per-point rank, kept in registers (n <= MAXT / 2 here); the keys first, so
    //    every load is in flight before the first LDS atomic
    constexpr int PER = (MAXT / 2 + nthreads - 1) / nthreads;
    // loads CI_LOADS at a time from a clamped index, no branch between them: a load under `if
    // (i < n)` is waited for inside its branch, one memory latency per row (measured: 16.5k of
    // the build's 64k cycles on a 12k-point cube)
    constexpr int CI_LOADS = PER < 8 ? PER : 8;
    uint32_t sr[PER];
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += CI_LOADS) {
      float4 p[CI_LOADS];
#pragma unroll
      for (int u = 0; u < CI_LOADS; ++u) p[u] = pts[min(tid + (uint32_t)(k0 + u) * nthreads, n - 1)];
#pragma unroll
      for (int u = 0; u < CI_LOADS; ++u)
        sr[k0 + u] = tid + (uint32_t)(k0 + u) * nthreads < n ? ci_local_key(p[u], corner) : CI_EMPTY;
    }
    // a cube's points come in VoxelGrid order (z, y, x rows), so neighbouring lanes often share a
    // cell: each run of equal keys in a wave takes its ranks with one table update by its first
    // lane (the order of points within a cell is free: kNN ties go by cube position, k_knn)
    const int lane = tid & 63;
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= this one
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t key = sr[k];
      const uint32_t prev = (uint32_t)__shfl_up((int)key, 1, 64);
      const uint64_t heads = __ballot(lane == 0 || prev != key);
      const int head = 63 - __clzll(heads & le);  // this lane's run starts here
      uint32_t base = 0;
      if (key != CI_EMPTY && head == lane) {
        const uint64_t after = heads & ~le;
        const uint32_t run = (uint32_t)((after ? __ffsll((long long)after) - 1 : 64) - lane);
        uint32_t h = ci_hash(key, mask);
        while (true) {
          const uint32_t old = atomicCAS(&lent[h], CI_EMPTY, key | (run << 18));
          if (old == CI_EMPTY) break;
          if ((old & CI_KEY_MASK) == key) {
            base = atomicAdd(&lent[h], run << 18) >> 18;
            break;
          }
          h = (h + 1) & mask;
        }
        base |= h << 15;  // slot < 2^15, rank < n <= 2^14
      }
      const uint32_t hb = (uint32_t)__shfl((int)base, head, 64);
      sr[k] = key == CI_EMPTY ? CI_EMPTY : hb + (uint32_t)(lane - head);
    }
    __syncthreads();
    if (prof && tid == 0) atomicAdd(prof, __builtin_readcyclecounter());  // minus the start below
    // 2. starts: exclusive scan of the counts over the slots a thread owns (tid, tid + nthreads,
    //    ...: the cells' order in cpts is free, and the table writes coalesce); the LDS word
    //    becomes the start
    uint32_t sum = 0;
    for (uint32_t h = tid; h < T; h += nthreads) {
      const uint32_t e = lent[h];
      if (e != CI_EMPTY) sum += e >> 18;
    }
    uint32_t tot;
    uint32_t pre = ci_block_scan<nthreads>(sum, ws, &tot);
    for (uint32_t h = tid; h < T; h += nthreads) {
      const uint32_t e = lent[h];
      ctab[h] = make_uint2(e, pre);
      lent[h] = pre;
      if (e != CI_EMPTY) pre += e >> 18;
    }
    __syncthreads();
    // 3. points by cell (loads batched as in 1.)
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += CI_LOADS) {
      float4 p[CI_LOADS];
#pragma unroll
      for (int u = 0; u < CI_LOADS; ++u) p[u] = pts[min(tid + (uint32_t)(k0 + u) * nthreads, n - 1)];
#pragma unroll
      for (int u = 0; u < CI_LOADS; ++u) {
        const uint32_t i = tid + (uint32_t)(k0 + u) * nthreads;
        if (i < n) cpts[lent[sr[k0 + u] >> 15] + (sr[k0 + u] & 0x7FFFu)] = make_float4(p[u].x, p[u].y, p[u].z, __int_as_float((int)i));
      }
    }
    __syncthreads();
    return ok;
  }
  // large cube: the same with the table in global memory (y = count, then start + fill)
  for (uint32_t i = tid; i < T; i += nthreads) ctab[i] = make_uint2(CI_EMPTY, 0);
  __syncthreads();
  for (uint32_t i = tid; i < n; i += nthreads) {
    const uint32_t key = ci_local_key(pts[i], corner);
    uint32_t h = ci_hash(key, mask);
    while (true) {
      const uint32_t old = atomicCAS(&ctab[h].x, CI_EMPTY, key);
      if (old == CI_EMPTY || old == key) break;
      h = (h + 1) & mask;
    }
    atomicAdd(&ctab[h].y, 1u);
  }
  __syncthreads();
  uint32_t sum = 0;
  for (uint32_t h = tid; h < T; h += nthreads) {
    const uint2 e = ctab[h];
    if (e.x != CI_EMPTY) sum += e.y;
  }
  uint32_t tot;
  uint32_t pre = ci_block_scan<nthreads>(sum, ws, &tot);
  for (uint32_t h = tid; h < T; h += nthreads) {
    const uint2 e = ctab[h];
    if (e.x == CI_EMPTY) continue;
    ok &= e.y < (1u << 14);
    ctab[h] = make_uint2(e.x | (e.y << 18), pre);
    pre += e.y;
  }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += nthreads) {  // y: start -> start + count while filling
    const float4 p = pts[i];
    const uint32_t key = ci_local_key(p, corner);
    uint32_t h = ci_hash(key, mask);
    while ((ctab[h].x & CI_KEY_MASK) != key) h = (h + 1) & mask;
    const uint32_t pos = atomicAdd(&ctab[h].y, 1u);
    cpts[pos] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));
  }
  __syncthreads();
  for (uint32_t h = tid; h < T; h += nthreads) {
    const uint2 e = ctab[h];
    if (e.x != CI_EMPTY) ctab[h].y = e.y - (e.x >> 18);
  }
  __syncthreads();
  return ok;
}

// Look up cell (local key) in a cube's table: returns (start, count) or count 0
__device__ inline uint2 ci_find(const uint2* ctab, uint32_t T, uint32_t key) {
  const uint32_t mask = T - 1;
  uint32_t h = ci_hash(key, mask);
  for (uint32_t p = 0; p < T; ++p) {
    const uint2 e = ctab[h];
    if (e.x == CI_EMPTY) break;
    if ((e.x & CI_KEY_MASK) == key) return make_uint2(e.y, e.x >> 18);
    h = (h + 1) & mask;
  }
  return make_uint2(0, 0);
}

}  // namespace loam
