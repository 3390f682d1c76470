// cellhash.h — 1 m voxel hash over a point set + exact radius-bounded kNN-5.
//
// Replaces pcl::KdTreeFLANN::nearestKSearch(k = 5) of laser_mapping.cpp:554/:633.  The
// reference only accepts a neighbourhood whose 5th neighbour has sqDis < 1.0 (:557, :642),
// so an exact answer needs only the points within 1 m of the query: the 27 cells around
// it.  Distances are FLANN's L2_Simple<float>; ties are broken by point index.
//
// Table entries are epoch-tagged (key and count words carry the build's epoch in their high
// 32 bits), so a table never needs clearing between frames: a slot whose epoch is not the
// current one is empty.  The build uses (key, count) words; queries read a packed 16-byte
// entry per slot written once the cell starts are known.
#pragma once
#include "common.h"
#include "device_math.h"

namespace loam {

__device__ inline uint32_t cell_key_rel(float px, float py, float pz, const int* origin) {
  int cx = (int)floorf(px) - origin[0];
  int cy = (int)floorf(py) - origin[1];
  int cz = (int)floorf(pz) - origin[2];
  cx = min(max(cx, 0), 511);
  cy = min(max(cy, 0), 511);
  cz = min(max(cz, 0), 511);
  return (uint32_t)cx | ((uint32_t)cy << 9) | ((uint32_t)cz << 18);
}

__device__ inline uint32_t cell_hash(uint32_t k, uint32_t mask) {
  uint32_t h = k * 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h & mask;
}

// claim (or find) the slot of `key` and take a rank within the cell; false if the table is full
__device__ inline bool hash_claim_rank(unsigned long long* hk, unsigned long long* hc, uint32_t mask,
                                       uint32_t epoch, uint32_t key, uint32_t* slot_out,
                                       uint32_t* rank_out) {
  const unsigned long long ep = (unsigned long long)epoch << 32;
  const unsigned long long want = ep | key;
  uint32_t h = cell_hash(key, mask);
  uint32_t slot = 0xFFFFFFFFu;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    unsigned long long cur = __hip_atomic_load(&hk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == want) {
      slot = h;
      break;
    }
    if ((cur >> 32) != epoch) {
      // stale slot: only current-epoch values ever replace it, so a failed CAS means the
      // slot now holds a current-epoch key (ours or another cell's)
      unsigned long long prev = atomicCAS(&hk[h], cur, want);
      if (prev == cur || prev == want) {
        slot = h;
        break;
      }
    }
    h = (h + 1) & mask;
  }
  if (slot == 0xFFFFFFFFu) return false;
  unsigned long long c = __hip_atomic_load(&hc[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    const bool fresh = (c >> 32) == epoch;
    const unsigned long long nc = fresh ? c + 1 : (ep | 1ull);
    const unsigned long long prev = atomicCAS(&hc[slot], c, nc);
    if (prev == c) {
      *rank_out = fresh ? (uint32_t)(c & 0xFFFFFFFFu) : 0u;
      break;
    }
    c = prev;
  }
  *slot_out = slot;
  return true;
}

// claim (or find) the slot of `key` and add `count` points to the cell; *base_out = the
// cell's count before the addition (the rank of this batch's first point), *fresh_out =
// whether this call started the cell in this epoch.  False if the table is full.
__device__ inline bool hash_claim_cell(unsigned long long* hk, unsigned long long* hc, uint32_t mask,
                                       uint32_t epoch, uint32_t key, uint32_t count, uint32_t* slot_out,
                                       uint32_t* base_out, bool* fresh_out) {
  const unsigned long long ep = (unsigned long long)epoch << 32;
  const unsigned long long want = ep | key;
  uint32_t h = cell_hash(key, mask);
  uint32_t slot = 0xFFFFFFFFu;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    unsigned long long cur = __hip_atomic_load(&hk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == want) {
      slot = h;
      break;
    }
    if ((cur >> 32) != epoch) {
      unsigned long long prev = atomicCAS(&hk[h], cur, want);
      if (prev == cur || prev == want) {
        slot = h;
        break;
      }
    }
    h = (h + 1) & mask;
  }
  if (slot == 0xFFFFFFFFu) return false;
  unsigned long long c = __hip_atomic_load(&hc[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    const bool fresh = (c >> 32) != epoch;
    const unsigned long long nc = fresh ? (ep | count) : c + count;
    const unsigned long long prev = atomicCAS(&hc[slot], c, nc);
    if (prev == c) {
      *base_out = fresh ? 0u : (uint32_t)(c & 0xFFFFFFFFu);
      *fresh_out = fresh;
      break;
    }
    c = prev;
  }
  *slot_out = slot;
  return true;
}

// Cell start allocation with one atomic per wave, and the packed query entry
// {key, epoch, start, count} (one 16-byte load per probe on the query side).  Called by
// whole waves: lanes with first = false (not the cell's rank-0 point, or past the end)
// take part in the scan with a zero count.
__device__ inline void hash_alloc_cell(bool first, uint32_t slot, const unsigned long long* hk,
                                       const unsigned long long* hc, uint32_t epoch, uint32_t* hs,
                                       uint4* qt, uint32_t* cursor) {
  const uint32_t cnt = first ? (uint32_t)(hc[slot] & 0xFFFFFFFFu) : 0u;
  const uint32_t inc = wave_incl_scan_u(cnt);
  const uint32_t tot = __shfl(inc, 63, 64);
  uint32_t base = 0;
  if ((threadIdx.x & 63) == 0 && tot) base = atomicAdd(cursor, tot);
  base = __shfl(base, 0, 64);
  if (first) {
    const uint32_t st = base + inc - cnt;
    hs[slot] = st;
    qt[slot] = make_uint4((uint32_t)(hk[slot] & 0xFFFFFFFFu), epoch, st, cnt);
  }
}

struct Top5 {
  float d[5];
  int id[5];
};

__device__ inline bool knn_less(float d, int i, float d2, int i2) {
  return d < d2 || (d == d2 && i < i2);
}

__device__ inline void top5_offer(Top5& T, float d, int id) {
  if (!knn_less(d, id, T.d[4], T.id[4])) return;
  T.d[4] = d; T.id[4] = id;
#pragma unroll
  for (int k = 4; k > 0; --k) {
    if (knn_less(T.d[k], T.id[k], T.d[k - 1], T.id[k - 1])) {
      float td = T.d[k]; T.d[k] = T.d[k - 1]; T.d[k - 1] = td;
      int ti = T.id[k]; T.id[k] = T.id[k - 1]; T.id[k - 1] = ti;
    }
  }
}

// the 27 neighbour cells, nearest first (own cell, 6 faces, 12 edges, 8 corners), so the
// 5th distance shrinks early and the gap test prunes more.  Cell o's code is 6 bits at
// (o mod 10) * 6 of word o / 10; code = (dx+1) | (dy+1) << 2 | (dz+1) << 4.
__device__ inline uint32_t cell_order_code(int o) {
  const unsigned long long w = o < 10 ? 0x612425159456515ull : (o < 20 ? 0x2984906690611aull : 0x2aa2280a202ull);
  return (uint32_t)(w >> (6 * (o % 10))) & 63u;
}

// 5 nearest (ascending (d2, index)) among points with d2 below ~radius2 (<= 1): sp holds the
// cell-sorted points with w = point index bits; qt the packed cell entries.
__device__ inline void knn5_hash(const float4 q, const int* origin, const uint4* qt,
                                 const float4* sp, uint32_t mask, uint32_t epoch, float radius2,
                                 Top5& T, uint32_t* ncand = nullptr) {
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    T.d[k] = INFINITY;
    T.id[k] = 0x7FFFFFFF;
  }
  const float fx = floorf(q.x), fy = floorf(q.y), fz = floorf(q.z);
  const int cx = (int)fx - origin[0], cy = (int)fy - origin[1], cz = (int)fz - origin[2];
  // distance from q to the faces of its own cell, for pruning the 26 neighbours
  const float lx = q.x - fx, hx = (fx + 1.0f) - q.x;
  const float ly = q.y - fy, hy = (fy + 1.0f) - q.y;
  const float lz = q.z - fz, hz = (fz + 1.0f) - q.z;
  for (int o = 0; o < 27; ++o) {
    const uint32_t code = cell_order_code(o);
    const int dx = (int)(code & 3u) - 1, dy = (int)((code >> 2) & 3u) - 1, dz = (int)(code >> 4) - 1;
    const int x = cx + dx, y = cy + dy, z = cz + dz;
    if ((uint32_t)x > 511u || (uint32_t)y > 511u || (uint32_t)z > 511u) continue;
    const float gx = dx < 0 ? lx : (dx > 0 ? hx : 0.f);
    const float gy = dy < 0 ? ly : (dy > 0 ? hy : 0.f);
    const float gz = dz < 0 ? lz : (dz > 0 ? hz : 0.f);
    const float gap2 = gx * gx + gy * gy + gz * gz;
    // a point in that cell is at least gap away; 1% + 1e-6 margin covers float rounding
    const float bound = fminf(T.d[4], radius2) * 1.01f + 1e-6f;
    if (gap2 > bound) continue;
    const uint32_t key = (uint32_t)x | ((uint32_t)y << 9) | ((uint32_t)z << 18);
    uint32_t h = cell_hash(key, mask);
    while (true) {
      const uint4 e = qt[h];
      if (e.y != epoch) break;  // empty in this epoch: cell absent
      if (e.x == key) {
        if (ncand) *ncand += e.w;
        uint32_t j = 0;
        for (; j + 2 <= e.w; j += 2) {  // two loads in flight
          const float4 p0 = sp[e.z + j], p1 = sp[e.z + j + 1];
          top5_offer(T, fdist2(q.x, q.y, q.z, p0.x, p0.y, p0.z), __float_as_int(p0.w));
          top5_offer(T, fdist2(q.x, q.y, q.z, p1.x, p1.y, p1.z), __float_as_int(p1.w));
        }
        if (j < e.w) {
          const float4 p0 = sp[e.z + j];
          top5_offer(T, fdist2(q.x, q.y, q.z, p0.x, p0.y, p0.z), __float_as_int(p0.w));
        }
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

}  // namespace loam
