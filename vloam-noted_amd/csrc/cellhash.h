// cellhash.h — 1 m voxel hash over a point set + exact radius-bounded kNN-5.
//
// Replaces pcl::KdTreeFLANN::nearestKSearch(k = 5) of laser_mapping.cpp:554/:633.  The
// reference only accepts a neighbourhood whose 5th neighbour has sqDis < 1.0 (:557, :642),
// so an exact answer needs only the points within 1 m of the query: the 27 cells around
// it.  Distances are FLANN's L2_Simple<float>; ties are broken by point index.
//
// Table entries are epoch-tagged (key and count words carry the build's epoch in their high
// 32 bits), so a table never needs clearing between frames: a slot whose epoch is not the
// current one is empty.
#pragma once
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

struct Top5 {
  float d[5];
  int id[5];
  float x[5], y[5], z[5];
};

__device__ inline bool knn_less(float d, int i, float d2, int i2) {
  return d < d2 || (d == d2 && i < i2);
}

__device__ inline void top5_offer(Top5& T, float d, int id, float px, float py, float pz) {
  if (!knn_less(d, id, T.d[4], T.id[4])) return;
  T.d[4] = d; T.id[4] = id; T.x[4] = px; T.y[4] = py; T.z[4] = pz;
#pragma unroll
  for (int k = 4; k > 0; --k) {
    if (knn_less(T.d[k], T.id[k], T.d[k - 1], T.id[k - 1])) {
      float td = T.d[k]; T.d[k] = T.d[k - 1]; T.d[k - 1] = td;
      int ti = T.id[k]; T.id[k] = T.id[k - 1]; T.id[k - 1] = ti;
      float tx = T.x[k]; T.x[k] = T.x[k - 1]; T.x[k - 1] = tx;
      float ty = T.y[k]; T.y[k] = T.y[k - 1]; T.y[k - 1] = ty;
      float tz = T.z[k]; T.z[k] = T.z[k - 1]; T.z[k - 1] = tz;
    }
  }
}

// 5 nearest (ascending (d2, index)) among points with d2 below ~radius2 (<= 1): sp holds the
// cell-sorted points with w = point index bits.
__device__ inline void knn5_hash(const float4 q, const int* origin, const unsigned long long* hk,
                                 const unsigned long long* hc, const uint32_t* hs,
                                 const float4* sp, uint32_t mask, uint32_t epoch, float radius2,
                                 Top5& T, uint32_t* ncand = nullptr) {
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    T.d[k] = INFINITY;
    T.id[k] = 0x7FFFFFFF;
    T.x[k] = T.y[k] = T.z[k] = 0.f;
  }
  const float fx = floorf(q.x), fy = floorf(q.y), fz = floorf(q.z);
  const int cx = (int)fx - origin[0], cy = (int)fy - origin[1], cz = (int)fz - origin[2];
  // distance from q to the faces of its own cell, for pruning the 26 neighbours
  const float lx = q.x - fx, hx = (fx + 1.0f) - q.x;
  const float ly = q.y - fy, hy = (fy + 1.0f) - q.y;
  const float lz = q.z - fz, hz = (fz + 1.0f) - q.z;
  const unsigned long long ep = (unsigned long long)epoch << 32;
  for (int dz = -1; dz <= 1; ++dz) {
    const int z = cz + dz;
    if (z < 0 || z > 511) continue;
    const float gz = dz < 0 ? lz : (dz > 0 ? hz : 0.f);
    for (int dy = -1; dy <= 1; ++dy) {
      const int y = cy + dy;
      if (y < 0 || y > 511) continue;
      const float gy = dy < 0 ? ly : (dy > 0 ? hy : 0.f);
      for (int dx = -1; dx <= 1; ++dx) {
        const int x = cx + dx;
        if (x < 0 || x > 511) continue;
        const float gx = dx < 0 ? lx : (dx > 0 ? hx : 0.f);
        const float gap2 = gx * gx + gy * gy + gz * gz;
        // a point in that cell is at least gap away; 1% + 1e-6 margin covers float rounding
        const float bound = fminf(T.d[4], radius2) * 1.01f + 1e-6f;
        if (gap2 > bound) continue;
        const uint32_t key = (uint32_t)x | ((uint32_t)y << 9) | ((uint32_t)z << 18);
        const unsigned long long want = ep | key;
        uint32_t h = cell_hash(key, mask);
        while (true) {
          const unsigned long long cur = hk[h];
          if (cur == want) {
            const uint32_t cnt = (uint32_t)(hc[h] & 0xFFFFFFFFu);
            const uint32_t st = hs[h];
            if (ncand) *ncand += cnt;
            for (uint32_t j = 0; j < cnt; ++j) {
              const float4 p = sp[st + j];
              const float d = fdist2(q.x, q.y, q.z, p.x, p.y, p.z);
              top5_offer(T, d, __float_as_int(p.w), p.x, p.y, p.z);
            }
            break;
          }
          if ((cur >> 32) != epoch) break;  // empty in this epoch: cell absent
          h = (h + 1) & mask;
        }
      }
    }
  }
}

}  // namespace loam
