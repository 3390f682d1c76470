// cubeindex.h — persistent 1 m cell index of every map cube (replaces the per-frame KD-tree
// build of laser_mapping.cpp:519-520), probe-free.
//
// A cube's content lives at arena[off .. off + n) in the reference order (VoxelGrid output
// order: the submap index of laser_mapping.cpp:448-489 is sub_off[window slot] + position).
// Its index is kept at the same offsets in two parallel arenas, so moving content (compaction)
// moves its index verbatim:
//   cpts[off + k]        the points grouped by 1 m cell, w = position in the cube (int bits)
//   dir[8 off + ..]      (the ctab arena as u32 words, 8 per point slot) a brick directory:
//     word 0             words used (the compaction copies that many)
//     word 1             word offset of cstart (0: a tiny cube, no directory: scan all points)
//     words 2 ..         per 64 bricks: occupancy bits (2 words) + occupied bricks before (1)
//     CI_BE ..           per occupied brick (in brick order): its 64-bit cell mask + the index of
//                        its first occupied cell
//     cstart[0 .. cells] cpts position of each occupied cell (brick order, then bit order), and
//                        the total
// Cells are grouped into bricks of 16 x 2 x 2 (x fastest within a brick: the bit of cell
// (x, y, z) is (2 (z & 1) + (y & 1)) 16 + (x & 15)), so the cells x - 1 .. x + 1 of a row (y, z)
// that fall in one brick are a contiguous bit range and their points one contiguous run of cpts:
// a query's 3 x 3 x 3 neighbourhood is 9 row segments (two where a row crosses a brick or cube
// boundary), each found by three dependent loads (occupancy word, brick entry, cstart pair) and
// no probing.  Directory size: 131 + 3 (bricks) + (cells) + 1 words <= 8 n for n >= CI_TINY.
//
// Local cell coordinates are relative to the cube's lower corner, (cube - cen) * 50 - 25 m
// per axis.  The reference's cube rule (laser_mapping.cpp:747-756: int((v + 25) / 50), minus
// one when v + 25 < 0) files a point with v + 25 an exact negative multiple of 50 in the cube
// below, where its local coordinate is 50: 51 cells per axis.
#pragma once
#include "common.h"
#include "device_math.h"

namespace loam {

constexpr int CI_BX = 4, CI_BY = 26, CI_BZ = 26;            // bricks per axis (16 x 2 x 2 cells each)
constexpr int CI_NB = CI_BX * CI_BY * CI_BZ;                 // 2704
constexpr int CI_NW = (CI_NB + 63) / 64;                     // 43 occupancy words
constexpr int CI_OCC = 2;                                    // occupancy (lo, hi, before) triples
constexpr int CI_BE = CI_OCC + 3 * CI_NW;                    // 131: brick entries (lo, hi, first cell)
constexpr uint32_t CI_TINY = 40;                             // fewer points: no directory
constexpr int CI_LDS_WORDS = 2 * CI_NB + CI_NB + 64;         // build scratch before the cell counts

__host__ __device__ inline uint32_t ci_max_words(uint32_t n) { return 8u * n; }
// lower corner (integer metres) of the cube whose grid index is c along an axis with centre cen
__device__ inline int ci_corner(int c, int cen) { return (c - cen) * 50 - 25; }
__device__ inline void ci_local(const float4& p, const int corner[3], int l[3]) {
  l[0] = ((int)floorf(p.x) - corner[0]) & 63;
  l[1] = ((int)floorf(p.y) - corner[1]) & 63;
  l[2] = ((int)floorf(p.z) - corner[2]) & 63;
}
__host__ __device__ inline uint32_t ci_brick(int lx, int ly, int lz) {
  return (uint32_t)(((lz >> 1) * CI_BY + (ly >> 1)) * CI_BX + (lx >> 4));
}
__host__ __device__ inline uint32_t ci_bit(int lx, int ly, int lz) {
  return (uint32_t)((((lz & 1) << 1) | (ly & 1)) << 4) | (uint32_t)(lx & 15);
}
__device__ inline uint64_t ci_below(uint32_t b) { return b ? (~0ull >> (64 - b)) : 0ull; }

// block-wide exclusive scan (nthreads threads); ws: nthreads / 64 + 1 LDS words
template <int nthreads>
__device__ inline uint32_t ci_block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  constexpr int W = nthreads / 64;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t inc = dpp_incl_scan_u(v);
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

// Build the index of one cube (whole workgroup of nthreads; n points at pts).  lds: lds_words
// words; the cell counters live there when the cells fit (lds_words - CI_LDS_WORDS of them),
// else in the directory's own cstart array (global atomics).  Returns false when the directory
// would not fit its 8 n words (n >= 2^16 points; fewer cannot overflow: 131 + 3 bricks + cells
// + 1 <= 131 + 4 n + 1 <= 8 n for n >= CI_TINY); *words_out: the directory's words.
template <int nthreads>
__device__ inline bool cube_index_build(const float4* pts, uint32_t n, const int corner[3], float4* cpts,
                                        uint32_t* dir, uint32_t* lds, uint32_t lds_words,
                                        unsigned long long* prof = nullptr, uint32_t* words_out = nullptr) {
  const int tid = threadIdx.x;
  if (words_out) *words_out = n == 0 ? 0u : (n < CI_TINY ? 2u : 0u);
  if (n == 0) return true;
  if (n < CI_TINY) {  // tiny: the points as they are, scanned whole
    for (uint32_t i = tid; i < n; i += nthreads) {
      const float4 p = pts[i];
      cpts[i] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));
    }
    if (tid == 0) {
      dir[0] = 2;
      dir[1] = 0;
    }
    __syncthreads();
    return true;
  }
  const unsigned long long t0 = prof ? __builtin_readcyclecounter() : 0ull;
  uint64_t* bmask = reinterpret_cast<uint64_t*>(lds);  // [CI_NB] cell masks
  uint32_t* bfirst = lds + 2 * CI_NB;                   // [CI_NB] first cell index
  uint32_t* ws = lds + 3 * CI_NB;                       // scan scratch (64 words)
  uint32_t* lcnt = lds + CI_LDS_WORDS;                  // cell counters, when they fit
  const uint32_t lcap = lds_words > (uint32_t)CI_LDS_WORDS ? lds_words - CI_LDS_WORDS : 0u;
  for (int b = tid; b < CI_NB; b += nthreads) bmask[b] = 0ull;
  __syncthreads();
  // 1. occupied cells
  for (uint32_t i0 = tid; i0 < n; i0 += 4 * nthreads) {
    float4 p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * nthreads < n) p[u] = pts[i0 + u * nthreads];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * nthreads >= n) continue;
      int l[3];
      ci_local(p[u], corner, l);
      atomicOr(reinterpret_cast<unsigned long long*>(&bmask[ci_brick(l[0], l[1], l[2])]),
               1ull << ci_bit(l[0], l[1], l[2]));
    }
  }
  __syncthreads();
  // 2. first cell of every brick, occupied bricks before it: one scan of (cells | bricks << 16)
  constexpr int BPT = (CI_NB + nthreads - 1) / nthreads;  // bricks per thread (consecutive)
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const int b = tid * BPT + k;
    if (b < CI_NB) {
      const uint64_t m = bmask[b];
      v += (uint32_t)__popcll(m) | (m ? (1u << 16) : 0u);
    }
  }
  uint32_t tot;
  uint32_t pre = ci_block_scan<nthreads>(v, ws, &tot);  // (cells < 2^16 for n < 2^16; checked below)
  const uint32_t ncell = tot & 0xFFFFu, nb = tot >> 16;
  const uint32_t cs = (uint32_t)CI_BE + 3u * nb;  // cstart word offset
  const uint32_t words = cs + ncell + 1;
  if (n >= 65536u || words > ci_max_words(n)) return false;  // (uniform)
  if (words_out) *words_out = words;
  for (int k = 0; k < BPT; ++k) {
    const int b = tid * BPT + k;
    if (b >= CI_NB) break;
    const uint64_t m = bmask[b];
    bfirst[b] = pre & 0xFFFFu;
    if (m) {
      const uint32_t e = CI_BE + 3u * (pre >> 16);
      dir[e] = (uint32_t)m;
      dir[e + 1] = (uint32_t)(m >> 32);
      dir[e + 2] = pre & 0xFFFFu;
    }
    pre += (uint32_t)__popcll(m) | (m ? (1u << 16) : 0u);
  }
  // occupancy words: the thread of word w (w < 43) gathers its 64 bricks; the bricks before it
  // are the first brick's scan value (bricks are consecutive per thread, 3 per thread at 1024)
  __syncthreads();
  for (int w = tid; w < CI_NW; w += nthreads) {
    uint64_t occ = 0;
    for (int k = 0; k < 64; ++k) {
      const int b = 64 * w + k;
      if (b < CI_NB && bmask[b]) occ |= 1ull << k;
    }
    dir[CI_OCC + 3 * w] = (uint32_t)occ;
    dir[CI_OCC + 3 * w + 1] = (uint32_t)(occ >> 32);
  }
  {
    // occupied bricks before word w: a second small scan over the 43 words (one wave)
    if (tid < 64) {
      uint32_t c = 0;
      if (tid < CI_NW)
        for (int k = 0; k < 64; ++k) {
          const int b = 64 * tid + k;
          c += (b < CI_NB && bmask[b]) ? 1u : 0u;
        }
      const uint32_t inc = dpp_incl_scan_u(c);
      if (tid < CI_NW) dir[CI_OCC + 3 * tid + 2] = inc - c;
    }
  }
  // 3. cells: counts (LDS when they fit, else the cstart array itself), then exclusive starts
  //    in place (cnt[ncell] = n)
  const bool in_lds = ncell + 1 <= lcap;
  uint32_t* cnt = in_lds ? lcnt : dir + cs;
  for (uint32_t c = tid; c <= ncell; c += nthreads) cnt[c] = 0u;
  __syncthreads();
  auto cell_of = [&](const float4& p) -> uint32_t {
    int l[3];
    ci_local(p, corner, l);
    const uint32_t b = ci_brick(l[0], l[1], l[2]);
    return bfirst[b] + (uint32_t)__popcll(bmask[b] & ci_below(ci_bit(l[0], l[1], l[2])));
  };
  for (uint32_t i = tid; i < n; i += nthreads) atomicAdd(&cnt[cell_of(pts[i])], 1u);
  __syncthreads();
  {
    constexpr int CPT = 16;  // consecutive cells per thread per pass
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 <= ncell; c0 += CPT * nthreads) {
      const uint32_t a0 = c0 + tid * CPT;
      uint32_t cc[CPT], sum = 0;
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        cc[k] = a0 + k < ncell ? cnt[a0 + k] : 0u;
        sum += cc[k];
      }
      uint32_t t2;
      uint32_t x = ci_block_scan<nthreads>(sum, ws, &t2) + base;  // (its barriers order the reads)
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        if (a0 + k <= ncell) {
          cnt[a0 + k] = x;
          if (in_lds) dir[cs + a0 + k] = x;
        }
        x += cc[k];
      }
      base += t2;
      __syncthreads();
    }
  }
  // 4. points by cell (the order inside a cell is free: a query keeps the (d, key) smallest)
  for (uint32_t i = tid; i < n; i += nthreads) {
    const float4 p = pts[i];
    const uint32_t pos = atomicAdd(&cnt[cell_of(p)], 1u);
    cpts[pos] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));
  }
  __syncthreads();
  if (!in_lds) {
    // the fill moved every start to its cell's end (= the next cell's start): shift back by one,
    // a chunk at a time (every read of a chunk before its writes)
    for (int32_t c0 = (int32_t)ncell; c0 > 0; c0 -= nthreads) {
      const int32_t c = c0 - tid;
      const uint32_t prev = c >= 1 ? dir[cs + c - 1] : 0u;
      __syncthreads();
      if (c >= 1) dir[cs + c] = prev;
      __syncthreads();
    }
    if (tid == 0) dir[cs] = 0u;
  }
  if (tid == 0) {
    dir[0] = words;
    dir[1] = cs;
  }
  __syncthreads();
  if (prof && tid == 0) atomicAdd(prof, __builtin_readcyclecounter() - t0);
  return true;
}

}  // namespace loam
