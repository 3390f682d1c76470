// voxel.h — pcl::VoxelGrid<PointXYZI> on the GPU, one 1024-thread workgroup per cloud
// ("segment"), everything staged in the CU's 160 KiB LDS.
//
// Semantics (PCL 1.10 voxel_grid.hpp applyFilter, used at scan_registration.cpp:497-501,
// laser_mapping.cpp:492-500 and :795-808):
//   bbox (min/max) -> inv = 1.0f/leaf -> ijk = (int)(floor(p*inv) - (float)min_b)
//   -> idx = i + j*dx + k*dx*dy -> output voxels in increasing idx, each the float centroid
//   of x, y, z, intensity (sum / (float)n); >INT32_MAX voxels -> input returned unchanged.
// PCL sorts (idx, point) pairs with an unstable std::sort; here (and in the oracle) the
// within-voxel summation order is the input order, so the float sums are reproducible.
//
// Algorithm (per workgroup):
//   1. virtual cloud = src0[0..n0) ++ {src1[i] : tag1[i] == tag}  (stable compaction)
//   2. bbox reduction
//   3. LDS open-addressing hash of the voxel idx -> per-voxel counts (ds atomics)
//   4. compact the U unique voxels, bitonic-sort them by idx (registers, vx_bitonic_regs)
//   5. exclusive scan of counts -> output slots; member lists (u16 in LDS when they fit,
//      else int in global scratch)
//   6. per voxel: members sorted by input index (insertion sort, lists are short and nearly
//      ordered), float sums in that order, centroid -> output
// Capacity: U <= VX_UCAP unique voxels per segment (else *err |= VX_ERR_CAPACITY).
#pragma once
#include "common.h"

namespace loam {

constexpr int VX_THREADS = 1024;
constexpr int VX_WAVES = VX_THREADS / 64;
constexpr int VX_HASH = 16384;  // LDS hash slots (u32 key + u32 count)
constexpr int VX_UCAP = 12288;  // max unique voxels per segment
constexpr uint32_t VX_EMPTY = 0xFFFFFFFFu;
constexpr int VX_ERR_CAPACITY = 1;
constexpr int VX_ERR_OUTPUT = 2;
constexpr int VX_LDS_WORDS = 40960;  // 160 KiB

// PCL's summation order (exact_voxel_order, voxel_hot.h): what the input-order filter records for
// the voxels of 3 or more members ("hot"), whose centroids depend on std::sort's order.  Global
// scratch of one filter; n points.
struct VxHot {
  uint32_t* rk;    // [n] per point: output slot << 1 | hot
  uint32_t* hl;    // [n] the hot voxels' member lists (point indices), grouped by voxel, any order
  uint32_t* hv;    // [3 * cap_h] per hot voxel: output slot, list start, member count
  uint32_t* fpos;  // [n] per hot point: its position after the emulated sort (voxel_hot.h)
  uint32_t cap_h;
  uint64_t* w = nullptr;  // [n] optional: scratch of the sorts over VH_MAX_N points (voxel_hot.h vh_sort_big)
};

struct VoxSeg {
  const float4* src0;
  int n0;
  const float4* src1;  // optional secondary source filtered by tag (tag1 == nullptr: all of it)
  const int* tag1;
  int n1;
  int tag;
  float leaf;
  int append_only;        // 1: no voxelization, copy the virtual cloud
  float4* out;            // output base (fixed) or arena base (with tail)
  uint32_t* tail;         // if set: out += atomicAdd(tail, count)
  uint32_t cap;           // capacity of out (absolute index bound)
  uint32_t* res_off;      // result offset (absolute index into out) — optional
  uint32_t* res_cnt;      // result count — optional
  uint32_t* stable_out = nullptr;  // optional: (result offset + 1) if the output is a VoxelGrid fixed
                          // point (every centroid inside its own voxel), else 0
  float4* scratch_pts;    // gathered secondary points
  int* scratch_idx;       // member lists
  uint32_t* scratch_tail; // if set, scratch slots are allocated from it (per segment)
  uint32_t scratch_cap;
  int* err;
  unsigned long long* prof = nullptr;  // optional: merge phase cycles [bbox, sort, runs, pass A, pass B]
  unsigned long long* prof_seg = nullptr;  // optional: full filter phase cycles [gather + bbox,
                                           // hash, sort + scan, member lists + centroids]
  VxHot hot{};  // exact order (hot.rk set): record the hot voxels instead of summing them (the
                // stable token then covers the cold voxels only; voxel_hot.h)
  // a map cube's merge (vx_merge_fixed_point): its lower corner in whole metres.  Every point of
  // the cube lies within [corner, corner + 50] (laser_mapping.cpp:747-756), so the voxel keys can
  // be taken relative to the corner's voxel instead of the points' bounding box: the same order
  // (PCL's idx is lexicographic in (z, y, x) whatever its origin) without the bounding-box pass;
  // a point outside the margin (content set through the API) falls back to the full filter
  int anchored = 0;
  int anchor[3] = {0, 0, 0};
};

// thread 0 adds the cycles since *t to prof[k] and restarts *t (phase counters; call after a barrier)
__device__ inline void vx_phase(unsigned long long* prof, int k, unsigned long long* t) {
  if (!prof || threadIdx.x != 0) return;
  const unsigned long long now = __builtin_readcyclecounter();
  atomicAdd(&prof[k], now - *t);
  *t = now;
}

__device__ inline uint32_t vx_hash(uint32_t k) { return (k * 0x9E3779B1u) >> (32 - 14); }
// slot of key k in a power-of-two table (mask = size - 1)
__device__ inline uint32_t vx_slot(uint32_t k, uint32_t mask) {
  uint32_t h = k * 0x9E3779B1u;
  h ^= h >> 15;
  return h & mask;
}

// block-wide exclusive scan of one value per thread (VX_THREADS); returns exclusive prefix,
// total in *total.  ws: LDS scratch of >= VX_WAVES + 1 words.
template <int NT>
__device__ inline uint32_t vx_block_scan_t(uint32_t v, uint32_t* ws, uint32_t* total) {
  constexpr int NW = NT / 64;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t inc = wave_incl_scan_u(v);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < NW; ++w) {
      uint32_t t = ws[w];
      ws[w] = acc;
      acc += t;
    }
    ws[NW] = acc;
  }
  __syncthreads();
  uint32_t r = ws[wid] + inc - v;
  *total = ws[NW];
  __syncthreads();
  return r;
}
__device__ inline uint32_t vx_block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  return vx_block_scan_t<VX_THREADS>(v, ws, total);
}

struct VxGeom {
  unsigned long long nvox;  // div_x * div_y * div_z
  float inv;
  int minbx, minby, minbz;
  int mul1, mul2;
  int overflow;
};

__device__ inline uint32_t vx_key(const VxGeom& g, float4 p) {
  int i0 = (int)(floorf(p.x * g.inv) - (float)g.minbx);
  int i1 = (int)(floorf(p.y * g.inv) - (float)g.minby);
  int i2 = (int)(floorf(p.z * g.inv) - (float)g.minbz);
  return (uint32_t)(i0 + i1 * g.mul1 + i2 * g.mul2);
}

struct VxMisc {
  uint32_t sbase[2];
  int sfail;
  int moved;
  uint32_t nbig;
  uint32_t hot_n, hot_l;  // exact order (VxHot): hot voxels recorded, their member-list length
  VxGeom g;
  float bb[VX_WAVES][6];
};
static_assert(sizeof(VxMisc) <= 192 * 4, "misc area");


// a hot voxel (output slot, cnt members member(0 ..)) -> hv / hl / rk.  One thread; counters in M
template <typename MF>
__device__ inline void vh_record(const VxHot& H, VxMisc& M, uint32_t slot, uint32_t cnt, const MF& member) {
  const uint32_t h = atomicAdd(&M.hot_n, 1u);
  const uint32_t st = atomicAdd(&M.hot_l, cnt);
  if (h < H.cap_h) {
    H.hv[3 * h] = slot;
    H.hv[3 * h + 1] = st;
    H.hv[3 * h + 2] = cnt;
  }
  for (uint32_t a = 0; a < cnt; ++a) {
    const uint32_t i = member(a);
    H.hl[st + a] = i;
    H.rk[i] = (slot << 1) | 1u;
  }
}


struct VxSrc {
  const float4* src0;
  int n0;
  const float4* sec;
  __device__ float4 operator()(uint32_t i) const { return (int)i < n0 ? src0[i] : sec[i - n0]; }
};

constexpr uint32_t VX_ALLOC = 0xFFFFFFFFu;     // vx_group: allocate exactly U at the tail
constexpr uint32_t VX_OVERFLOW = 0xFFFFFFFFu;  // vx_group: unique voxels exceed the LDS
constexpr int VX_NB = 2048;                    // idx buckets of the grouped path
constexpr int VX_HIST_WORD = 3 * VX_UCAP;      // LDS words [36864, 38912): bucket histogram
constexpr int VX_GEND_WORD = VX_HIST_WORD + VX_NB;  // [38912, 40704): group ends
constexpr int VX_MAX_GROUPS = VX_LDS_WORDS - 256 - VX_GEND_WORD;

constexpr int VX_UNROLL = 4;

// voxel keys of points i0 + u * VX_THREADS (u < VX_UNROLL), loads issued together; VX_EMPTY
// past the end
__device__ inline void vx_keys4(const VxGeom& g, const VxSrc& P, uint32_t N, uint32_t i0,
                                uint32_t* kk) {
  float4 p[VX_UNROLL];
#pragma unroll
  for (int u = 0; u < VX_UNROLL; ++u) {
    const uint32_t i = i0 + u * VX_THREADS;
    if (i < N) p[u] = P(i);
  }
#pragma unroll
  for (int u = 0; u < VX_UNROLL; ++u) kk[u] = i0 + u * VX_THREADS < N ? vx_key(g, p[u]) : VX_EMPTY;
}

// Member lists, then per voxel: members sorted by input index, float sums in that order,
// centroid -> out[j].
// Returns true if some centroid left its voxel (float rounding): then the output is not a
// fixed point of the filter.  Phases:
//   1. member lists, chunk by chunk with a barrier (members of earlier chunks precede later
//      ones, so each list is nearly sorted); the next chunk's points are loaded before the
//      barrier so the load latency overlaps it
//   2. per voxel: insertion sort of the list by input index; voxels with <= VX_BIG members
//      are summed by their thread (gathers batched 4 at a time)
//   3. voxels with more members: one wave each, 64 member points gathered at once, summed in
//      input order by a shuffle chain (the same float additions, in the same order)
constexpr uint32_t VX_BIG = 128;

template <typename MT>
__device__ inline bool vx_centroids(const VxGeom& g, const VxSrc& P, uint32_t N, MT* members,
                                    uint32_t klo, uint32_t khi, uint32_t U, const uint32_t* ukey,
                                    const uint32_t* uoff, uint32_t* ufill, float4* out,
                                    uint32_t* big_list, uint32_t big_cap, VxMisc& M,
                                    unsigned long long* dprof = nullptr, const VxHot* H = nullptr,
                                    uint32_t rank0 = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  unsigned long long tq = __builtin_readcyclecounter();
  bool moved = false;
  // one chunk per barrier (members of earlier chunks precede later ones, so each list is nearly
  // sorted), the next chunk's point loaded before the barrier.  Measured and not kept: four chunks'
  // loads and lower_bound searches per step, the appends chunk by chunk (the stack VoxelGrid
  // 0.50 -> 0.57-0.62 ms per step at B = 128 and one-stream blocking frames 0.459 -> 0.470 ms,
  // profiles/r6_member_chunks_ab.txt); with the four chunks' appends racing, the lists came out
  // shuffled and their insertion sorts cost more than the pass (profiles/r6_stack_member_pass.txt)
  float4 pn = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((uint32_t)tid < N) pn = P(tid);
  for (uint32_t c = 0; c < N; c += VX_THREADS) {
    const uint32_t i = c + tid;
    const float4 p = pn;
    if (i + VX_THREADS < N) pn = P(i + VX_THREADS);  // next chunk, in flight across the barrier
    if (i < N) {
      const uint32_t k = vx_key(g, p);
      if (k >= klo && k < khi) {
        uint32_t lo = 0, hi = U;  // lower_bound
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (ukey[mid] < k) lo = mid + 1; else hi = mid;
        }
        const uint32_t pos = uoff[lo] + atomicAdd(&ufill[lo], 1u);
        members[pos] = (MT)i;
        if (H) H->rk[i] = (rank0 + lo) << 1;  // the hot ones are re-marked below
      }
    }
    __syncthreads();
  }
  if (tid == 0) M.nbig = 0;
  __syncthreads();
  vx_phase(dprof, 0, &tq);
  for (uint32_t j = tid; j < U; j += VX_THREADS) {
    const uint32_t b = uoff[j];
    const uint32_t n = ufill[j];
    if (H && n >= 3) {  // exact order: summed later in std::sort's order (voxel_hot.h)
      vh_record(*H, M, rank0 + j, n, [&](uint32_t a) { return (uint32_t)members[b + a]; });
      continue;
    }
    for (uint32_t a = 1; a < n; ++a) {  // insertion sort (nearly ordered lists)
      const MT v = members[b + a];
      uint32_t q = a;
      while (q > 0 && members[b + q - 1] > v) {
        members[b + q] = members[b + q - 1];
        --q;
      }
      members[b + q] = v;
    }
    if (n > VX_BIG) {
      const uint32_t e = atomicAdd(&M.nbig, 1u);
      if (e < big_cap) {
        big_list[e] = j;
        continue;
      }
    }
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    for (uint32_t a = 0; a < n; a += 4) {  // gathers issued together, summed in order
      float4 pp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < n) pp[u] = P((uint32_t)members[b + a + u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < n) {
          sx += pp[u].x; sy += pp[u].y; sz += pp[u].z; si += pp[u].w;
        }
    }
    const float fn = (float)n;
    const float4 cc = make_float4(sx / fn, sy / fn, sz / fn, si / fn);
    out[j] = cc;
    moved |= vx_key(g, cc) != ukey[j];
  }
  __syncthreads();
  vx_phase(dprof, 1, &tq);
  const uint32_t nbig = min(M.nbig, big_cap);
  for (uint32_t e = wid; e < nbig; e += VX_WAVES) {
    const uint32_t j = big_list[e];
    const uint32_t b = uoff[j], n = ufill[j];
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;  // every lane keeps the same running sum
    for (uint32_t a = 0; a < n; a += 64) {
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a + lane < n) p = P((uint32_t)members[b + a + lane]);
      const uint32_t m = min(64u, n - a);
      for (uint32_t l = 0; l < m; ++l) {  // lane l's point as scalars (uniform l: v_readlane)
        sx += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), (int)l));
        sy += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), (int)l));
        sz += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), (int)l));
        si += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.w), (int)l));
      }
    }
    if (lane == 0) {
      const float fn = (float)n;
      const float4 cc = make_float4(sx / fn, sy / fn, sz / fn, si / fn);
      out[j] = cc;
      moved |= vx_key(g, cc) != ukey[j];
    }
  }
  return moved;
}

// Steps 3-6 for the points whose voxel idx lies in [klo, khi): LDS hash -> sorted unique
// voxels -> member lists -> centroids written at out[base + j].  out_base == VX_ALLOC:
// allocate exactly U (at *tail or at 0) once U is known.  Returns U, or VX_OVERFLOW (no side
// effects on the output) when the unique voxels do not fit the LDS.
template <int NT, int E, typename KF>
__device__ inline void vx_bitonic_regs(uint64_t* sk, uint64_t* xb0, uint64_t* xb1, uint32_t npad, const KF& key);

__device__ inline uint32_t vx_group(const VoxSeg& S, const VxGeom& g, const VxSrc& P, uint32_t N,
                                    int* members, uint32_t klo, uint32_t khi, uint32_t out_base,
                                    uint32_t lds_limit, uint32_t* lds, uint32_t* ws, VxMisc& M,
                                    int* moved_out, uint32_t rank0 = 0) {
  const int tid = threadIdx.x;
  unsigned long long tp = __builtin_readcyclecounter();
  uint32_t* hkey = lds;
  uint32_t* hcnt = lds + VX_HASH;
  for (int i = tid; i < VX_HASH; i += VX_THREADS) {
    hkey[i] = VX_EMPTY;
    hcnt[i] = 0;
  }
  if (tid == 0) {
    M.sfail = 0;
    M.moved = 0;
  }
  __syncthreads();
  for (uint32_t i0 = tid; i0 < N; i0 += VX_UNROLL * VX_THREADS) {
    uint32_t kk4[VX_UNROLL];
    vx_keys4(g, P, N, i0, kk4);
#pragma unroll
    for (int u = 0; u < VX_UNROLL; ++u) {
      const uint32_t k = kk4[u];
      if (k < klo || k >= khi) continue;  // also skips i >= N (key VX_EMPTY)
      uint32_t h = vx_hash(k);
      int probes = 0;
      while (true) {
        uint32_t old = atomicCAS(&hkey[h], VX_EMPTY, k);
        if (old == VX_EMPTY || old == k) {
          atomicAdd(&hcnt[h], 1u);
          break;
        }
        h = (h + 1) & (VX_HASH - 1);
        if (++probes >= VX_HASH) {
          M.sfail = 1;
          break;
        }
      }
    }
  }
  __syncthreads();
  // compact unique voxels (16 slots per thread), bitonic sort by idx
  constexpr int SPT = VX_HASH / VX_THREADS;  // 16
  uint32_t mk[SPT], mc[SPT];
  uint32_t nm = 0;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    uint32_t slot = tid * SPT + s;
    mk[s] = hkey[slot];
    mc[s] = hcnt[slot];
    nm += (mk[s] != VX_EMPTY) ? 1u : 0u;
  }
  uint32_t U;
  uint32_t mpos = vx_block_scan(nm, ws, &U);
  const int fail = M.sfail;
  __syncthreads();
  vx_phase(S.prof_seg, 1, &tp);
  if (U > VX_UCAP || fail) return VX_OVERFLOW;
  uint32_t Upad = 64;
  while (Upad < U) Upad <<= 1;
  uint64_t* s64 = reinterpret_cast<uint64_t*>(lds);  // overlays the (consumed) hash
#pragma unroll
  for (int s = 0; s < SPT; ++s)
    if (mk[s] != VX_EMPTY) s64[mpos++] = ((uint64_t)mk[s] << 32) | mc[s];
  __syncthreads();
  // sort by idx in registers (E keys per thread; cross-wave stages through the hash area, the
  // one buffer that is free: Upad u64 <= VX_HASH u64); an LDS network above 8192
  {
    auto key = [&](uint32_t i) -> uint64_t { return i < U ? s64[i] : ~0ull; };
    static_assert(8 * VX_THREADS <= VX_HASH, "one-buffer register sort");
    if (Upad <= 1u * VX_THREADS) vx_bitonic_regs<VX_THREADS, 1>(s64, s64, s64, Upad, key);
    else if (Upad <= 2u * VX_THREADS) vx_bitonic_regs<VX_THREADS, 2>(s64, s64, s64, Upad, key);
    else if (Upad <= 4u * VX_THREADS) vx_bitonic_regs<VX_THREADS, 4>(s64, s64, s64, Upad, key);
    else if (Upad <= 8u * VX_THREADS) vx_bitonic_regs<VX_THREADS, 8>(s64, s64, s64, Upad, key);
    else {  // > 8192 unique voxels (rare: full re-filters of the largest cubes): in LDS, as 16
            // keys per thread in registers would spill
      for (uint32_t i = U + tid; i < Upad; i += VX_THREADS) s64[i] = ~0ull;
      __syncthreads();
      for (uint32_t k = 2; k <= Upad; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
          for (uint32_t i = tid; i < Upad; i += VX_THREADS) {
            const uint32_t ixj = i ^ j;
            if (ixj > i) {
              const uint64_t a = s64[i], b = s64[ixj];
              if ((a > b) == ((i & k) == 0)) {
                s64[i] = b;
                s64[ixj] = a;
              }
            }
          }
          __syncthreads();
        }
      }
    }
  }
  // keys / counts -> exclusive offsets (thread t owns entries [t*EPT, (t+1)*EPT))
  constexpr int EPT = VX_UCAP / VX_THREADS;  // 12
  uint32_t kk[EPT], cc[EPT];
  uint32_t csum = 0;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    uint32_t j = tid * EPT + e;
    uint64_t v = j < U ? s64[j] : 0ull;
    kk[e] = (uint32_t)(v >> 32);
    cc[e] = j < U ? (uint32_t)(v & 0xFFFFFFFFu) : 0u;
    csum += cc[e];
  }
  uint32_t tot;
  uint32_t cpre = vx_block_scan(csum, ws, &tot);  // its barriers order the s64 reads
  uint32_t* ukey = lds;  // packed: ukey[U] | uoff[U] | ufill[U] | LDS member lists
  uint32_t* uoff = lds + U;
  uint32_t* ufill = lds + 2 * U;
  vx_phase(S.prof_seg, 2, &tp);
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    uint32_t j = tid * EPT + e;
    if (j < U) {
      ukey[j] = kk[e];
      uoff[j] = cpre;
      ufill[j] = 0;
    }
    cpre += cc[e];
  }
  __syncthreads();
  uint32_t ob = out_base;
  if (out_base == VX_ALLOC) {
    if (tid == 0) {
      uint32_t b = S.tail ? atomicAdd(S.tail, U) : 0;
      if (b + U > S.cap) {
        atomicOr(S.err, VX_ERR_OUTPUT);
        b = 0xFFFFFFFFu;
      }
      M.sbase[1] = b;
    }
    __syncthreads();
    ob = M.sbase[1];
    if (ob == 0xFFFFFFFFu) return 0;
  }
  // member lists in LDS as u16 point indices when they fit, else in global scratch
  // LDS after the tables: u16 member lists (when they fit), then the big-voxel list
  bool moved;
  const uint32_t mem_words = (N <= 65536u) ? (tot + 1) / 2 : 0u;
  if (N <= 65536u && 3 * U + mem_words + 64 <= lds_limit) {
    uint32_t* big = lds + 3 * U + mem_words;
    moved = vx_centroids(g, P, N, reinterpret_cast<uint16_t*>(lds + 3 * U), klo, khi, U, ukey, uoff,
                         ufill, S.out + ob, big, lds_limit - (3 * U + mem_words), M, S.prof_seg ? S.prof_seg + 4 : nullptr,
                         S.hot.rk ? &S.hot : nullptr, rank0);
  } else {
    uint32_t* big = lds + 3 * U;
    const uint32_t cap = lds_limit > 3 * U ? lds_limit - 3 * U : 0u;
    moved = vx_centroids(g, P, N, members, klo, khi, U, ukey, uoff, ufill, S.out + ob, big, cap, M, nullptr,
                         S.hot.rk ? &S.hot : nullptr, rank0);
  }
  if (moved) M.moved = 1;
  __syncthreads();
  vx_phase(S.prof_seg, 3, &tp);
  *moved_out |= M.moved;
  if (out_base == VX_ALLOC && tid == 0) {
    if (S.res_off) *S.res_off = ob;
    if (S.res_cnt) *S.res_cnt = U;
    if (S.stable_out) *S.stable_out = *moved_out ? 0u : ob + 1;
  }
  __syncthreads();
  return U;
}

// More unique voxels than one LDS pass: histogram the voxel idx over VX_NB buckets, cut the
// idx range into consecutive groups whose unique-voxel bound fits the LDS, run vx_group per
// group in idx order.  The output slot is reserved for N points (upper bound; the arena
// compaction reclaims the slack).
__device__ inline void vx_grouped(const VoxSeg& S, const VxGeom& g, const VxSrc& P, uint32_t N,
                                  int* members, uint32_t* lds, uint32_t* ws, VxMisc& M) {
  const int tid = threadIdx.x;
  uint32_t* hist = lds + VX_HIST_WORD;
  uint32_t* gend = lds + VX_GEND_WORD;
  const unsigned long long V = g.nvox;
  auto bucket = [&](uint32_t k) { return (uint32_t)(((unsigned long long)k * VX_NB) / V); };
  auto blo = [&](uint32_t b) { return (uint32_t)(((unsigned long long)b * V + VX_NB - 1) / VX_NB); };
  for (int b = tid; b < VX_NB; b += VX_THREADS) hist[b] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < N; i += VX_THREADS) atomicAdd(&hist[bucket(vx_key(g, P(i)))], 1u);
  __syncthreads();
  if (tid == 0) {
    int ng = 0, bad = 0;
    uint32_t acc = 0;
    for (int b = 0; b < VX_NB; ++b) {
      uint32_t w = blo(b + 1) - blo(b);
      uint32_t c = hist[b] < w ? hist[b] : w;
      if (c > (uint32_t)VX_UCAP) bad = 1;
      if (acc + c > (uint32_t)VX_UCAP && acc > 0) {
        if (ng < VX_MAX_GROUPS) gend[ng] = b;
        ++ng;
        acc = 0;
      }
      acc += c;
    }
    if (ng < VX_MAX_GROUPS) gend[ng] = VX_NB;
    ++ng;
    if (ng > VX_MAX_GROUPS) bad = 1;
    uint32_t b0 = S.tail ? atomicAdd(S.tail, N) : 0;
    if (b0 + N > S.cap) {
      atomicOr(S.err, VX_ERR_OUTPUT);
      bad = 1;
    }
    if (bad) atomicOr(S.err, VX_ERR_CAPACITY);
    M.sbase[1] = bad ? 0xFFFFFFFFu : b0;
    M.sfail = ng;
  }
  __syncthreads();
  const uint32_t ob = M.sbase[1];
  const int ng = M.sfail;
  __syncthreads();  // every thread has read ng / ob before vx_group reuses M
  if (ob == 0xFFFFFFFFu) return;
  uint32_t acc = 0;
  int gstart = 0;
  int moved = 0;
  for (int gi = 0; gi < ng; ++gi) {
    const int ge = (int)gend[gi];
    const uint32_t U = vx_group(S, g, P, N, members, blo(gstart), ge >= VX_NB ? 0xFFFFFFFFu : blo(ge),
                                ob + acc, VX_HIST_WORD, lds, ws, M, &moved, acc);
    if (U == VX_OVERFLOW) {
      if (tid == 0) atomicOr(S.err, VX_ERR_CAPACITY);
      return;
    }
    acc += U;
    gstart = ge;
  }
  if (tid == 0) {
    if (S.res_off) *S.res_off = ob;
    if (S.res_cnt) *S.res_cnt = acc;
    if (S.stable_out) *S.stable_out = 0;  // slack in the reserved slot: never skipped
  }
}

// block min/max of the per-thread bounds and the grid geometry of leaf -> M.g (all threads;
// result valid after the trailing barrier)
template <int NT = VX_THREADS>
__device__ inline void vx_geometry_finish(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                          float leaf, VxMisc& M) {
  const int tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
  mnx = wave_min_f(mnx); mny = wave_min_f(mny); mnz = wave_min_f(mnz);
  mxx = wave_max_f(mxx); mxy = wave_max_f(mxy); mxz = wave_max_f(mxz);
  float (*sbb)[6] = M.bb;
  if (lane == 0) {
    sbb[wid][0] = mnx; sbb[wid][1] = mny; sbb[wid][2] = mnz;
    sbb[wid][3] = mxx; sbb[wid][4] = mxy; sbb[wid][5] = mxz;
  }
  __syncthreads();
  VxGeom& sg = M.g;
  if (tid == 0) {
    for (int w = 1; w < NT / 64; ++w) {
      mnx = fminf(mnx, sbb[w][0]); mny = fminf(mny, sbb[w][1]); mnz = fminf(mnz, sbb[w][2]);
      mxx = fmaxf(mxx, sbb[w][3]); mxy = fmaxf(mxy, sbb[w][4]); mxz = fmaxf(mxz, sbb[w][5]);
    }
    VxGeom g;
    g.inv = 1.0f / leaf;
    long long dx = (long long)((mxx - mnx) * g.inv) + 1;
    long long dy = (long long)((mxy - mny) * g.inv) + 1;
    long long dz = (long long)((mxz - mnz) * g.inv) + 1;
    g.overflow = (dx * dy * dz > 2147483647LL) ? 1 : 0;
    g.minbx = (int)floorf(mnx * g.inv);
    int maxbx = (int)floorf(mxx * g.inv);
    g.minby = (int)floorf(mny * g.inv);
    int maxby = (int)floorf(mxy * g.inv);
    g.minbz = (int)floorf(mnz * g.inv);
    int divx = maxbx - g.minbx + 1, divy = maxby - g.minby + 1;
    g.mul1 = divx;
    g.mul2 = divx * divy;
    int maxbz = (int)floorf(mxz * g.inv);
    g.nvox = (unsigned long long)divx * (unsigned long long)divy * (unsigned long long)(maxbz - g.minbz + 1);
    sg = g;
  }
  __syncthreads();
}

// bounding box (pcl::getMinMax3D) of the N points P(i) and the grid geometry of leaf -> M.g
template <typename PF, int NT = VX_THREADS>
__device__ inline void vx_geometry(const PF& P, uint32_t N, float leaf, VxMisc& M) {
  const int tid = threadIdx.x;
  float mnx = 3.402823466e38f, mny = 3.402823466e38f, mnz = 3.402823466e38f;
  float mxx = -3.402823466e38f, mxy = -3.402823466e38f, mxz = -3.402823466e38f;
  for (uint32_t i0 = tid; i0 < N; i0 += VX_UNROLL * NT) {
    float4 p[VX_UNROLL];
#pragma unroll
    for (int u = 0; u < VX_UNROLL; ++u)
      if (i0 + u * NT < N) p[u] = P(i0 + u * NT);
#pragma unroll
    for (int u = 0; u < VX_UNROLL; ++u) {
      if (i0 + u * NT >= N) continue;
      mnx = fminf(mnx, p[u].x); mny = fminf(mny, p[u].y); mnz = fminf(mnz, p[u].z);
      mxx = fmaxf(mxx, p[u].x); mxy = fmaxf(mxy, p[u].y); mxz = fmaxf(mxz, p[u].z);
    }
  }
  vx_geometry_finish<NT>(mnx, mny, mnz, mxx, mxy, mxz, leaf, M);
}

// The workgroup routine.  lds: VX_LDS_WORDS u32 words (the whole 160 KiB; the last 256 words
// hold scan scratch + VxMisc).  All threads of the block call it.
__device__ inline void voxel_segment(const VoxSeg& S, uint32_t* lds) {
  const int tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
  uint32_t* ws = lds + VX_LDS_WORDS - 256;  // scan scratch (64 words)
  VxMisc& M = *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192);
  if (tid == 0) {
    M.hot_n = 0;
    M.hot_l = 0;
  }

  // ---- 1. count secondary matches, allocate scratch, gather (stable)
  uint32_t m1 = 0;
  const bool direct = S.src1 && !S.tag1;  // secondary source used whole, no gather
  if (direct) {
    m1 = (uint32_t)max(S.n1, 0);
  } else if (S.src1 && S.n1 > 0) {
    uint32_t local = 0;
    for (int i = tid; i < S.n1; i += VX_THREADS) local += (S.tag1[i] == S.tag) ? 1u : 0u;
    uint32_t tot;
    vx_block_scan(local, ws, &tot);
    m1 = tot;
  }
  const int n0 = S.n0;
  const uint32_t N = (uint32_t)n0 + m1;
  // scratch: gathered secondary points (m1, gather mode) and member lists (N, voxelize mode)
  const uint32_t req = S.append_only ? (direct ? 0u : m1) : N;
  uint32_t* sbase = M.sbase;
  if (tid == 0) {
    uint32_t b = 0;
    if (S.scratch_tail) b = atomicAdd(S.scratch_tail, req);
    if (b + req > S.scratch_cap) {
      atomicOr(S.err, VX_ERR_CAPACITY);
      b = 0xFFFFFFFFu;
    }
    sbase[0] = b;
  }
  __syncthreads();
  const uint32_t sb = sbase[0];
  if (sb == 0xFFFFFFFFu) return;
  float4* sec = direct ? const_cast<float4*>(S.src1) : S.scratch_pts + sb;  // secondary points (m1)
  int* members = S.scratch_idx + sb;  // member lists (N, voxelize mode)
  if (m1 > 0 && !direct) {
    uint32_t base = 0;
    for (int c = 0; c < S.n1; c += VX_THREADS) {
      int i = c + tid;
      bool pred = i < S.n1 && S.tag1[i] == S.tag;
      uint64_t bal = __ballot(pred);
      uint32_t pre = __popcll(bal & lanemask_lt());
      if (lane == 0) ws[wid] = __popcll(bal);
      __syncthreads();
      uint32_t woff = 0, tot = 0;
      for (int w = 0; w < VX_WAVES; ++w) {
        uint32_t t = ws[w];
        if (w < wid) woff += t;
        tot += t;
      }
      if (pred) sec[base + woff + pre] = S.src1[i];
      base += tot;
      __syncthreads();
    }
  }
  __syncthreads();
  auto P = [&](uint32_t i) -> float4 { return (int)i < n0 ? S.src0[i] : sec[i - n0]; };

  // ---- append-only (cube outside the window receiving new points, laser_mapping.cpp:762)
  if (S.append_only || N == 0) {
    if (N == 0 && !S.append_only) {
      if (tid == 0) {
        if (S.res_cnt) *S.res_cnt = 0;
        if (S.stable_out) *S.stable_out = 0;
        if (S.res_off) *S.res_off = 0;
      }
      return;
    }
    if (tid == 0) {
      uint32_t b = S.tail ? atomicAdd(S.tail, N) : 0;
      if (b + N > S.cap) {
        atomicOr(S.err, VX_ERR_OUTPUT);
        b = 0xFFFFFFFFu;
      }
      sbase[1] = b;
    }
    __syncthreads();
    uint32_t ob = sbase[1];
    if (ob == 0xFFFFFFFFu) return;
    for (uint32_t i = tid; i < N; i += VX_THREADS) S.out[ob + i] = P(i);
    if (tid == 0) {
      if (S.res_off) *S.res_off = ob;
      if (S.res_cnt) *S.res_cnt = N;
      if (S.stable_out) *S.stable_out = 0;
    }
    return;
  }

  // ---- 2. bounding box + geometry
  unsigned long long tp = __builtin_readcyclecounter();
  vx_geometry(P, N, S.leaf, M);
  const VxGeom g = M.g;
  vx_phase(S.prof_seg, 0, &tp);
  if (g.overflow) {  // PCL: "Leaf size is too small" -> output = input
    if (tid == 0) {
      uint32_t b = S.tail ? atomicAdd(S.tail, N) : 0;
      if (b + N > S.cap) {
        atomicOr(S.err, VX_ERR_OUTPUT);
        b = 0xFFFFFFFFu;
      }
      sbase[1] = b;
    }
    __syncthreads();
    uint32_t ob = sbase[1];
    if (ob == 0xFFFFFFFFu) return;
    for (uint32_t i = tid; i < N; i += VX_THREADS) S.out[ob + i] = P(i);
    if (tid == 0) {
      if (S.res_off) *S.res_off = ob;
      if (S.res_cnt) *S.res_cnt = N;
      if (S.stable_out) *S.stable_out = 0;
    }
    return;
  }

  // ---- 3-6 in one LDS pass when the unique voxels fit, else in idx-range groups
  const VxSrc src{S.src0, n0, sec};
  int moved = 0;
  uint32_t U = vx_group(S, g, src, N, members, 0u, 0xFFFFFFFFu, VX_ALLOC, VX_LDS_WORDS - 256, lds, ws,
                        M, &moved);
  if (U != VX_OVERFLOW) return;
  vx_grouped(S, g, src, N, members, lds, ws, M);
}

// Block bitonic sort of npad (a power of two, 64 <= npad <= E NT) 64-bit keys held in registers:
// element i = (wave * E + e) * 64 + lane.  Partners closer than 64 are exchanged by lane
// shuffles, partners within a lane's E registers directly; only partners in another wave go
// through LDS (xb0 / xb1: npad u64 each, alternating, one barrier per such stage; xb0 == xb1:
// one buffer, two barriers per such stage).  Waves past npad / (64 E) take part in the
// barriers only.  key(i) gives the key of element i (~0 for
// padding; it may read LDS that sk / xb0 / xb1 alias); the sorted keys end in sk[0 .. npad).
template <int NT, int E, typename KF>
__device__ inline void vx_bitonic_regs(uint64_t* sk, uint64_t* xb0, uint64_t* xb1, uint32_t npad, const KF& key) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool active = (uint32_t)(w * E * 64) < npad;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = active ? key((uint32_t)((w * E + e) * 64 + lane)) : ~0ull;
  __syncthreads();  // the key source may alias sk / xb0 / xb1
  int buf = 0;
  for (uint32_t k = 2; k <= npad; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64u * E) {  // partner in another wave
        uint64_t* xb = buf ? xb1 : xb0;
        buf ^= 1;
        if (active) {
#pragma unroll
          for (int e = 0; e < E; ++e) xb[(w * E + e) * 64 + lane] = v[e];
        }
        __syncthreads();
        if (active) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const uint32_t i = (uint32_t)((w * E + e) * 64 + lane);
            const uint64_t p = xb[i ^ j];
            const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
            v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
          }
        }
        if (xb0 == xb1) __syncthreads();  // one buffer: every read before the next write
      } else if (j >= 64) {  // partner in this lane's registers
        const int ej = (int)(j >> 6);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int f = e ^ ej;
          if (f > e) {
            const uint32_t i = (uint32_t)((w * E + e) * 64 + lane);
            const uint64_t a = v[e], b = v[f];
            const bool asc = (i & k) == 0;  // i < partner here
            v[e] = asc ? (a < b ? a : b) : (a < b ? b : a);
            v[f] = asc ? (a < b ? b : a) : (a < b ? a : b);
          }
        }
      } else if (active) {  // partner in this wave
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t i = (uint32_t)((w * E + e) * 64 + lane);
          const uint64_t p = __shfl_xor(v[e], (int)j, 64);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
        }
      }
    }
  }
  __syncthreads();  // the last cross-wave buffer may alias sk
  if (active) {
#pragma unroll
    for (int e = 0; e < E; ++e) sk[(w * E + e) * 64 + lane] = v[e];
  }
  __syncthreads();
}

// PCL's "leaf size too small" result (output = input): C ++ A copied to the tail (NT threads)
template <int NT>
__device__ inline void vx_copy_through(const VoxSeg& S, uint32_t* sbase) {
  const uint32_t n0 = (uint32_t)S.n0, N = n0 + (uint32_t)S.n1;
  if (threadIdx.x == 0) {
    uint32_t b = S.tail ? atomicAdd(S.tail, N) : 0;
    if (b + N > S.cap) {
      atomicOr(S.err, VX_ERR_OUTPUT);
      b = 0xFFFFFFFFu;
    }
    *sbase = b;
  }
  __syncthreads();
  const uint32_t ob = *sbase;
  if (ob == 0xFFFFFFFFu) return;
  for (uint32_t i = threadIdx.x; i < N; i += NT) S.out[ob + i] = i < n0 ? S.src0[i] : S.src1[i - n0];
  if (threadIdx.x == 0) {
    if (S.res_off) *S.res_off = ob;
    if (S.res_cnt) *S.res_cnt = N;
    if (S.stable_out) *S.stable_out = 0;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------
// VoxelGrid of C ++ A where C (src0, n0 points) is already a fixed point of the filter (at
// most one point per voxel, in voxel order: a previous output whose centroids all stayed in
// their voxels) and A (src1 used whole, n1 <= VX_MERGE_CAP) are new points.  Exactly the
// full filter's result, without hashing C:
//   voxels holding only a C point      -> that point, unchanged ((0 + c) / 1 == c)
//   voxels holding C point c and A's   -> (0 + c + a1 + a2 ...) / n, A in input order
//   voxels holding only A points       -> (0 + a1 + ...) / n, inserted in voxel order
// A's voxels go into an LDS hash (with member lists); C points look themselves up in it.  Only
// the voxels holding A points alone need sorting, and there are few: the map is dense where
// new points land.  Returns false, with nothing written, when the grid overflows (the caller
// then runs the full filter).
// HOT (PCL's summation order wanted, exact_voxel_order = 1): a voxel of at most 2 members sums
// alike in any order ((0 + a) + b == (0 + b) + a in IEEE arithmetic: commutative, and the leading
// 0 + x turns a -0 into +0 either way), so the merge gives PCL's bits for it.  A voxel of 3 or
// more members is not summed here but recorded in S.hot (its members, its output slot; every
// point's slot), for voxel_hot.h to sum in std::sort's order; the stable token covers the
// other voxels.
// ---------------------------------------------------------------------------------------
constexpr uint32_t VX_MERGE_CAP = 4096;

// NT threads, up to CAP new points, LW LDS words (scan scratch and misc in the last 256)
template <int NT = VX_THREADS, int CAP = (int)VX_MERGE_CAP, int LW = VX_LDS_WORDS, bool HOT = false>
__device__ inline bool vx_merge_fixed_point(const VoxSeg& S, uint32_t* lds) {
  constexpr int TMAX = 2 * CAP;       // hash slots (load factor <= 1/2)
  constexpr int RX = 2 * TMAX + CAP;  // start of the shared region: C hits, then the sort
  static_assert(RX + 4 * CAP <= LW - 256, "merge LDS layout");
  static_assert(CAP <= 4 * NT && (CAP & (CAP - 1)) == 0, "merge: at most 4 new points per thread");
  constexpr int U = VX_UNROLL;       // C points per thread kept in registers
  constexpr int UA = CAP / NT;       // A points per thread
  constexpr int SPT = TMAX / NT;     // hash slots per thread
  static_assert(SPT <= 32, "new-only flags in one word");
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  uint32_t* ws = lds + LW - 256;
  VxMisc& M = *reinterpret_cast<VxMisc*>(lds + LW - 192);
  const float4* C = S.src0;
  const float4* A = S.src1;
  const uint32_t n0 = (uint32_t)S.n0, n1 = (uint32_t)S.n1;
  unsigned long long tp = __builtin_readcyclecounter();
  // C points tid + u NT (u < U) and A points tid + u NT (u < UA) stay in registers
  float4 cc[U], aa[UA];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (tid + u * NT < n0) cc[u] = C[tid + u * NT];
#pragma unroll
  for (int u = 0; u < UA; ++u)
    if (tid + u * NT < n1) aa[u] = A[tid + u * NT];
  VxGeom g;
  int W = 0;  // anchored: voxels per axis of the key box
  if (S.anchored) {  // keys from the cube's corner voxel (VoxSeg::anchored): no bounding-box pass
    g.inv = 1.0f / S.leaf;
    g.minbx = (int)floorf((float)S.anchor[0] * g.inv) - 1;
    g.minby = (int)floorf((float)S.anchor[1] * g.inv) - 1;
    g.minbz = (int)floorf((float)S.anchor[2] * g.inv) - 1;
    W = (int)ceilf(50.0f * g.inv) + 3;  // the 50 m edge, one voxel of margin on each side, rounding
    g.mul1 = W;
    g.mul2 = W * W;
    g.nvox = (unsigned long long)W * W * W;
    g.overflow = 0;
    if (tid == 0) M.g = g;  // (read after later barriers: the exact order's fix-up)
  } else {
    float mnx = 3.402823466e38f, mny = 3.402823466e38f, mnz = 3.402823466e38f;
    float mxx = -3.402823466e38f, mxy = -3.402823466e38f, mxz = -3.402823466e38f;
    auto acc = [&](const float4& p) {
      mnx = fminf(mnx, p.x); mny = fminf(mny, p.y); mnz = fminf(mnz, p.z);
      mxx = fmaxf(mxx, p.x); mxy = fmaxf(mxy, p.y); mxz = fmaxf(mxz, p.z);
    };
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (tid + u * NT < n0) acc(cc[u]);
    // C points past the register-held ones: 4 loads in flight per step (one at a time, each pass
    // over a large cube's remainder was a chain of memory round trips)
    for (uint32_t k = tid + U * NT; k < n0; k += 4 * NT) {
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k + u * NT < n0) p[u] = C[k + u * NT];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k + u * NT < n0) acc(p[u]);
    }
#pragma unroll
    for (int u = 0; u < UA; ++u)
      if (tid + u * NT < n1) acc(aa[u]);
    vx_geometry_finish<NT>(mnx, mny, mnz, mxx, mxy, mxz, S.leaf, M);
    g = M.g;
  }
  vx_phase(S.prof, 0, &tp);
  if (g.overflow) return false;
  // anchored keys are valid only inside the key box: checked for every point on the way (pass A)
  int bad = 0;
  auto outside = [&](const float4& p) -> int {
    if (!W) return 0;
    const int ix = (int)(floorf(p.x * g.inv) - (float)g.minbx), iy = (int)(floorf(p.y * g.inv) - (float)g.minby),
              iz = (int)(floorf(p.z * g.inv) - (float)g.minbz);
    return ((unsigned)ix >= (unsigned)W) | ((unsigned)iy >= (unsigned)W) | ((unsigned)iz >= (unsigned)W);
  };
  uint32_t T = 64;
  while (T < 2 * n1) T <<= 1;
  const uint32_t mask = T - 1;
  uint32_t* hkey = lds;                                   // T: voxel key
  uint32_t* hcnt = lds + TMAX;                            // T: member count, then start << 13 | count
  uint32_t* mem = lds + 2 * TMAX;                         // n1: members, grouped by voxel
  int* hit = reinterpret_cast<int*>(lds + RX);            // T: the C point of the voxel, or -1
  uint64_t* srt = reinterpret_cast<uint64_t*>(lds + RX);  // later: the new-only voxels (key, slot)
  for (uint32_t h = tid; h < T; h += NT) {
    hkey[h] = NONE;
    hcnt[h] = 0;
    hit[h] = -1;
  }
  if (tid == 0) M.sfail = 0;  // the anchored key box check (pass A)
  __syncthreads();
  // 1. A's voxels: slot and rank of every new point
  uint32_t ar[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    ar[u] = NONE;
    if (tid + u * NT >= n1) continue;
    bad |= outside(aa[u]);
    const uint32_t key = vx_key(g, aa[u]);
    uint32_t h = vx_slot(key, mask);
    while (true) {
      const uint32_t old = atomicCAS(&hkey[h], NONE, key);
      if (old == NONE || old == key) break;
      h = (h + 1) & mask;
    }
    ar[u] = (h << 13) | atomicAdd(&hcnt[h], 1u);  // h < 2^14, rank < 2^13
  }
  __syncthreads();
  // 2. member ranges (slots tid, tid + NT, ...) and the members
  {
    uint32_t sum = 0;
    for (uint32_t h = tid; h < T; h += NT) sum += hcnt[h];
    uint32_t tot;
    uint32_t pre = vx_block_scan_t<NT>(sum, ws, &tot);
    for (uint32_t h = tid; h < T; h += NT) {
      const uint32_t c = hcnt[h];
      hcnt[h] = (pre << 13) | c;
      pre += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < UA; ++u)
    if (ar[u] != NONE) mem[(hcnt[ar[u] >> 13] >> 13) + (ar[u] & 0x1FFFu)] = tid + u * NT;
  // 3. pass A: every C point looks its voxel up; hit voxels remember it
  auto lookup = [&](uint32_t key) -> uint32_t {
    uint32_t h = vx_slot(key, mask);
    while (true) {
      const uint32_t k2 = hkey[h];
      if (k2 == key) return h;
      if (k2 == NONE) return NONE;
      h = (h + 1) & mask;
    }
  };
  uint32_t cl[U], ck[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t k = tid + u * NT;
    cl[u] = NONE;
    ck[u] = 0;
    if (k < n0) {
      bad |= outside(cc[u]);
      ck[u] = vx_key(g, cc[u]);
      cl[u] = lookup(ck[u]);
      if (cl[u] != NONE) hit[cl[u]] = (int)k;
    }
  }
  for (uint32_t k = tid + U * NT; k < n0; k += 4 * NT) {
    float4 p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (k + u * NT < n0) p[u] = C[k + u * NT];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (k + u * NT < n0) {
        bad |= outside(p[u]);
        const uint32_t h = lookup(vx_key(g, p[u]));
        if (h != NONE) hit[h] = (int)(k + u * NT);
      }
  }
  if (bad) atomicOr(&M.sfail, 1);
  __syncthreads();
  if (W && __builtin_amdgcn_readfirstlane(M.sfail)) return false;  // a point outside the anchored key box: full filter
  vx_phase(S.prof, 1, &tp);
  // 4. the voxels holding A points only, listed then sorted by key
  uint32_t fmask = 0, cnt = 0;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const uint32_t h = tid + q * NT;
    if (h < T && hkey[h] != NONE && hit[h] < 0) {
      fmask |= 1u << q;
      ++cnt;
    }
  }
  uint32_t Dn;
  uint32_t pre = vx_block_scan_t<NT>(cnt, ws, &Dn);  // its barriers end every read of hit
#pragma unroll
  for (int q = 0; q < SPT; ++q)
    if (fmask & (1u << q)) {
      const uint32_t h = tid + q * NT;
      srt[pre++] = ((uint64_t)hkey[h] << 32) | h;
    }
  __syncthreads();
  uint32_t npad = 64;
  while (npad < Dn) npad <<= 1;
  if (Dn > 1) {
    auto key = [&](uint32_t i) -> uint64_t { return i < Dn ? srt[i] : ~0ull; };
    uint64_t* xb1 = srt + npad;
    if (npad <= (uint32_t)NT) vx_bitonic_regs<NT, 1>(srt, srt, xb1, npad, key);
    else if (npad <= 2u * NT) vx_bitonic_regs<NT, 2>(srt, srt, xb1, npad, key);
    else vx_bitonic_regs<NT, 4>(srt, srt, xb1, npad, key);
  }
  uint32_t* cbelow = reinterpret_cast<uint32_t*>(srt + npad);  // Dn + 1 <= 2 npad words
  for (uint32_t r = tid; r <= Dn; r += NT) cbelow[r] = 0;
  // a bucket directory over the new-only voxels' keys for below(): bucket b = (key - kmin) >> sh,
  // bdir[b] the first voxel of a bucket >= b (bdir[MB] = Dn), so a lookup searches one bucket
  // (~Dn / MB voxels) instead of all Dn (pass B looks up every C point)
  constexpr int MB = 1024;
  static_assert(RX + 4 * CAP + MB + 1 <= LW - 256, "merge LDS layout: bucket directory");
  uint32_t* bdir = lds + RX + 4 * CAP;
  const uint32_t kmin = Dn ? (uint32_t)(srt[0] >> 32) : 0u, kmax = Dn ? (uint32_t)(srt[Dn - 1] >> 32) : 0u;
  int sh = 0;
  while ((((uint64_t)kmax - kmin) >> sh) >= (uint64_t)MB) ++sh;  // every bucket < MB: bdir[b + 1] exists
  for (uint32_t r = tid; r < Dn; r += NT) {
    const int b = (int)(((uint32_t)(srt[r] >> 32) - kmin) >> sh);
    const int bp = r ? (int)(((uint32_t)(srt[r - 1] >> 32) - kmin) >> sh) : -1;
    for (int q = bp + 1; q <= b; ++q) bdir[q] = r;
    if (r == Dn - 1)
      for (int q = b + 1; q <= MB; ++q) bdir[q] = Dn;
  }
  if (tid == 0) {
    M.moved = 0;
    M.hot_n = 0;
    M.hot_l = 0;
    uint32_t b = S.tail ? atomicAdd(S.tail, n0 + Dn) : 0;
    if (b + n0 + Dn > S.cap) {
      atomicOr(S.err, VX_ERR_OUTPUT);
      b = 0xFFFFFFFFu;
    }
    M.sbase[1] = b;
  }
  __syncthreads();
  vx_phase(S.prof, 2, &tp);
  const uint32_t ob = M.sbase[1];
  if (ob == 0xFFFFFFFFu) return true;
  float4* out = S.out + ob;
  bool moved = false;
  // sum of slot h's members after the optional C point, in input order (the owner sorts the
  // member range in place first: atomics ranked them in arbitrary order)
  auto centroid = [&](uint32_t h, float sx, float sy, float sz, float si, uint32_t n) -> float4 {
    const uint32_t e = hcnt[h], m0 = e >> 13, mc = e & 0x1FFFu;
    for (uint32_t a = 1; a < mc; ++a) {
      const uint32_t x = mem[m0 + a];
      uint32_t b = a;
      while (b > 0 && mem[m0 + b - 1] > x) {
        mem[m0 + b] = mem[m0 + b - 1];
        --b;
      }
      mem[m0 + b] = x;
    }
    for (uint32_t t = 0; t < mc; t += 4) {
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (t + u < mc) p[u] = A[mem[m0 + t + u]];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (t + u < mc) {
          sx += p[u].x; sy += p[u].y; sz += p[u].z; si += p[u].w;
        }
    }
    n += mc;
    const float fn = (float)n;
    return make_float4(sx / fn, sy / fn, sz / fn, si / fn);
  };
  // new-only voxels with key below `key` (the bucket of `key`, then a search inside it)
  auto below = [&](uint32_t key) -> uint32_t {
    if (Dn == 0 || key <= kmin) return 0u;
    if (key > kmax) return Dn;
    const uint32_t b = (key - kmin) >> sh;
    uint32_t lo = bdir[b], hi = bdir[b + 1];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((uint32_t)(srt[mid] >> 32) < key) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  // 5. pass B: C point k goes to k + (new-only voxels before it); merged voxels re-averaged.
  // cbelow[b] counts the C points with b new-only voxels before them: C is in key order, so a
  // wave's lanes (consecutive C points) mostly share b, and each run of equal b adds its length
  // with one atomic by its first lane (lanes past n0 end every run).  All lanes of a wave call it.
  const int lane = tid & 63;
  auto count_below = [&](bool act, uint32_t b) {
    const uint32_t bb = act ? b : 0xFFFFFFFFu;
    const uint32_t prev = (uint32_t)__shfl_up((int)bb, 1, 64);
    const uint64_t starts = __ballot(!act || lane == 0 || prev != bb);
    if (act && ((starts >> lane) & 1ull)) {
      const uint64_t after = lane == 63 ? 0ull : starts & (~0ull << (lane + 1));
      const uint32_t run = (uint32_t)((after ? __ffsll((long long)after) - 1 : 64) - lane);
      atomicAdd(&cbelow[b], run);
    }
  };
  auto emit = [&](uint32_t k, const float4& c, uint32_t key, uint32_t h, uint32_t b) {
    float4 v = c;
    if (h != NONE) {
      if constexpr (HOT) {
        const uint32_t e = hcnt[h], m0 = e >> 13, mc = e & 0x1FFFu;
        if (mc + 1 >= 3) {
          vh_record(S.hot, M, k + b, mc + 1, [&](uint32_t a) { return a == 0 ? k : n0 + mem[m0 + a - 1]; });
          return;
        }
        for (uint32_t a = 0; a < mc; ++a) S.hot.rk[n0 + mem[m0 + a]] = (k + b) << 1;
      }
      v = centroid(h, 0.f + c.x, 0.f + c.y, 0.f + c.z, 0.f + c.w, 1u);
      moved |= vx_key(g, v) != key;
    }
    if constexpr (HOT) S.hot.rk[k] = (k + b) << 1;
    out[k + b] = v;
  };
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool act = tid + u * NT < n0;
    const uint32_t b = act ? below(ck[u]) : 0u;
    count_below(act, b);
    if (act) emit(tid + u * NT, cc[u], ck[u], cl[u], b);
  }
  // (a wave-uniform loop: count_below needs every lane of the wave)
  for (uint32_t kb = (uint32_t)(tid & ~63) + U * NT; kb < n0; kb += 4 * NT) {
    const uint32_t k = kb + lane;
    float4 p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (k + u * NT < n0) p[u] = C[k + u * NT];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool act = k + u * NT < n0;
      const uint32_t key = act ? vx_key(g, p[u]) : 0u;
      const uint32_t b = act ? below(key) : 0u;
      count_below(act, b);
      if (act) emit(k + u * NT, p[u], key, lookup(key), b);
    }
  }
  __syncthreads();
  // C points below new-only voxel r: inclusive prefix of cbelow (Dn + 1 entries)
  for (uint32_t r0 = 0; r0 <= Dn; r0 += NT) {
    const uint32_t r = r0 + tid;
    const uint32_t v = r <= Dn ? cbelow[r] : 0u;
    uint32_t tot;
    const uint32_t ex = vx_block_scan_t<NT>(v, ws, &tot);
    if (r <= Dn) cbelow[r] = ex + v + (r0 ? cbelow[r0 - 1] : 0u);
    __syncthreads();
  }
  for (uint32_t r = tid; r < Dn; r += NT) {
    const uint32_t h = (uint32_t)srt[r];
    if constexpr (HOT) {
      const uint32_t e = hcnt[h], m0 = e >> 13, mc = e & 0x1FFFu, slot = r + cbelow[r];
      if (mc >= 3) {
        vh_record(S.hot, M, slot, mc, [&](uint32_t a) { return n0 + mem[m0 + a]; });
        continue;
      }
      for (uint32_t a = 0; a < mc; ++a) S.hot.rk[n0 + mem[m0 + a]] = slot << 1;
    }
    const float4 v = centroid(h, 0.f, 0.f, 0.f, 0.f, 0u);
    out[r + cbelow[r]] = v;
    moved |= vx_key(g, v) != (uint32_t)(srt[r] >> 32);
  }
  if (moved) M.moved = 1;
  __syncthreads();
  vx_phase(S.prof, 3, &tp);
  if (tid == 0) {
    if (S.res_off) *S.res_off = ob;
    if (S.res_cnt) *S.res_cnt = n0 + Dn;
    if (S.stable_out) *S.stable_out = M.moved ? 0u : ob + 1;
  }
  return true;
}

}  // namespace loam
