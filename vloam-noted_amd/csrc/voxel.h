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
//   4. compact the U unique voxels, bitonic-sort them in LDS by idx
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

struct VoxSeg {
  const float4* src0;
  int n0;
  const float4* src1;  // optional secondary source filtered by tag
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
  float4* scratch_pts;    // gathered secondary points
  int* scratch_idx;       // member lists
  uint32_t* scratch_tail; // if set, scratch slots are allocated from it (per segment)
  uint32_t scratch_cap;
  int* err;
};

__device__ inline uint32_t vx_hash(uint32_t k) { return (k * 0x9E3779B1u) >> (32 - 14); }

// block-wide exclusive scan of one value per thread (VX_THREADS); returns exclusive prefix,
// total in *total.  ws: LDS scratch of >= VX_WAVES + 1 words.
__device__ inline uint32_t vx_block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t inc = wave_incl_scan_u(v);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < VX_WAVES; ++w) {
      uint32_t t = ws[w];
      ws[w] = acc;
      acc += t;
    }
    ws[VX_WAVES] = acc;
  }
  __syncthreads();
  uint32_t r = ws[wid] + inc - v;
  *total = ws[VX_WAVES];
  __syncthreads();
  return r;
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
  VxGeom g;
  float bb[VX_WAVES][6];
};
static_assert(sizeof(VxMisc) <= 192 * 4, "misc area");


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

// Member lists (chunk by chunk: members of earlier chunks precede later ones), then per
// voxel: members sorted by input index, float sums in that order, centroid -> out[j].
template <typename MT>
__device__ inline void vx_centroids(const VxGeom& g, const VxSrc& P, uint32_t N, MT* members,
                                    uint32_t klo, uint32_t khi, uint32_t U, const uint32_t* ukey,
                                    const uint32_t* uoff, uint32_t* ufill, float4* out) {
  const int tid = threadIdx.x;
  for (uint32_t c = 0; c < N; c += VX_THREADS) {
    uint32_t i = c + tid;
    if (i < N) {
      uint32_t k = vx_key(g, P(i));
      if (k >= klo && k < khi) {
        uint32_t lo = 0, hi = U;  // lower_bound
        while (lo < hi) {
          uint32_t mid = (lo + hi) >> 1;
          if (ukey[mid] < k) lo = mid + 1; else hi = mid;
        }
        uint32_t pos = uoff[lo] + atomicAdd(&ufill[lo], 1u);
        members[pos] = (MT)i;
      }
    }
    __syncthreads();
  }
  for (uint32_t j = tid; j < U; j += VX_THREADS) {
    const uint32_t b = uoff[j];
    const uint32_t n = ufill[j];
    for (uint32_t a = 1; a < n; ++a) {  // insertion sort (lists are short and nearly ordered)
      const MT v = members[b + a];
      uint32_t q = a;
      while (q > 0 && members[b + q - 1] > v) {
        members[b + q] = members[b + q - 1];
        --q;
      }
      members[b + q] = v;
    }
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    for (uint32_t a = 0; a < n; a += 4) {  // gathers issued together, summed in order
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < n) p[u] = P((uint32_t)members[b + a + u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < n) {
          sx += p[u].x; sy += p[u].y; sz += p[u].z; si += p[u].w;
        }
    }
    const float fn = (float)n;
    out[j] = make_float4(sx / fn, sy / fn, sz / fn, si / fn);
  }
}

// Steps 3-6 for the points whose voxel idx lies in [klo, khi): LDS hash -> sorted unique
// voxels -> member lists -> centroids written at out[base + j].  out_base == VX_ALLOC:
// allocate exactly U (at *tail or at 0) once U is known.  Returns U, or VX_OVERFLOW (no side
// effects on the output) when the unique voxels do not fit the LDS.
__device__ inline uint32_t vx_group(const VoxSeg& S, const VxGeom& g, const VxSrc& P, uint32_t N,
                                    int* members, uint32_t klo, uint32_t khi, uint32_t out_base,
                                    uint32_t lds_limit, uint32_t* lds, uint32_t* ws, VxMisc& M) {
  const int tid = threadIdx.x;
  uint32_t* hkey = lds;
  uint32_t* hcnt = lds + VX_HASH;
  for (int i = tid; i < VX_HASH; i += VX_THREADS) {
    hkey[i] = VX_EMPTY;
    hcnt[i] = 0;
  }
  if (tid == 0) M.sfail = 0;
  __syncthreads();
  for (uint32_t i = tid; i < N; i += VX_THREADS) {
    const uint32_t k = vx_key(g, P(i));
    if (k < klo || k >= khi) continue;
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
  if (U > VX_UCAP || fail) return VX_OVERFLOW;
  uint32_t Upad = 1;
  while (Upad < U) Upad <<= 1;
  uint64_t* s64 = reinterpret_cast<uint64_t*>(lds);  // overlays the (consumed) hash
#pragma unroll
  for (int s = 0; s < SPT; ++s)
    if (mk[s] != VX_EMPTY) s64[mpos++] = ((uint64_t)mk[s] << 32) | mc[s];
  for (uint32_t i = U + tid; i < Upad; i += VX_THREADS) s64[i] = 0xFFFFFFFFFFFFFFFFull;
  __syncthreads();
  for (uint32_t k = 2; k <= Upad; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = tid; i < Upad; i += VX_THREADS) {
        uint32_t ixj = i ^ j;
        if (ixj > i) {
          uint64_t a = s64[i], b = s64[ixj];
          bool asc = (i & k) == 0;
          if ((a > b) == asc) {
            s64[i] = b;
            s64[ixj] = a;
          }
        }
      }
      __syncthreads();
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
  if (N <= 65536u && 3 * U + (tot + 1) / 2 <= lds_limit)
    vx_centroids(g, P, N, reinterpret_cast<uint16_t*>(lds + 3 * U), klo, khi, U, ukey, uoff, ufill,
                 S.out + ob);
  else
    vx_centroids(g, P, N, members, klo, khi, U, ukey, uoff, ufill, S.out + ob);
  if (out_base == VX_ALLOC && tid == 0) {
    if (S.res_off) *S.res_off = ob;
    if (S.res_cnt) *S.res_cnt = U;
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
  for (int gi = 0; gi < ng; ++gi) {
    const int ge = (int)gend[gi];
    const uint32_t U = vx_group(S, g, P, N, members, blo(gstart), ge >= VX_NB ? 0xFFFFFFFFu : blo(ge),
                                ob + acc, VX_HIST_WORD, lds, ws, M);
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
  }
}

// The workgroup routine.  lds: VX_LDS_WORDS u32 words (the whole 160 KiB; the last 256 words
// hold scan scratch + VxMisc).  All threads of the block call it.
__device__ inline void voxel_segment(const VoxSeg& S, uint32_t* lds) {
  const int tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
  uint32_t* ws = lds + VX_LDS_WORDS - 256;  // scan scratch (64 words)
  VxMisc& M = *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192);

  // ---- 1. count secondary matches, allocate scratch, gather (stable)
  uint32_t m1 = 0;
  if (S.src1 && S.n1 > 0) {
    uint32_t local = 0;
    for (int i = tid; i < S.n1; i += VX_THREADS) local += (S.tag1[i] == S.tag) ? 1u : 0u;
    uint32_t tot;
    vx_block_scan(local, ws, &tot);
    m1 = tot;
  }
  const int n0 = S.n0;
  const uint32_t N = (uint32_t)n0 + m1;
  const uint32_t req = S.append_only ? m1 : N;  // append: gathered points only
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
  float4* sec = S.scratch_pts + sb;  // gathered secondary points (m1)
  int* members = S.scratch_idx + sb;  // member lists (N, voxelize mode)
  if (m1 > 0) {
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
    }
    return;
  }

  // ---- 2. bounding box (pcl::getMinMax3D)
  float mnx = 3.402823466e38f, mny = 3.402823466e38f, mnz = 3.402823466e38f;
  float mxx = -3.402823466e38f, mxy = -3.402823466e38f, mxz = -3.402823466e38f;
  for (uint32_t i = tid; i < N; i += VX_THREADS) {
    float4 p = P(i);
    mnx = fminf(mnx, p.x); mny = fminf(mny, p.y); mnz = fminf(mnz, p.z);
    mxx = fmaxf(mxx, p.x); mxy = fmaxf(mxy, p.y); mxz = fmaxf(mxz, p.z);
  }
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
    for (int w = 1; w < VX_WAVES; ++w) {
      mnx = fminf(mnx, sbb[w][0]); mny = fminf(mny, sbb[w][1]); mnz = fminf(mnz, sbb[w][2]);
      mxx = fmaxf(mxx, sbb[w][3]); mxy = fmaxf(mxy, sbb[w][4]); mxz = fmaxf(mxz, sbb[w][5]);
    }
    VxGeom g;
    g.inv = 1.0f / S.leaf;
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
  const VxGeom g = sg;
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
    }
    return;
  }

  // ---- 3-6 in one LDS pass when the unique voxels fit, else in idx-range groups
  const VxSrc src{S.src0, n0, sec};
  uint32_t U = vx_group(S, g, src, N, members, 0u, 0xFFFFFFFFu, VX_ALLOC, VX_LDS_WORDS - 256, lds, ws,
                        M);
  if (U != VX_OVERFLOW) return;
  vx_grouped(S, g, src, N, members, lds, ws, M);
}

}  // namespace loam
