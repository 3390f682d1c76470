// voxel_pcl.h — pcl::VoxelGrid<PointXYZI> with PCL's own summation order, one workgroup.
//
// PCL 1.8-1.12 voxel_grid.hpp applyFilter: getMinMax3D -> the int32 overflow check (output =
// input) -> min_b / div_b / divb_mul -> (idx, point index) pairs in input order -> std::sort
// with operator< on idx alone -> one output point per run of equal idx, in increasing idx, the
// CentroidPoint of the run's points added in the sorted order (float sums of x, y, z and
// intensity, each divided by (float)count).  The within-run order is libstdc++'s introsort
// permutation, reproduced exactly by stdsort.h, so the centroids carry PCL's bits.
//
// Used where the clouds are small enough for the sort to be cheap on the critical path: the
// per-ring lessFlat filter of ScanRegistration (scan_registration.cpp:497-501, ~10^3 points per
// ring).  The mapper's filters (stack and cube VoxelGrids, 10^4-10^5 points) use voxel.h, which
// sums a voxel's points in input order (DESIGN.md §6 states and tests the difference).
#pragma once
#include "stdsort.h"
#include "voxel.h"

namespace loam {

// A sort too large for the LDS (E in global memory): segments of at most `defer` elements are
// sorted whole in LDS (ss_sort_deferred) instead of level by level in global memory.
struct VxPclDefer {
  int defer;
  int* dseg;  // [dcap][3], global
  int dcap;
  uint64_t* lE;
  uint32_t* lA;
  uint32_t* lB;
  int* lseg0;
  int* lseg1;
  int lcap;
  SsLevels* LL;  // LDS
};

struct VxPclScratch {
  uint64_t* E;   // n: (idx << 32 | point), permuted by the sort
  uint32_t* A;   // n
  uint32_t* B;   // n
  uint64_t* S;   // n: sorted
  SsLevels* lev;  // LDS
  int* seg[2];    // 3 * cap ints each (LDS or global)
  int cap;        // >= n / 17 + 1
  uint32_t* loc = nullptr;  // LDS for the waves' subtree sorts (SS_LOC_WORDS each) when E is global
  unsigned long long* prof = nullptr;  // optional phase cycles: [0] bbox + keys, [1] sort levels,
                                       // [2] final pass, [3] centroids (a sort in global memory:
                                       // [1] its deferred segments, its own levels in glob)
  unsigned long long* heap = nullptr;  // optional: depth-limit segments [0] and their elements [1]
  unsigned long long* glob = nullptr;  // optional: cycles of a global-memory sort's own levels
};

struct VxPtrSrc {
  const float4* p;
  __device__ float4 operator()(uint32_t i) const { return p[i]; }
};

struct VxIdxLess {
  static constexpr int free_run = 2;  // a voxel's centroid: 2 members sum alike in either order
  __device__ bool operator()(uint64_t a, uint64_t b) const { return (uint32_t)(a >> 32) < (uint32_t)(b >> 32); }
};

// Where the centroids go: out[0 ..) (tail == nullptr), or a block of exactly the output
// count allocated at *tail (the mapper's arena).  res_off / res_cnt / stable_out optional:
// the block's offset and count, and (offset + 1) when the output is a VoxelGrid fixed point
// (every centroid inside its own voxel: re-filtering it is the identity), else 0.
struct VxPclOut {
  float4* out;
  uint32_t* tail = nullptr;
  uint32_t cap = 0xFFFFFFFFu;
  uint32_t* res_off = nullptr;
  uint32_t* res_cnt = nullptr;
  uint32_t* stable_out = nullptr;
  // a block an earlier filter of the same points already allocated (the mapper's fall-back from
  // the LDS emulation, mapper.hip): reused when the output fits it, instead of a second block
  uint32_t reuse_off = 0xFFFFFFFFu, reuse_cnt = 0;
};

// All NT threads call it.  P(i): the i-th input point (i < n).  ws: >= NT / 64 + 1 words of
// LDS; M: LDS misc.  err |= 4: level list overflow, |= 2 (VX_ERR_OUTPUT): output block past cap.
// DEFER (a sort in global memory): segments that fit the LDS are sorted there whole (dfr).
template <int NT, bool DEFER = false, typename PF>
__device__ inline void voxel_grid_pcl(const PF& P, int n, float leaf, const VxPclOut& O, const VxPclScratch& X,
                                      VxMisc& M, uint32_t* ws, int* err, const VxPclDefer* dfr = nullptr) {
  const int tid = threadIdx.x;
  auto finish = [&](uint32_t base, uint32_t cnt, bool fixed) {
    if (O.res_off) *O.res_off = base;
    if (O.res_cnt) *O.res_cnt = cnt;
    if (O.stable_out) *O.stable_out = fixed ? base + 1 : 0u;
  };
  auto alloc = [&](uint32_t cnt) {  // thread 0; 0xFFFFFFFF: no room
    if (O.reuse_off != 0xFFFFFFFFu && cnt <= O.reuse_cnt) return O.reuse_off;
    uint32_t b = O.tail ? atomicAdd(O.tail, cnt) : 0u;
    if (b + cnt > O.cap) {
      atomicOr(err, VX_ERR_OUTPUT);
      b = 0xFFFFFFFFu;
    }
    return b;
  };
  if (n <= 0) {
    if (tid == 0) finish(0, 0, false);
    return;
  }
  vx_geometry<PF, NT>(P, (uint32_t)n, leaf, M);
  const VxGeom g = M.g;
  if (g.overflow) {  // "Leaf size is too small for the input dataset": output = input
    if (tid == 0) M.sbase[1] = alloc((uint32_t)n);
    __syncthreads();
    const uint32_t b = M.sbase[1];
    if (b == 0xFFFFFFFFu) return;
    for (int i = tid; i < n; i += NT) O.out[b + i] = P((uint32_t)i);
    if (tid == 0) finish(b, (uint32_t)n, false);
    return;
  }
  unsigned long long tp = __builtin_readcyclecounter();
  for (int i = tid; i < n; i += NT) X.E[i] = ((uint64_t)vx_key(g, P((uint32_t)i)) << 32) | (uint32_t)i;
  if (tid == 0) {
    ss_levels_init(X.lev, n, X.seg[0], X.seg[1], X.cap);
    X.lev->loc = X.loc;
    X.lev->hctr = X.heap;
    if (DEFER) {
      X.lev->defer = dfr->defer;
      X.lev->dcap = dfr->dcap;
    }
    M.moved = 0;
  }
  const VxIdxLess less;
  __syncthreads();
  vx_phase(X.prof, 0, &tp);
  if constexpr (DEFER) {
    ss_levels<true, NT, true>(X.E, X.A, X.B, X.lev, tid >> 6, NT / 64, less, X.seg[0], X.seg[1], X.loc, dfr->dseg);
    __syncthreads();
    vx_phase(X.glob, 0, &tp);  // the global-memory levels; prof[1]: the deferred LDS sorts
    ss_sort_deferred<NT>(X.E, X.A, X.B, X.lev, dfr->dseg, less, dfr->lE, dfr->lA, dfr->lB, dfr->lseg0, dfr->lseg1,
                         dfr->lcap, dfr->LL);
  } else {
    ss_levels<true, NT>(X.E, X.A, X.B, X.lev, tid >> 6, NT / 64, less, X.seg[0], X.seg[1], X.loc);
  }
  __syncthreads();
  vx_phase(X.prof, 1, &tp);
  if (tid == 0 && X.lev->err) atomicOr(err, 4);
  ss_final(X.E, X.A, X.B, n, X.S, tid, NT, less);
  __syncthreads();
  vx_phase(X.prof, 2, &tp);
  // runs of equal idx: thread t owns positions [t * per, (t + 1) * per)
  const int per = (n + NT - 1) / NT;
  const int p0 = min(n, tid * per), p1 = min(n, p0 + per);
  uint32_t starts = 0;
  for (int i = p0; i < p1; ++i)
    starts += (i == 0 || (uint32_t)(X.S[i] >> 32) != (uint32_t)(X.S[i - 1] >> 32)) ? 1u : 0u;
  uint32_t tot;
  uint32_t o = vx_block_scan_t<NT>(starts, ws, &tot);
  if (tid == 0) M.sbase[1] = alloc(tot);
  __syncthreads();
  const uint32_t b = M.sbase[1];
  if (b == 0xFFFFFFFFu) return;
  bool moved = false;
  for (int i = p0; i < p1; ++i) {
    const uint32_t key = (uint32_t)(X.S[i] >> 32);
    if (i > 0 && (uint32_t)(X.S[i - 1] >> 32) == key) continue;
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    int j = i;
    for (; j < n && (uint32_t)(X.S[j] >> 32) == key; ++j) {
      const float4 p = P((uint32_t)X.S[j]);
      sx += p.x;
      sy += p.y;
      sz += p.z;
      si += p.w;
    }
    const float c = (float)(j - i);
    const float4 cen = make_float4(sx / c, sy / c, sz / c, si / c);
    moved |= vx_key(g, cen) != key;
    O.out[b + o++] = cen;
  }
  if (moved) M.moved = 1;
  __syncthreads();
  vx_phase(X.prof, 3, &tp);
  if (tid == 0) finish(b, tot, M.moved == 0);
}

}  // namespace loam
