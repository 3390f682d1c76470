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

struct VxPclScratch {
  uint64_t* E;   // n: (idx << 32 | point), permuted by the sort
  uint32_t* A;   // n
  uint32_t* B;   // n
  uint64_t* S;   // n: sorted
  SsCtl* ctl;    // LDS
  int* stk;      // LDS, 3 * stk_cap
  int stk_cap;
};

struct VxPtrSrc {
  const float4* p;
  __device__ float4 operator()(uint32_t i) const { return p[i]; }
};

struct VxIdxLess {
  __device__ bool operator()(uint64_t a, uint64_t b) const { return (uint32_t)(a >> 32) < (uint32_t)(b >> 32); }
};

// All NT threads call it.  out receives the centroids (at most n), *out_n their count.
// ws: >= NT / 64 + 1 words of LDS; M: LDS misc.
template <int NT>
__device__ inline void voxel_grid_pcl(const float4* src, int n, float leaf, float4* out, uint32_t* out_n,
                                      const VxPclScratch& X, VxMisc& M, uint32_t* ws, int* err) {
  const int tid = threadIdx.x;
  if (n <= 0) {
    if (tid == 0) *out_n = 0;
    return;
  }
  vx_geometry<VxPtrSrc, NT>(VxPtrSrc{src}, (uint32_t)n, leaf, M);
  const VxGeom g = M.g;
  if (g.overflow) {  // "Leaf size is too small for the input dataset": output = input
    for (int i = tid; i < n; i += NT) out[i] = src[i];
    if (tid == 0) *out_n = (uint32_t)n;
    return;
  }
  for (int i = tid; i < n; i += NT) X.E[i] = ((uint64_t)vx_key(g, src[i]) << 32) | (uint32_t)i;
  if (tid == 0) ss_init(X.ctl, X.stk, n);
  __syncthreads();
  const VxIdxLess less;
  ss_loop(X.E, X.A, X.B, X.ctl, X.stk, X.stk_cap, less);
  __syncthreads();
  if (tid == 0 && X.ctl->err) atomicOr(err, 4);
  ss_final(X.E, X.A, X.B, n, X.S, tid, NT, less);
  __syncthreads();
  // runs of equal idx: thread t owns positions [t * per, (t + 1) * per)
  const int per = (n + NT - 1) / NT;
  const int p0 = min(n, tid * per), p1 = min(n, p0 + per);
  uint32_t starts = 0;
  for (int i = p0; i < p1; ++i)
    starts += (i == 0 || (uint32_t)(X.S[i] >> 32) != (uint32_t)(X.S[i - 1] >> 32)) ? 1u : 0u;
  uint32_t tot;
  uint32_t o = vx_block_scan_t<NT>(starts, ws, &tot);
  for (int i = p0; i < p1; ++i) {
    const uint32_t key = (uint32_t)(X.S[i] >> 32);
    if (i > 0 && (uint32_t)(X.S[i - 1] >> 32) == key) continue;
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    int j = i;
    for (; j < n && (uint32_t)(X.S[j] >> 32) == key; ++j) {
      const float4 p = src[(uint32_t)X.S[j]];
      sx += p.x;
      sy += p.y;
      sz += p.z;
      si += p.w;
    }
    const float c = (float)(j - i);
    out[o++] = make_float4(sx / c, sy / c, sz / c, si / c);
  }
  if (tid == 0) *out_n = tot;
}

}  // namespace loam
