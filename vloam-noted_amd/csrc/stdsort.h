// stdsort.h — the exact permutation of libstdc++'s std::sort, computed by waves.
//
// Two places in the reference sort with std::sort and a comparator that ignores part of the
// element, so ties are left in whatever order the algorithm produces, and that order decides
// results:
//   - the sector sort of scan_registration.cpp:365-366 (indices by curvature): with equal
//     curvatures it decides which point becomes sharp / flat (:371-483);
//   - pcl::VoxelGrid::applyFilter (PCL 1.8-1.12 voxel_grid.hpp, "second pass": std::sort of
//     (idx, point) pairs with cloud_point_index_idx::operator< comparing idx only): the order
//     of a voxel's points is the float summation order of its centroid.
// libstdc++ (GCC 4.9 through 13, bits/stl_algo.h) implements std::sort as
//   __introsort_loop(first, last, 2 * __lg(n)):
//       while (last - first > 16):
//           if depth_limit == 0: __partial_sort(first, last, last)  (heap sort); return
//           --depth_limit
//           cut = __unguarded_partition_pivot(first, last)
//                 (__move_median_to_first(first, first + 1, mid, last - 1), then the Hoare
//                  scan __unguarded_partition(first + 1, last, pivot = *first))
//           __introsort_loop(cut, last, depth_limit); last = cut
//   __final_insertion_sort(first, last)
// and this header reproduces its output permutation exactly:
//   * segments are independent, so any processing order gives the same result: the waves
//     take the segments level by level (one wave per segment, a barrier between levels);
//   * the Hoare scan is computed in parallel: with l_k the k-th position (ascending) in
//     [first+1, last) whose key is !(key < pivot) and r_k the k-th position (descending) in
//     [first, last) whose key is !(pivot < key) (first itself, the pivot, is the last r), the
//     scan swaps (l_k, r_k) for k = 1 .. S, S = #{k : l_k < r_k} (a prefix, l rises, r falls),
//     and returns cut = min(l_{S+1}, r_S) (l_{S+1} = +inf when absent, r_0 = last).  Between
//     the two scan pointers the array is untouched, so the stops are those of the original
//     segment; the scan that runs into the swapped region stops at r_S;
//   * the depth-limit heap sort (rare; adversarial inputs) runs on one lane, a literal
//     restatement of __make_heap / __adjust_heap / __push_heap / __pop_heap / __sort_heap;
//   * the final insertion sort is stable and never moves an element out of its <= 16 segment
//     (every key of a left segment is <= every key of a right one), so it equals a stable sort
//     of each small segment: one rank count per element (heap-sorted segments are sorted).
// Checked against std::sort itself: tests/test_gpu_scanreg.py (tied curvatures, adversarial
// median-of-3 inputs) and tests/test_gpu_primitives.py (VoxelGrid in PCL order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace loam {

constexpr int SS_THRESHOLD = 16;  // _S_threshold

// Pending segments of one sort, level by level: the segments of depth level `lev` are in
// seg[lev & 1]: the ones for one wave each at [0, cnt), the long ones (more than SS_BIG elements,
// depth budget left) from the end, at cap - 1 - t for t < nbig; every one longer than 16
// elements.  Segments of one level are disjoint, so a level holds at most n / 17 + 1 (cap).
struct SsLevels {
  int cnt[2];
  int nbig[2];
  int err;
  int cap;
  int* seg[2];  // [cap][3] (lo, hi, depth budget), LDS or global
  uint32_t ws[17];  // block-scan scratch of the cooperative partition
  int sh[2];
  uint32_t* loc;  // optional LDS for wave-local subtree sorts (SS_LOC_WORDS per wave), else nullptr
  // deferral (ss_levels<..., true>, a sort whose elements live in global memory): segments of at
  // most `defer` elements are not partitioned level by level but listed in the caller's
  // dseg[dcap][3] (lo, hi, depth budget), each then sorted whole in LDS (ss_sort_deferred)
  int dcnt, dcap, defer;
  unsigned long long* hctr;  // optional: [0] depth-limit heap sorts, [1] their elements (diagnostics)
};

// Wave-local subtree sort: a segment of at most SS_LOCAL elements whose array lives in global
// memory is copied into the wave's LDS, its whole introsort subtree runs there (a wave-local
// LIFO, no level barriers), and the result goes back with identity annotations.
constexpr int SS_LOCAL = 512;
// pending right parts are disjoint and longer than 16 elements: at most SS_LOCAL / 17 + 1
constexpr int SS_LOC_STK = SS_LOCAL / (SS_THRESHOLD + 1) + 2;
constexpr int SS_LOC_WORDS = 2 * SS_LOCAL + 2 * SS_LOCAL + 3 * SS_LOC_STK;

constexpr int SS_BIG = 1024;  // longer segments are partitioned by the whole workgroup
constexpr int SS_WG_CHUNK = 16;  // positions per thread of a workgroup partition in one pass

// Elements are 64-bit; Less compares two elements (the reference's comparator).  Per sort:
//   E[n]    the elements, permuted in place by the partitions (LDS or global)
//   A[n], B[n]  u32 scratch: partition stop lists, then the final segments' bounds
// the wave's lanes see each other's writes (LDS or global: workgroup scope waits for the
// stores; the CU's L1 is write-through, so no invalidation is needed at this scope)
__device__ inline void ss_wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// libstdc++ __adjust_heap + __push_heap on E[first ..], one lane
template <typename T, typename Less>
__device__ inline void ss_adjust_heap(T* E, int first, int hole, int len, T value, const Less& less) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (less(E[first + second], E[first + second - 1])) second--;
    E[first + hole] = E[first + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    E[first + hole] = E[first + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && less(E[first + parent], value)) {
    E[first + hole] = E[first + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  E[first + hole] = value;
}

__device__ inline void ss_heap_count(unsigned long long* hctr, int m) {
  if (hctr) {
    atomicAdd(hctr, 1ull);
    atomicAdd(hctr + 1, (unsigned long long)m);
  }
}

// __partial_sort(first, last, last): __make_heap then __sort_heap, one lane
template <typename T, typename Less>
__device__ inline void ss_heap_sort(T* E, int lo, int hi, const Less& less) {
  const int len = hi - lo;
  if (len >= 2) {
    int parent = (len - 2) / 2;
    while (true) {
      const T v = E[lo + parent];
      ss_adjust_heap(E, lo, parent, len, v, less);
      if (parent == 0) break;
      parent--;
    }
  }
  int last = hi;
  while (last - lo > 1) {
    --last;
    const T v = E[last];
    E[last] = E[lo];
    ss_adjust_heap(E, lo, 0, last - lo, v, less);
  }
}

// The depth-limit fallback (__partial_sort) of one segment by a wave.  Its result only matters
// where it orders equal keys, and often not even there, so the wave first sorts the segment by
// (key, element) -- by rank up to SS_RANK_MAX elements, else a bitonic network -- and keeps that
// order when it is indistinguishable from the heap's:
//   * Less::free_run is the longest run of equal keys whose internal order cannot show: 1 for
//     sorts whose tie order is visible (scan registration's sector sort, the plain permutation),
//     2 for VoxelGrid (a centroid sums its voxel's points from 0: (0 + a) + b == (0 + b) + a);
//   * a run longer than that inside the segment needs the heap's order;
//   * keys strictly between the segment's smallest and largest have all their elements inside
//     it (the partitions above it cut by pivot values), but the smallest and largest key may
//     have elements in neighbouring segments, so with free_run 2 a pair at either end counts
//     as a longer run.
// Otherwise the segment is restored (A / B hold a copy) and heap-sorted literally on one lane.
// (The exact mode's cube re-filters reach the depth limit on old, already sorted content with a
// few new points appended, where median-of-3 degenerates: segments of thousands of points.)
constexpr int SS_RANK_PER = 4;
constexpr int SS_RANK_MAX = 64 * SS_RANK_PER;

template <typename Less>
__device__ inline bool ss_full_less(uint64_t a, uint64_t b, const Less& less) {
  return less(a, b) || (!less(b, a) && (uint32_t)a < (uint32_t)b);
}

template <typename Less>
__device__ inline void ss_depth_limit(uint64_t* E, uint32_t* A, uint32_t* B, int lo, int hi, const Less& less) {
  const int lane = threadIdx.x & 63;
  const int m = hi - lo;
  for (int i = lane; i < m; i += 64) {  // the copy the heap sort restarts from
    const uint64_t e = E[lo + i];
    A[lo + i] = (uint32_t)e;
    B[lo + i] = (uint32_t)(e >> 32);
  }
  if (m <= SS_RANK_MAX) {
    uint64_t e[SS_RANK_PER];
    int r[SS_RANK_PER];
#pragma unroll
    for (int u = 0; u < SS_RANK_PER; ++u) {
      r[u] = 0;
      if (lane + 64 * u < m) e[u] = E[lo + lane + 64 * u];
    }
    for (int j = 0; j < m; ++j) {
      const uint64_t x = E[lo + j];
#pragma unroll
      for (int u = 0; u < SS_RANK_PER; ++u)
        if (lane + 64 * u < m && ss_full_less(x, e[u], less)) ++r[u];
    }
    ss_wave_fence();  // every read of the segment before the writes
#pragma unroll
    for (int u = 0; u < SS_RANK_PER; ++u)
      if (lane + 64 * u < m) E[lo + r[u]] = e[u];
  } else {  // bitonic network over the next power of two; positions >= m act as +inf
    int K = 1;
    while (K < m) K <<= 1;
    for (int k = 2; k <= K; k <<= 1) {
      for (int j = k >> 1; j >= 1; j >>= 1) {
        ss_wave_fence();
        for (int t = lane; t < (K >> 1); t += 64) {
          const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));  // bit log2(j) of i is 0
          const int l = j == (k >> 1) ? (i ^ (k - 1)) : (i + j);
          if (l < m) {
            const uint64_t a = E[lo + i], b = E[lo + l];
            if (ss_full_less(b, a, less)) {
              E[lo + i] = b;
              E[lo + l] = a;
            }
          }
        }
      }
    }
  }
  ss_wave_fence();
  constexpr int FR = Less::free_run;
  bool keep = true;
  for (int i = lane + FR; i < m; i += 64) keep &= less(E[lo + i - FR], E[lo + i]);
  if (FR >= 2 && m >= 2) keep &= less(E[lo], E[lo + 1]) && less(E[lo + m - 2], E[lo + m - 1]);
  if (__ballot(!keep) == 0ull) return;
  ss_wave_fence();
  for (int i = lane; i < m; i += 64) E[lo + i] = ((uint64_t)B[lo + i] << 32) | A[lo + i];
  ss_wave_fence();
  if (lane == 0) ss_heap_sort(E, lo, hi, less);
  ss_wave_fence();
}

// One segment [lo, hi) with depth budget d: partition and return the cut (wave-uniform)
template <typename T, typename Less>
__device__ inline int ss_partition(T* E, uint32_t* A, uint32_t* B, int lo, int hi, const Less& less) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) {  // __move_median_to_first(lo, lo + 1, mid, hi - 1)
    const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
    const T ea = E[a], eb = E[b], ec = E[c];
    int m;
    if (less(ea, eb)) {
      if (less(eb, ec)) m = b;
      else if (less(ea, ec)) m = c;
      else m = a;
    } else if (less(ea, ec)) {
      m = a;
    } else if (less(eb, ec)) {
      m = c;
    } else {
      m = b;
    }
    const T t = E[lo];
    E[lo] = E[m];
    E[m] = t;
  }
  ss_wave_fence();
  const T p = E[lo];
  // left stops l_k at A[lo + k] (k >= 1), right stops ascending at B[lo + t] (t = 0: the pivot)
  int nl = 0, nr = 1;
  if (lane == 0) B[lo] = (uint32_t)lo;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int c0 = lo + 1; c0 < hi; c0 += 64) {
    const int i = c0 + lane;
    const bool v = i < hi;
    T e{};
    if (v) e = E[i];
    const bool isl = v && !less(e, p);
    const bool isr = v && !less(p, e);
    const uint64_t bl = __ballot(isl), br = __ballot(isr);
    if (isl) A[lo + 1 + nl + __popcll(bl & lt)] = (uint32_t)i;
    if (isr) B[lo + nr + __popcll(br & lt)] = (uint32_t)i;
    nl += __popcll(bl);
    nr += __popcll(br);
  }
  ss_wave_fence();
  // S = #{k <= min(nl, nr) : l_k < r_k}, r_k = B[lo + nr - k]
  const int kmax = min(nl, nr);
  int S = 0;
  for (int k0 = 1; k0 <= kmax; k0 += 64) {
    const int k = k0 + lane;
    const bool pr = k <= kmax && A[lo + k] < B[lo + nr - k];
    const uint64_t b = __ballot(pr);
    S += __popcll(b);
    if (b != ~0ull) break;  // the predicate is a prefix
  }
  const int lK = S + 1 <= nl ? (int)A[lo + S + 1] : 0x7FFFFFFF;
  const int rS = S >= 1 ? (int)B[lo + nr - S] : hi;
  const int cut = min(lK, rS);
  for (int k0 = 1; k0 <= S; k0 += 64) {
    const int k = k0 + lane;
    if (k <= S) {
      const int x = (int)A[lo + k], y = (int)B[lo + nr - k];
      const T ex = E[x], ey = E[y];
      E[x] = ey;
      E[y] = ex;
    }
  }
  ss_wave_fence();
  return cut;
}

// The same partition of one segment by all NT threads of the workgroup (segments longer than
// SS_BIG, the first levels of a large sort, where one wave per segment would leave the others
// idle): the stop lists are built tile by tile with a block scan (left / right counts packed in
// one word), then the prefix length S, the cut and the swaps.
template <int NT, typename T, typename Less>
__device__ inline int ss_partition_wg(T* E, uint32_t* A, uint32_t* B, int lo, int hi, SsLevels* L, const Less& less) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  if (tid == 0) {  // __move_median_to_first(lo, lo + 1, mid, hi - 1)
    const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
    const T ea = E[a], eb = E[b], ec = E[c];
    int m;
    if (less(ea, eb)) {
      if (less(eb, ec)) m = b;
      else if (less(ea, ec)) m = c;
      else m = a;
    } else if (less(ea, ec)) {
      m = a;
    } else if (less(eb, ec)) {
      m = c;
    } else {
      m = b;
    }
    const T t = E[lo];
    E[lo] = E[m];
    E[m] = t;
    B[lo] = (uint32_t)lo;
  }
  __syncthreads();
  const T p = E[lo];
  uint32_t nl = 0, nr = 1;
  const int len = hi - lo - 1;  // the scanned positions lo + 1 .. hi - 1
  if (len <= NT * SS_WG_CHUNK) {
    // each thread classifies a contiguous chunk (its loads all in flight at once), and one block
    // scan of the per-thread stop counts places every stop: no barrier per tile
    const int c = (len + NT - 1) / NT;
    const int b0 = lo + 1 + tid * c;
    uint32_t ml = 0, mr = 0;  // bit u: position b0 + u is a left / right stop
#pragma unroll
    for (int u = 0; u < SS_WG_CHUNK; ++u) {
      const int i = b0 + u;
      if (u < c && i < hi) {
        const T e = E[i];
        if (!less(e, p)) ml |= 1u << u;
        if (!less(p, e)) mr |= 1u << u;
      }
    }
    const uint32_t v = (uint32_t)__popc(ml) | ((uint32_t)__popc(mr) << 16);  // totals < 2^16
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) L->ws[wid] = x;
    __syncthreads();
    uint32_t off = x - v, tot = 0;
    for (int w = 0; w < NW; ++w) {
      const uint32_t t = L->ws[w];
      off += w < wid ? t : 0u;
      tot += t;
    }
    uint32_t ol = (uint32_t)lo + 1u + (off & 0xFFFFu), orr = (uint32_t)lo + 1u + (off >> 16);
#pragma unroll
    for (int u = 0; u < SS_WG_CHUNK; ++u) {
      if (ml & (1u << u)) A[ol++] = (uint32_t)(b0 + u);
      if (mr & (1u << u)) B[orr++] = (uint32_t)(b0 + u);
    }
    nl = tot & 0xFFFFu;
    nr = 1u + (tot >> 16);
    __syncthreads();  // the stop lists complete, ws free
  } else {
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int c0 = lo + 1; c0 < hi; c0 += NT) {
      const int i = c0 + tid;
      bool isl = false, isr = false;
      if (i < hi) {
        const T e = E[i];
        isl = !less(e, p);
        isr = !less(p, e);
      }
      const uint64_t bl = __ballot(isl), br = __ballot(isr);
      if (lane == 0) L->ws[wid] = (uint32_t)__popcll(bl) | ((uint32_t)__popcll(br) << 16);
      __syncthreads();
      uint32_t off = 0, tot = 0;
      for (int w = 0; w < NW; ++w) {
        const uint32_t v = L->ws[w];
        off += w < wid ? v : 0u;
        tot += v;
      }
      if (isl) A[lo + 1 + nl + (off & 0xFFFFu) + __popcll(bl & lt)] = (uint32_t)i;
      if (isr) B[lo + nr + (off >> 16) + __popcll(br & lt)] = (uint32_t)i;
      nl += tot & 0xFFFFu;
      nr += tot >> 16;
      __syncthreads();  // ws is rewritten by the next tile
    }
  }
  const int kmax = min((int)nl, (int)nr);
  if (tid == 0) L->sh[0] = kmax + 1;  // first k with !(l_k < r_k)
  __syncthreads();
  for (int k0 = 1; k0 <= kmax; k0 += NT) {
    const int k = k0 + tid;
    if (k <= kmax && !(A[lo + k] < B[lo + nr - k])) atomicMin(&L->sh[0], k);
    __syncthreads();
    const int ff = L->sh[0];
    __syncthreads();
    if (ff <= kmax) break;
  }
  const int S = L->sh[0] - 1;
  const int lK = S + 1 <= (int)nl ? (int)A[lo + S + 1] : 0x7FFFFFFF;
  const int rS = S >= 1 ? (int)B[lo + nr - S] : hi;
  const int cut = min(lK, rS);
  for (int k0 = 1; k0 <= S; k0 += NT) {
    const int k = k0 + tid;
    if (k <= S) {
      const int x = (int)A[lo + k], y = (int)B[lo + nr - k];
      const T ex = E[x], ey = E[y];
      E[x] = ey;
      E[y] = ex;
    }
  }
  __syncthreads();
  return cut;
}

// Record a final segment for the stable per-segment pass
__device__ inline void ss_mark(uint32_t* A, uint32_t* B, int lo, int hi, bool sorted) {
  const int lane = threadIdx.x & 63;
  for (int i = lo + lane; i < hi; i += 64) {
    A[i] = sorted ? (uint32_t)i : (uint32_t)lo;
    B[i] = sorted ? (uint32_t)(i + 1) : (uint32_t)hi;
  }
}

template <typename T, typename Less>
__device__ inline void ss_local_sort(T* E, uint32_t* A, uint32_t* B, int lo, int hi, int d, uint32_t* loc,
                                     const Less& less, unsigned long long* hctr = nullptr) {
  const int lane = threadIdx.x & 63;
  const int m = hi - lo;
  T* lE = reinterpret_cast<T*>(loc);
  uint32_t* lA = loc + 2 * SS_LOCAL;
  uint32_t* lB = lA + SS_LOCAL;
  int* stk = reinterpret_cast<int*>(lB + SS_LOCAL);
  for (int i = lane; i < m; i += 64) lE[i] = E[lo + i];
  if (lane == 0) {
    stk[0] = 0;
    stk[1] = m;
    stk[2] = d;
  }
  int top = 1;
  ss_wave_fence();
  while (top > 0) {
    --top;
    int a = __builtin_amdgcn_readfirstlane(stk[3 * top]);
    int b = __builtin_amdgcn_readfirstlane(stk[3 * top + 1]);
    int dd = __builtin_amdgcn_readfirstlane(stk[3 * top + 2]);
    while (true) {
      if (b - a <= SS_THRESHOLD) {
        ss_mark(lA, lB, a, b, false);
        break;
      }
      if (dd == 0) {
        if (lane == 0) ss_heap_count(hctr, b - a);
        ss_depth_limit(lE, lA, lB, a, b, less);
        ss_mark(lA, lB, a, b, true);
        break;
      }
      --dd;
      const int cut = __builtin_amdgcn_readfirstlane(ss_partition(lE, lA, lB, a, b, less));
      if (b - cut > SS_THRESHOLD) {
        if (lane == 0) {
          stk[3 * top] = cut;
          stk[3 * top + 1] = b;
          stk[3 * top + 2] = dd;
        }
        ++top;
      } else {
        ss_mark(lA, lB, cut, b, false);
      }
      ss_wave_fence();
      b = cut;
    }
  }
  ss_wave_fence();
  // the final insertion sort of the subtree (stable within each final segment) -> E[lo ..)
  for (int i = lane; i < m; i += 64) {
    const int a = (int)lA[i], b = (int)lB[i];
    const T ei = lE[i];
    int r = 0;
    for (int j = a; j < b; ++j) {
      const T ej = lE[j];
      r += (less(ej, ei) || (j < i && !less(ei, ej))) ? 1 : 0;
    }
    E[lo + a + r] = ei;
  }
  for (int i = lane; i < m; i += 64) {  // sorted in place: ss_final copies it through
    A[lo + i] = (uint32_t)(lo + i);
    B[lo + i] = (uint32_t)(lo + i + 1);
  }
  ss_wave_fence();
}

// Init with the root segment [0, n) (one thread; a barrier / wave fence before ss_levels).
// depth: the root's depth budget (< 0: 2 * __lg(n), std::sort's; a deferred subtree's own).
__device__ inline void ss_levels_init(SsLevels* L, int n, int* seg0, int* seg1, int cap, int depth = -1) {
  L->seg[0] = seg0;
  L->seg[1] = seg1;
  L->cap = cap;
  L->err = 0;
  L->cnt[0] = L->cnt[1] = L->nbig[0] = L->nbig[1] = 0;
  L->loc = nullptr;
  L->dcnt = L->dcap = L->defer = 0;
  L->hctr = nullptr;
  if (n > SS_THRESHOLD) {
    const int d = depth >= 0 ? depth : 2 * (31 - __clz(n));  // 2 * __lg(n)
    const bool big = n > SS_BIG && d > 0;
    int* o = seg0 + 3 * (big ? cap - 1 : 0);
    o[0] = 0;
    o[1] = n;
    o[2] = d;
    if (big) L->nbig[0] = 1;
    else L->cnt[0] = 1;
  }
}

// The introsort loop over [0, n), level by level.  Every wave of the group calls it (WG: the
// whole workgroup, barriers are __syncthreads; else one wave alone); waves w < nw take the
// level's segments w, w + nw, ...  No waiting on other waves outside the barriers, and at most
// 2 * __lg(n) + 1 levels (each level lowers the depth budget by one).
// The list / buffer pointers are arguments (not read back from L, which lives in LDS): named
// directly from __shared__ arrays at the call site they keep their LDS address space, so the
// compiler emits ds_* instead of flat_* accesses.
template <bool WG, int NT = 64, bool DEFER = false, typename T, typename Less>
__device__ inline void ss_levels(T* E, uint32_t* A, uint32_t* B, SsLevels* L, int wave, int nw, const Less& less,
                                 int* seg0, int* seg1, uint32_t* loc, int* dseg = nullptr) {
  const int lane = threadIdx.x & 63;
  int* const segs[2] = {seg0, seg1};
  auto barrier = [] {
    if (WG) __syncthreads();
    else ss_wave_fence();
  };
  auto push = [&](int nxt, int a, int b, int d) {  // one lane
    if (DEFER && b - a <= L->defer && (d > 0 || b - a > SS_RANK_MAX)) {  // sorted whole later in LDS (ss_sort_deferred)
      const int t = atomicAdd(&L->dcnt, 1);
      if (t < L->dcap) {
        int* o = dseg + 3 * t;
        o[0] = a;
        o[1] = b;
        o[2] = d;
      } else {
        atomicOr(&L->err, 2);
      }
      return;
    }
    const bool big = b - a > SS_BIG && d > 0;
    const int t = atomicAdd(big ? &L->nbig[nxt] : &L->cnt[nxt], 1);
    const int slot = big ? L->cap - 1 - t : t;
    if (t < L->cap && slot >= 0) {
      int* o = segs[nxt] + 3 * slot;
      o[0] = a;
      o[1] = b;
      o[2] = d;
    } else {
      atomicOr(&L->err, 2);
    }
  };
  for (int lev = 0;; ++lev) {
    barrier();
    const int cur = lev & 1, nxt = cur ^ 1;
    const int cnt = L->cnt[cur], nb = L->nbig[cur];
    if (cnt + nb == 0) break;
    if (cnt + nb > L->cap) {  // the two ends met: the lists were overwritten (cannot happen with cap >= n / 17 + 1)
      if (threadIdx.x == 0) atomicOr(&L->err, 2);
      break;
    }
    const int* sg = segs[cur];
    if (WG) {  // long segments: the whole workgroup on each in turn
      for (int t = 0; t < nb; ++t) {
        const int* e = sg + 3 * (L->cap - 1 - t);
        const int lo = e[0], hi = e[1], d = e[2];
        const int cut = ss_partition_wg<NT>(E, A, B, lo, hi, L, less);
        const int parts[2][2] = {{lo, cut}, {cut, hi}};
        for (int q = 0; q < 2; ++q) {
          const int a = parts[q][0], b = parts[q][1];
          if (b - a > SS_THRESHOLD) {
            if (threadIdx.x == 0) push(nxt, a, b, d - 1);
          } else {
            for (int i = a + (int)threadIdx.x; i < b; i += NT) {
              A[i] = (uint32_t)a;
              B[i] = (uint32_t)b;
            }
          }
        }
        __syncthreads();
      }
    }
    // one wave per segment (and, for a single wave, the long ones too)
    const int tot = WG ? cnt : cnt + nb;
    for (int k = wave; wave < nw && k < tot; k += nw) {
      const int* e = sg + 3 * (k < cnt ? k : L->cap - 1 - (k - cnt));
      const int lo = e[0], hi = e[1], d = e[2];
      if (loc && hi - lo <= SS_LOCAL) {
        ss_local_sort(E, A, B, lo, hi, d, loc + wave * SS_LOC_WORDS, less, L->hctr);
        continue;
      }
      if (d == 0) {  // depth limit: __partial_sort(first, last, last)
        if (lane == 0) ss_heap_count(L->hctr, hi - lo);
        ss_depth_limit(E, A, B, lo, hi, less);
        ss_mark(A, B, lo, hi, true);
        continue;
      }
      const int cut = ss_partition(E, A, B, lo, hi, less);
      const int parts[2][2] = {{lo, cut}, {cut, hi}};
      for (int q = 0; q < 2; ++q) {
        const int a = parts[q][0], b = parts[q][1];
        if (b - a > SS_THRESHOLD) {
          if (lane == 0) push(nxt, a, b, d - 1);
        } else {
          ss_mark(A, B, a, b, false);
        }
      }
    }
    barrier();  // every append to level lev + 1 done, every read of this level's count done
    if (wave == 0 && lane == 0) L->cnt[cur] = L->nbig[cur] = 0;
  }
}

// The final stable pass: out[lo + rank] = E[i] for every i (all threads of the caller's
// group call it with their index t of nt; small inputs (n <= 16) are one segment)
template <typename T, typename Less>
__device__ inline void ss_final(const T* E, const uint32_t* A, const uint32_t* B, int n, T* out, int t, int nt,
                                const Less& less) {
  for (int i = t; i < n; i += nt) {
    int lo, hi;
    if (n <= SS_THRESHOLD) {
      lo = 0;
      hi = n;
    } else {
      lo = (int)A[i];
      hi = (int)B[i];
    }
    const T ei = E[i];
    int r = 0;
    for (int j = lo; j < hi; ++j) {
      const T ej = E[j];
      r += (less(ej, ei) || (j < i && !less(ei, ej))) ? 1 : 0;
    }
    out[lo + r] = ei;
  }
}

// The deferred segments of a sort in global memory (ss_levels with L->defer), one after the
// other by the whole workgroup: the segment is copied into LDS (lE / lA / lB, level lists
// lseg0 / lseg1 of lcap entries, state LL), its whole introsort subtree runs there with the
// depth budget it was deferred with, and the final stable pass writes it back sorted; its
// bounds become the identity (sorted in place, like ss_local_sort).  Segments are disjoint and
// independent, so this order gives std::sort's permutation.
template <int NT, typename T, typename Less>
__device__ inline void ss_sort_deferred(T* E, uint32_t* A, uint32_t* B, SsLevels* L, const int* dseg, const Less& less,
                                        T* lE, uint32_t* lA, uint32_t* lB, int* lseg0, int* lseg1, int lcap,
                                        SsLevels* LL) {
  const int tid = threadIdx.x;
  __syncthreads();
  const int nd = min(L->dcnt, L->dcap);
  for (int k = 0; k < nd; ++k) {
    const int lo = dseg[3 * k], hi = dseg[3 * k + 1], d = dseg[3 * k + 2];
    const int m = hi - lo;
    for (int i = tid; i < m; i += NT) lE[i] = E[lo + i];
    if (tid == 0) {
      ss_levels_init(LL, m, lseg0, lseg1, lcap, d);
      LL->hctr = L->hctr;
    }
    __syncthreads();
    ss_levels<true, NT>(lE, lA, lB, LL, tid >> 6, NT / 64, less, lseg0, lseg1, nullptr);
    __syncthreads();
    if (tid == 0 && LL->err) atomicOr(&L->err, LL->err);
    ss_final(lE, lA, lB, m, E + lo, tid, NT, less);
    for (int i = tid; i < m; i += NT) {
      A[lo + i] = (uint32_t)(lo + i);
      B[lo + i] = (uint32_t)(lo + i + 1);
    }
    __syncthreads();
  }
}

}  // namespace loam
