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
//   * segments are independent, so any processing order gives the same result; waves pop
//     segments from a shared LDS stack (one wave per segment);
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

// Shared state of one sort (LDS): a stack of pending segments guarded by a lock, and the
// count of segments not yet finished (the exit condition every wave reaches).
struct SsCtl {
  int lock;
  int top;
  int pending;
  int err;
};

// Elements are 64-bit; Less compares two elements (the reference's comparator).  Per sort:
//   E[n]    the elements, permuted in place by the partitions (LDS or global)
//   A[n+1], B[n+1]  u32 scratch: partition stop lists, then the small-segment bounds
//   stk     3 * stk_cap ints of LDS
// the wave's lanes see each other's writes (LDS or global: workgroup scope waits for the
// stores; the CU's L1 is write-through, so no invalidation is needed at this scope)
__device__ inline void ss_wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ inline void ss_lock(SsCtl* c) {
  while (atomicCAS(&c->lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ inline void ss_unlock(SsCtl* c) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  atomicExch(&c->lock, 0);
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

// Record a final segment for the stable per-segment pass
__device__ inline void ss_mark(uint32_t* A, uint32_t* B, int lo, int hi, bool sorted) {
  const int lane = threadIdx.x & 63;
  for (int i = lo + lane; i < hi; i += 64) {
    A[i] = sorted ? (uint32_t)i : (uint32_t)lo;
    B[i] = sorted ? (uint32_t)(i + 1) : (uint32_t)hi;
  }
}

// The introsort loop over [0, n), run by every wave that shares `ctl` (nw waves call it);
// the caller initialised ctl (ss_init) and a barrier separates that from this call.
// stk_cap: stack entries.  max_spins bounds the idle waiting (ctl->err set when exceeded).
template <typename T, typename Less>
__device__ inline void ss_loop(T* E, uint32_t* A, uint32_t* B, SsCtl* ctl, int* stk, int stk_cap,
                               const Less& less) {
  const int lane = threadIdx.x & 63;
  int spins = 0;
  while (true) {
    int lo = 0, hi = 0, d = -1, state = 0;  // state: 0 got a segment, 1 idle, 2 done
    if (lane == 0) {
      ss_lock(ctl);
      if (ctl->top > 0) {
        const int t = --ctl->top;
        lo = stk[3 * t];
        hi = stk[3 * t + 1];
        d = stk[3 * t + 2];
      } else {
        state = ctl->pending == 0 ? 2 : 1;
      }
      ss_unlock(ctl);
    }
    state = __builtin_amdgcn_readfirstlane(state);
    if (state == 2) break;
    if (state == 1) {
      if (++spins > (1 << 22)) {  // cannot happen while the waves progress; never hang
        if (lane == 0) atomicOr(&ctl->err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    d = __builtin_amdgcn_readfirstlane(d);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // run this segment down its left spine, pushing the right parts
    while (true) {
      if (hi - lo <= SS_THRESHOLD) {
        ss_mark(A, B, lo, hi, false);
        break;
      }
      if (d == 0) {
        if (lane == 0) ss_heap_sort(E, lo, hi, less);
        ss_wave_fence();
        ss_mark(A, B, lo, hi, true);
        break;
      }
      --d;
      const int cut = ss_partition(E, A, B, lo, hi, less);
      // right part [cut, hi) to the stack (other waves may take it), continue with the left
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (hi - cut > SS_THRESHOLD) {
        if (lane == 0) {
          ss_lock(ctl);
          const int t = ctl->top;
          if (t < stk_cap) {
            stk[3 * t] = cut;
            stk[3 * t + 1] = hi;
            stk[3 * t + 2] = d;
            ctl->top = t + 1;
            ctl->pending += 1;
          } else {
            ctl->err |= 2;
          }
          ss_unlock(ctl);
        }
      } else {
        ss_mark(A, B, cut, hi, false);
      }
      hi = cut;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) {
      ss_lock(ctl);
      ctl->pending -= 1;
      ss_unlock(ctl);
    }
    spins = 0;
  }
}

// Init of the shared state with the root segment [0, n), by one thread (then a barrier / wave
// fence before ss_loop)
__device__ inline void ss_init(SsCtl* ctl, int* stk, int n) {
  ctl->lock = 0;
  ctl->err = 0;
  if (n > SS_THRESHOLD) {
    int lg = 31 - __clz(n);
    stk[0] = 0;
    stk[1] = n;
    stk[2] = 2 * lg;
    ctl->top = 1;
    ctl->pending = 1;
  } else {
    ctl->top = 0;
    ctl->pending = 0;
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

}  // namespace loam
