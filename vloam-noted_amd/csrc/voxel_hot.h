// voxel_hot.h — PCL's VoxelGrid summation order (std::sort's permutation) for the voxels where it
// shows, LDS-resident, pruned to the segments that can still reorder such a voxel.
//
// PCL 1.8-1.12 voxel_grid.hpp applyFilter sorts (idx, point) pairs with std::sort on idx alone
// and sums each voxel's points in the sorted order (laser_mapping.cpp:492-500, :795-808,
// scan_registration.cpp:497-501).  Float addition is not associative, but a voxel with at most
// two members sums alike in either order ((0 + a) + b == (0 + b) + a), so only voxels with 3 or
// more members ("hot") need that order.  And the order is cheap to read off: libstdc++'s
// __final_insertion_sort is stable and never moves an element out of its final segment, so the
// members of a voxel end in the order of their positions once the partitions (and the depth-limit
// heap sorts) are done.  Hence, per filter:
//   phase 1 (voxel.h, the input-order filter): every cold voxel's centroid (exact: order-free);
//            per point its output slot and hot bit (VxHot::rk); the hot voxels' member lists;
//   phase 2 (vh_sort): libstdc++'s __introsort_loop on E[i] = slot << 16 | hot << 15 | i in LDS,
//            exactly (stdsort.h's parallel Hoare formulation), except that
//              * a segment holding fewer than two hot elements is not partitioned: nothing below
//                it can reorder two members of one hot voxel;
//              * a depth-limit segment is heap-sorted (literally, one lane) only when two members
//                of one hot voxel lie in it, else left as it is;
//              * the final insertion sort is skipped (it keeps the position order);
//            then each hot point's position -> VxHot::fpos;
//   phase 3 (vh_centroids): each hot voxel summed in its members' position order.
// The rule is pinned against libstdc++ itself on cube- and stack-shaped clouds
// (tests/test_sort_rule.py::test_hot_pruned_rule_keeps_pcl_centroids) and on the GPU against the
// oracle (tests/test_gpu_primitives.py, the mapping and long-stream tests in exact mode).
//
// Workgroup partitions (segments over VH_BIG elements, the first levels and the degenerate chains
// of cube re-filters): each thread classifies a contiguous chunk held in registers, one block scan
// places the stops; wave partitions (the subtrees below VH_BIG) run without barriers, one wave
// each, smaller part first.  The Hoare scan's swap pairs (l_k, r_k) come from the test
// l_k < r_k  <=>  k <= #(right stops right of l_k), so only r_1 .. r_{(m-1)/2} are listed (u16,
// a segment [lo, hi) owns Bs[lo/2 ..)), and every read of the segment precedes every write.
#pragma once
#include <cstdlib>
#include <mutex>

#include "stdsort.h"
#include "voxel.h"

namespace loam {

constexpr int VH_BIG = 1024;      // longer segments: partitioned by the workgroup
constexpr int VH_MAX_N = 30720;   // LDS-resident emulation up to this many points (30 per thread)
constexpr int VH_CHUNK = VH_MAX_N / VX_THREADS;  // positions per thread of a workgroup partition
constexpr int VH_ROOTS = 512;     // wave subtrees listed per drain
constexpr int VH_SHARE = 96;      // a wave lists the larger part of a partition when longer and it has the smaller part to do
constexpr int VH_BIGC = 32;       // workgroup segments of one level (segments > VH_BIG are disjoint: <= 30)
constexpr int VH_LIFO = 8;        // wave-local pending parts (smaller part first: depth <= 6)
constexpr int VH_WAVE_W = VH_LIFO + 64;  // per wave: LIFO + the dup check's keys
constexpr int VH_SMALL = 32;      // hot voxels up to this many members: summed by one thread
constexpr int VH_REG = 8;         // hot voxels up to 64 * VH_REG members: rank-sorted by a wave
constexpr uint32_t VH_HOT = 0x8000u;
// error bits (above the mapper's MAP_ERR_* and scan registration's SR_ERR_*, which share the
// flag words these are or-ed into): a list overflow (cannot happen), a drain wait that ran out
constexpr int VH_ERR_ROOTS = 1 << 12, VH_ERR_LIST = 1 << 13, VH_ERR_SPIN = 1 << 14;
constexpr int VH_ERR_ANY = VH_ERR_ROOTS | VH_ERR_LIST | VH_ERR_SPIN;

// The drain's bounded wait (vh_drain): spins of a wave whose claimed list entry is not listed yet
// while some listed subtree is unfinished.  2^24 spins of s_sleep 1 (~seconds) cannot run out
// while the workgroup makes progress; when it does, the subtree that entry would have held is
// left unsorted, so the filter flags VH_ERR_SPIN (-> LOAM_ERR_SYNC) instead of a silently wrong
// centroid.  LOAM_VH_SPIN_LIMIT (environment) lowers it: tests/test_gpu_vh_spin.py sets 0 to show
// the flag reaches the caller.  vh_spin_limit_from_env(device) writes it once per device of this
// translation unit's code object; the caller has made `device` current (hipMemcpyToSymbol writes
// the current device's copy), and handles created from several threads serialise on the mutex.
static __device__ uint32_t vh_spin_limit_g = 1u << 24;
static inline void vh_spin_limit_from_env(int device) {
  const char* e = getenv("LOAM_VH_SPIN_LIMIT");
  if (!e || device < 0 || device >= 64) return;
  static std::mutex mu;
  static uint64_t done = 0;  // bit d: device d written
  std::lock_guard<std::mutex> lk(mu);
  if ((done >> device) & 1ull) return;
  const uint32_t v = (uint32_t)strtoul(e, nullptr, 10);
  if (hipMemcpyToSymbol(HIP_SYMBOL(vh_spin_limit_g), &v, sizeof(v)) == hipSuccess) done |= 1ull << device;
}

struct VhLess {
  __device__ bool operator()(uint32_t a, uint32_t b) const { return (a >> 16) < (b >> 16); }
};

struct VhLvl {  // the workgroup partitions of one level, all its segments at once
  int tstart[VH_BIGC + 1];   // each segment's first thread (and the end)
  int hot[VH_BIGC], S[VH_BIGC], cut[VH_BIGC];
  uint32_t base[VH_BIGC], endv[VH_BIGC];  // the packed scan before the segment's first thread / after its last
  int c;                     // positions per thread
};

struct VhCtl {
  VhLvl lv;
  int nbig[2];               // workgroup segments of this / the next level
  int nroot, root_take;      // wave subtrees listed, the next one to claim
  int pending;               // listed subtrees not finished (a drain ends at 0)
  int dup;
  int err;
  int heap_el;  // elements heap-sorted literally (diagnostics)
  unsigned long long* dprof;  // optional detail counters (diagnostics): wave partitions by size
                              // class (5), wave busy cycles in drains, the longest wave's, heap-sort
                              // cycles, subtrees
  uint32_t ws[VX_WAVES + 1];  // block-scan scratch of the workgroup partition
};

// a wave subtree / LIFO entry: lo (15 bits) | length (11 bits) | depth budget (5 bits)
__device__ inline uint32_t vh_pack(int lo, int len, int d) {
  return (uint32_t)lo | ((uint32_t)len << 15) | ((uint32_t)d << 26);
}

struct VhLds {
  uint32_t* E;
  uint16_t* Bs;
  uint32_t* roots;
  uint32_t* bigl;  // [2][VH_BIGC]: lo | hi << 15
  uint32_t* wave;  // [waves][VH_WAVE_W]
  VhCtl* C;
};

template <int NT>
__device__ inline VhLds vh_layout(uint32_t* lds, int n) {
  VhLds L;
  L.E = lds;
  L.Bs = reinterpret_cast<uint16_t*>(lds + n);
  L.roots = lds + n + n / 4 + 2;
  L.bigl = L.roots + VH_ROOTS;
  L.wave = L.bigl + 2 * VH_BIGC;
  L.C = reinterpret_cast<VhCtl*>(L.wave + (NT / 64) * VH_WAVE_W);
  return L;
}
template <int NT>
constexpr int vh_lds_words(int n) {
  return n + n / 4 + 2 + VH_ROOTS + 2 * VH_BIGC + (NT / 64) * VH_WAVE_W + (int)(sizeof(VhCtl) / 4) + 1;
}
static_assert(vh_lds_words<VX_THREADS>(VH_MAX_N) <= VX_LDS_WORDS - 256, "hot sort LDS layout");

// One segment [lo, hi) (65 < m <= 64 U + 1) partitioned by one wave: lane l classifies the c
// consecutive positions lo + 1 + l c .. (c = ceil((m - 1) / 64) <= U) into two bit masks, one
// DPP scan of the packed counts places every stop, and the lane walks its positions in order
// (ranks by counting, no per-chunk ballots).  Returns the cut, or -1 when fewer than two hot
// elements lie in it (nothing to do below it).  Every lane returns the same.
template <int U>
__device__ inline int vh_partition_wave_u(uint32_t* E, uint16_t* Bs, int lo, int hi) {
  static_assert(U <= 32, "masks in one word");
  const int lane = threadIdx.x & 63;
  // __move_median_to_first on every lane: the classification sees the swap, lane 0 makes it later
  const VhLess less;
  const uint32_t elo = E[lo];
  int mm;
  uint32_t pe;
  {
    const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
    const uint32_t ea = E[a], eb = E[b], ec = E[c];
    if (less(ea, eb)) {
      if (less(eb, ec)) mm = b;
      else if (less(ea, ec)) mm = c;
      else mm = a;
    } else if (less(ea, ec)) {
      mm = a;
    } else if (less(eb, ec)) {
      mm = c;
    } else {
      mm = b;
    }
    pe = mm == a ? ea : (mm == b ? eb : ec);
  }
  const uint32_t p = pe >> 16;
  const int c = (hi - lo - 1 + 63) >> 6;
  const int b0 = lo + 1 + lane * c;
  uint32_t ml = 0, mr = 0, nh = 0;
  {
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = E[min(b0 + u, hi - 1)];  // (clamped: every load issued at once)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = b0 + u;
      const uint32_t x = i == mm ? elo : e[u];
      const uint32_t in = (u < c && i < hi) ? 1u : 0u;
      const uint32_t k = x >> 16;
      ml |= (in & (k < p ? 0u : 1u)) << u;
      mr |= (in & (p < k ? 0u : 1u)) << u;
      nh += in & ((x & VH_HOT) ? 1u : 0u);
    }
  }
  if (dpp_wave_sum_u(nh) + ((pe & VH_HOT) ? 1u : 0u) < 2u) return -1;
  ss_wave_fence();  // every lane's reads of E before the median swap
  if (lane == 0) {
    E[lo] = pe;
    E[mm] = elo;
  }
  const uint32_t v = (uint32_t)__popc(ml) | ((uint32_t)__popc(mr) << 16);  // totals < 2^16
  const uint32_t x = dpp_incl_scan_u(v);
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  const uint32_t off = x - v;
  const int nr = 1 + (int)(tot >> 16), nl = (int)(tot & 0xFFFFu);
  const int m = hi - lo, KB = (m - 1) / 2, bb = lo >> 1;
  uint32_t S = 0;
  {
    // (bitwise counts: straight-line code, only the Bs stores predicated)
    int kl = (int)(off & 0xFFFFu), t = 1 + (int)(off >> 16);  // t: ascending right-stop index
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int isl = (int)((ml >> u) & 1u), isr = (int)((mr >> u) & 1u);
      kl += isl;
      S += (uint32_t)(isl & (kl <= nr - (t + isr) ? 1 : 0));
      if (isr & (nr - t <= KB ? 1 : 0)) Bs[bb + nr - t - 1] = (uint16_t)(b0 + u);
      t += isr;
    }
    if (lane == 0 && nr <= KB) Bs[bb + nr - 1] = (uint16_t)lo;
  }
  S = dpp_wave_sum_u(S);
  ss_wave_fence();
  // the swaps (each pair (l_k, r_k), k <= S, read and written by the lane of l_k alone: l_k < cut
  // <= r_k, no position is in two pairs) and l_{S+1}, four of a lane's positions at a time: their
  // r_k at once, then E[r_k] and E[l_k] at once (two LDS latencies per four, not two per one),
  // then the writes (later groups read other pairs' positions only)
  int lK = 0x7FFFFFFF;
  {
    int kl = (int)(off & 0xFFFFu);
    constexpr int G = U < 4 ? U : 4;
#pragma unroll
    for (int u0 = 0; u0 < U; u0 += G) {
      int y[G];
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int isl = (int)((ml >> (u0 + j)) & 1u);
        kl += isl;
        const bool sw = isl && kl <= (int)S;
        y[j] = (int)Bs[sw ? bb + kl - 1 : bb] | (sw ? 0 : 0x10000);  // (bit 16: no swap)
        lK = (isl && kl == (int)S + 1) ? b0 + u0 + j : lK;
      }
      uint32_t tv[G], lv[G];
#pragma unroll
      for (int j = 0; j < G; ++j) {
        tv[j] = E[y[j] & 0xFFFF];
        lv[j] = E[(y[j] & 0x10000) ? b0 : b0 + u0 + j];
      }
      ss_wave_fence();
#pragma unroll
      for (int j = 0; j < G; ++j) {
        if (!(y[j] & 0x10000)) {
          E[y[j]] = lv[j];
          E[b0 + u0 + j] = tv[j];
        }
      }
    }
  }
  const uint64_t hk = __ballot(lK != 0x7FFFFFFF);  // at most one lane holds l_{S+1}
  const int lKs = (int)S + 1 <= nl ? __builtin_amdgcn_readlane(lK, __ffsll((unsigned long long)hk) - 1) : 0x7FFFFFFF;
  const int rS = S >= 1 ? (int)Bs[bb + S - 1] : hi;
  ss_wave_fence();
  return __builtin_amdgcn_readfirstlane(min(lKs, rS));
}
__device__ inline int vh_partition_wave(uint32_t* E, uint16_t* Bs, int lo, int hi, unsigned long long* dp = nullptr) {
  static_assert(VH_BIG == 1024, "size classes");
  const int m = hi - lo;  // positions lo + 1 .. hi - 1: m - 1 of them
  if (dp && (threadIdx.x & 63) == 0) atomicAdd(dp + (m <= 65 ? 0 : m <= 129 ? 1 : m <= 257 ? 2 : m <= 513 ? 3 : 4), 1ull);
  if (m <= 129) return vh_partition_wave_u<2>(E, Bs, lo, hi);
  if (m <= 257) return vh_partition_wave_u<4>(E, Bs, lo, hi);
  if (m <= 513) return vh_partition_wave_u<8>(E, Bs, lo, hi);
  return vh_partition_wave_u<16>(E, Bs, lo, hi);
}

// libstdc++'s __partial_sort(first, last, last) (= __make_heap + __sort_heap) on E[lo, hi), one
// whole wave, the same permutation as the one-lane restatement ss_heap_sort:
//   * __make_heap calls __adjust_heap(parent) for parent = (len - 2) / 2 down to 0; one call only
//     touches the parent's subtree, so the parents of one depth (disjoint subtrees, all after
//     the deeper ones) run on separate lanes;
//   * each __pop_heap's hole descends to a leaf along the larger children (the right one unless
//     right < left).  The wave loads the 5 levels below the hole at once (62 lanes) and decides
//     every sibling pair with one DPP shift and one ballot; the scalar unit follows the path
//     through the ballot bits (no lane reads on the chain) and keeps it as a bit code: path node
//     j is (1 << j) - 1 + (the code's first j bits).  Then every lane loads its path node's child
//     at once, the path's values shift up one place, and __push_heap's value lands below the
//     lowest ancestor not less than it (the path is non-increasing downwards: one ballot).
// __make_heap on E[lo, hi), one wave: the parents of one depth on separate lanes
__device__ inline void vh_make_heap_wave(uint32_t* E, int lo, int hi) {
  const int lane = threadIdx.x & 63;
  const VhLess less;
  const int len = hi - lo;
  const int pmax = (len - 2) / 2;
  for (int d = 31 - __clz(pmax + 1); d >= 0; --d) {
    const int a = (1 << d) - 1, b = min(pmax, (1 << (d + 1)) - 2);
    for (int p = b - lane; p >= a; p -= 64) ss_adjust_heap(E, lo, p, len, E[lo + p], less);
    ss_wave_fence();
  }
}

// __sort_heap on the heap E[lo, hi) in LDS, one wave: its first `pops` pops (the rest of the heap
// is then left as a heap)
__device__ inline void vh_sort_heap_wave(uint32_t* E, int lo, int hi, int pops) {
  const int lane = threadIdx.x & 63;
  const VhLess less;
  // lane l < 62 of a look-ahead: depth lj = 1 .. 5 below the hole, index lt in that depth
  const int lj = 31 - __clz(lane + 2), lt = lane + 2 - (1 << lj);
  for (int last = hi - 1; last > hi - 1 - pops; --last) {
    const int n = last - lo;
    const uint32_t v = E[last], top = E[lo];
    const int lim = (n - 1) / 2;
    int h = 0, k = 0;  // hole; path length
    uint32_t code = 0;  // the path's directions, first step highest (k <= 15)
    while (h < lim) {
      const int node = ((h + 1) << lj) - 1 + lt;
      const uint32_t x = (lane < 62 && node < n) ? E[lo + node] : 0u;
      const uint32_t xr = dpp_from_next(x);  // the right sibling (left children: lt even)
      const uint64_t rw = __ballot(!less(xr, x));
      int tt = 0;
#pragma unroll
      for (int jj = 0; jj < 5; ++jj) {
        if (h >= lim) break;
        const int dir = (int)((rw >> ((1 << (jj + 1)) - 2 + 2 * tt)) & 1ull);
        h = 2 * h + 1 + dir;
        tt = 2 * tt + dir;
        code = 2 * code + (uint32_t)dir;
        ++k;
      }
    }
    if ((n & 1) == 0 && h == (n - 2) / 2) {  // one child left
      h = 2 * h + 1;
      code = 2 * code;
      ++k;
    }
    // lane j < k: path node j (its position hj) takes the value of path node j + 1 (pv)
    const int j1 = lane + 1;
    const int hj = lane == 0 || lane > k ? 0 : (1 << lane) - 1 + (int)(code >> (k - lane));
    const int cj = j1 <= k ? (1 << j1) - 1 + (int)(code >> (k - j1)) : 0;
    const uint32_t pv = lane < k ? E[lo + cj] : 0u;
    // __push_heap: v rises while its parent is less; it stops at q = k - #{j < k : pv_j < v}
    const int q = k - __popcll(__ballot(lane < k && less(pv, v)));
    ss_wave_fence();  // every read of this pop before its writes
    if (lane < q) E[lo + hj] = pv;
    if (lane == q) E[lo + hj] = v;
    if (lane == 0) E[last] = top;
    ss_wave_fence();
  }
}

// compiler-only ordering of one wave's LDS accesses: the LDS executes a wave's instructions in
// order, so a lane's read in the next round sees another lane's write of this one
__device__ inline void vh_lds_order() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// one round of every sifting pop (n != 0: its heap size, 0 once its sift ended) from the hole's
// children a, b (c1 = 2 h + 1, loaded at min(c1, npops - 1)): the larger one (right unless
// right < left) moves up while it is not less than v, else v is put and the sift ends
__device__ inline void vh_pipe_move(uint32_t* Eb, int& h, int& n, uint32_t v, int c1, uint32_t a, uint32_t b) {
  const bool right = c1 + 1 < n && (b >> 16) >= (a >> 16);
  const uint32_t cv = right ? b : a;
  const bool go = c1 < n && (cv >> 16) >= (v >> 16);
  if (n != 0) Eb[h] = go ? cv : v;
  h = go ? c1 + (right ? 1 : 0) : h;
  n = go ? n : 0;
}
__device__ inline void vh_pipe_step(uint32_t* Eb, int npops, int& h, int& n, uint32_t v) {
  const int c1 = 2 * h + 1;
  const int ca = min(c1, npops - 1);
  const uint32_t a = Eb[ca], b = Eb[ca + 1];
  vh_pipe_move(Eb, h, n, v, c1, a, b);
}

// __sort_heap on the heap E[lo, hi), one wave, pops pipelined (tools/heap_pipe_model.py checks
// the schedule against libstdc++'s sequential pops).  A __pop_heap (hole to a leaf along the
// larger children, then __push_heap of the tail value v) is the same as a top-down sift of v: the
// larger child moves up while it is not less than v.  Top-down, pops overlap: each in-flight pop
// (one per lane, lanes 0..15 in pop order mod 16) advances one level per round (reads its hole's
// children, writes its hole), so a pop at depth d reads depth d + 1 and writes depth d.  A new pop
// starts when every unfinished older pop is at least two levels deep and none of them can still
// end at the tail position L the new pop takes v from: one whose hole is an ancestor of L (or L)
// ends there only by moving E[L] up, i.e. if E[L] is not less than its v.  A start is considered
// every second round (the two-level spacing makes that the rate anyway): round A reads E[L], the
// root and its children with the holes' children (one LDS latency), decides a start and moves;
// round B moves.  A pop's output (its old root to its tail position) is written by its lane when
// the slot starts its next pop, 2 S >= D + 1 rounds later, when every older pop has finished
// (older pops may read that position as a child), or after the last rounds.  ~2.4 rounds per pop
// and ~100 instructions per two rounds (the start and block tests bitwise: 964 -> 888 cycles a pop,
// profiles/r5_mb_heap_branchfree.txt): the wave is issue-bound (a variant that precomputed both
// next addresses to shorten the dependent chain issued more and ran slower).
__device__ inline void vh_sort_heap_pipe(uint32_t* E, int lo, int hi, int pops) {
  const int lane = threadIdx.x & 63;
  const int len = hi - lo;
  const int npops = len - 1;
  const int todo = min(pops, npops);  // the pops made (the first ones of __sort_heap)
  if (todo < 1) return;
  const int D = 31 - __clz(len);  // depth of the deepest node (<= 14: len <= VH_MAX_N)
  constexpr int S = 16;
  int h = 0, n = 0, L = -1;
  uint32_t v = 0, top = 0;
  uint32_t* const Eb = E + lo;
  const int cr = min(1, npops - 1);  // the root's children, loaded at cr, cr + 1
  int tail = 0;  // pops started (wave-uniform)
  while (tail < todo) {
    // ---- round A
    const int Ln = npops - tail;
    const uint32_t eln = Eb[Ln], e0 = Eb[0], r1 = Eb[cr], r2 = Eb[cr + 1];
    int c1 = 2 * h + 1;
    const int ca = min(c1, npops - 1);
    uint32_t a = Eb[ca], b = Eb[ca + 1];
    const int k = __clz(h + 1) - __clz(Ln + 1);  // depth of Ln minus the hole's
    // (bitwise, not short-circuit: straight-line compares instead of nested exec branches)
    const bool anc = (k >= 0) & (((Ln + 1) >> (k & 31)) == h + 1);
    const bool blocks = (n != 0) & ((h < 3) | (anc & ((eln >> 16) >= (v >> 16))));
    const bool can = __ballot(blocks) == 0ull;
    const bool start = can & (lane == (tail & (S - 1)));
    tail += can ? 1 : 0;
    if (start && L >= 0) Eb[L] = top;  // the slot's previous pop
    v = start ? eln : v;
    top = start ? e0 : top;
    h = start ? 0 : h;
    n = start ? Ln : n;
    L = start ? Ln : L;
    c1 = start ? 1 : c1;
    a = start ? r1 : a;
    b = start ? r2 : b;
    vh_pipe_move(Eb, h, n, v, c1, a, b);
    vh_lds_order();
    // ---- round B
    vh_pipe_step(Eb, npops, h, n, v);
    vh_lds_order();
  }
  for (int r = 0; r < D + 1; ++r) {  // the last pops' sifts
    vh_pipe_step(Eb, npops, h, n, v);
    vh_lds_order();
  }
  if (lane < S && L >= 0) Eb[L] = top;
  vh_lds_order();
}

// (tools/mb_heap.hip, one wave per CU: 1227 -> 958 cycles per element at 1024 elements, 1786 ->
// 1148 with 16 waves per CU; below ~128 elements the look-ahead pops are as fast)
constexpr int VH_PIPE_MIN = 192;
// __make_heap, then the first `pops` pops of __sort_heap (at most hi - lo - 1: all of them)
__device__ inline void vh_heap_sort_wave(uint32_t* E, int lo, int hi, int pops) {
  if (hi - lo < 2) return;
  pops = min(pops, hi - lo - 1);
  vh_make_heap_wave(E, lo, hi);
  if (hi - lo >= VH_PIPE_MIN) {
    ss_wave_fence();
    vh_sort_heap_pipe(E, lo, hi, pops);
  } else {
    vh_sort_heap_wave(E, lo, hi, pops);
  }
}

// The pops a depth-limit heap sort needs: __sort_heap pops in descending key order, so once every
// element with a key not less than kmin (the smallest key two hot members of the segment share)
// is popped, the order among the members of each hot voxel in the segment is final; the elements
// left in the heap all have smaller keys, and their order inside the segment is never read (a hot
// point's position is compared only with its own voxel's members, and those of its voxel outside
// the segment lie outside it).  One wave; the count of E[lo, hi) with key >= kmin.
__device__ inline int vh_pops_needed(const uint32_t* E, int lo, int hi, uint32_t kmin) {
  const int lane = threadIdx.x & 63;
  int c = 0;
  for (int c0 = lo; c0 < hi; c0 += 64) {
    const int i = c0 + lane;
    c += __popcll(__ballot(i < hi && (E[i] >> 16) >= kmin));
  }
  return c;
}

// A depth-limit segment on one wave: heap-sorted literally when two members of one hot voxel lie
// in it (their order is the heap's), else left as it is.  kb: the wave's 64-word key buffer.
__device__ inline void vh_depth_limit_wave(uint32_t* E, int lo, int hi, uint32_t* kb, int* heap_el) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int nh = 0;
  bool dup = false;
  uint32_t kmin = 0;  // the smallest shared hot key (0: not known, every pop)
  for (int c0 = lo; c0 < hi; c0 += 64) {
    const int i = c0 + lane;
    const uint32_t e = i < hi ? E[i] : 0u;
    const bool h = i < hi && (e & VH_HOT);
    const uint64_t b = __ballot(h);
    const int slot = nh + __popcll(b & lt);
    if (h && slot < 64) kb[slot] = e >> 16;
    nh += __popcll(b);
  }
  if (nh < 2) return;
  if (nh > 64) {
    dup = true;  // more than the buffer: assume the order shows
  } else {
    ss_wave_fence();
    const uint32_t mine = lane < nh ? kb[lane] : 0xFFFFFFFFu;
    bool d = false;
    for (int j = 0; j < nh; ++j) d |= lane < nh && j != lane && kb[j] == mine;
    dup = __ballot(d) != 0ull;
    kmin = (uint32_t)wave_min_i(d ? (int)mine : 0x7FFFFFFF);
  }
  if (!dup) return;
  ss_wave_fence();
  const int pops = kmin ? vh_pops_needed(E, lo, hi, kmin) : hi - lo;
  if (lane == 0) atomicAdd(heap_el, pops);
  vh_heap_sort_wave(E, lo, hi, pops);
}

// position of the k-th highest / lowest set bit of m (k >= 1, at least k bits set), per lane
__device__ inline int vh_kth_high(uint64_t m, int k) {
  int t = 0;
#pragma unroll
  for (int s = 32; s; s >>= 1)
    if (__popcll(m >> (t + s)) >= k) t += s;
  return t;
}
__device__ inline int vh_kth_low(uint64_t m, int k) {
  int t = 0;
#pragma unroll
  for (int s = 32; s; s >>= 1)
    if (__popcll(m & ((1ull << (t + s)) - 1ull)) < k) t += s;
  return t;
}

// The whole subtree of a segment of at most 64 elements in one wave's registers (lane i: the
// element at lo + i): every partition is ballots over the segment's lanes, the Hoare pairs
// (l_k, r_k) are found per lane from the stop masks and exchanged with one lane permutation, the
// smaller part goes first; a depth-limit segment goes through the LDS (vh_depth_limit_wave).  The
// same pruning as the LDS partitions: parts with fewer than two hot elements are left.
__device__ inline void vh_subtree64(uint32_t* E, int lo, int len, int d, uint32_t* kb, int* heap_el) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint64_t gt = lane == 63 ? 0ull : (~0ull << (lane + 1));
  const VhLess less;
  uint32_t e = lane < len ? E[lo + lane] : 0u;
  if (__popcll(__ballot(lane < len && (e & VH_HOT))) < 2) return;
  bool dirty = false;
  // pending parts (a | b << 8 | d << 16) as a 3-deep register stack p0 (top), p1, p2: the smaller
  // part goes first, so each pending part is larger than the one worked on and at most 2 wait
  uint32_t p0 = 0, p1 = 0, p2 = 0;
  int top = 0;
  int a = 0, b = len, dd = d;
  while (true) {
    bool next = true;
    const uint64_t rng = (b >= 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((1ull << a) - 1ull);
    if (b - a > SS_THRESHOLD && __popcll(__ballot(e & VH_HOT) & rng) >= 2) {
      if (dd == 0) {
        if (dirty && lane < len) E[lo + lane] = e;
        ss_wave_fence();
        vh_depth_limit_wave(E, lo + a, lo + b, kb, heap_el);
        e = lane < len ? E[lo + lane] : 0u;
        dirty = false;
      } else {
        const int ia = a + 1, ib = a + (b - a) / 2, ic = b - 1;
        const uint32_t ea = __builtin_amdgcn_readlane(e, ia), eb = __builtin_amdgcn_readlane(e, ib),
                       ec = __builtin_amdgcn_readlane(e, ic), ev = __builtin_amdgcn_readlane(e, a);
        int mm;
        if (less(ea, eb)) {
          if (less(eb, ec)) mm = ib;
          else if (less(ea, ec)) mm = ic;
          else mm = ia;
        } else if (less(ea, ec)) {
          mm = ia;
        } else if (less(eb, ec)) {
          mm = ic;
        } else {
          mm = ib;
        }
        const uint32_t em = mm == ia ? ea : (mm == ib ? eb : ec);
        if (lane == a) e = em;
        if (lane == mm) e = ev;
        const uint32_t p = em >> 16, k = e >> 16;
        const bool in = lane > a && lane < b;
        const uint64_t bl = __ballot(in && !(k < p));
        const uint64_t br = __ballot(in && !(p < k)) | (1ull << a);
        const bool isl = (bl >> lane) & 1ull, isr = (br >> lane) & 1ull;
        const int kl = __popcll(bl & lt) + 1;  // ascending rank among the left stops
        const int kr = __popcll(br & gt) + 1;  // descending rank among the right stops
        const int S = __popcll(__ballot(isl && kl <= kr - 1));  // #right stops above l_k >= k
        int partner = lane;
        if (isl && kl <= S) partner = vh_kth_high(br, kl);
        if (isr && kr <= S) partner = vh_kth_low(bl, kr);
        e = __shfl(e, partner, 64);
        const uint64_t bk = __ballot(isl && kl == S + 1), bs = __ballot(isr && kr == S);
        const int lK = bk ? __ffsll((unsigned long long)bk) - 1 : 64;
        const int rS = S >= 1 ? __ffsll((unsigned long long)bs) - 1 : b;
        const int cut = min(lK, rS);
        dirty = true;
        --dd;
        const int l0 = cut - a, l1 = b - cut;
        const bool left_small = l0 <= l1;
        const int sa = left_small ? a : cut, sb = left_small ? cut : b;
        const int ba = left_small ? cut : a, bb = left_small ? b : cut;
        if (bb - ba > SS_THRESHOLD) {
          p2 = p1;
          p1 = p0;
          p0 = (uint32_t)ba | ((uint32_t)bb << 8) | ((uint32_t)dd << 16);
          ++top;
        }
        if (sb - sa > SS_THRESHOLD) {
          a = sa;
          b = sb;
          next = false;
        }
      }
    }
    if (next) {
      if (top == 0) break;
      const uint32_t q = p0;
      p0 = p1;
      p1 = p2;
      --top;
      a = (int)(q & 0xFFu);
      b = (int)((q >> 8) & 0xFFu);
      dd = (int)(q >> 16);
    }
  }
  if (dirty && lane < len) E[lo + lane] = e;
}

// The subtree below one pending segment, one wave, no barriers
__device__ inline void vh_wave_subtree(uint32_t* E, uint16_t* Bs, uint32_t root, uint32_t* wa, int* heap_el,
                                       VhCtl* C, uint32_t* roots, unsigned long long* dp = nullptr) {
  const int lane = threadIdx.x & 63;
  uint32_t* stk = wa;
  uint32_t* kb = wa + VH_LIFO;
  int top = 0;
  uint32_t cur = root;
  while (true) {
    const int lo = (int)(cur & 0x7FFFu), len = (int)((cur >> 15) & 0x7FFu), d = (int)(cur >> 26);
    const int hi = lo + len;
    bool next = true;  // take the next pending entry
    if (len > SS_THRESHOLD && len <= 64) {
      vh_subtree64(E, lo, len, d, kb, heap_el);
      ss_wave_fence();
    } else if (len > SS_THRESHOLD) {
      if (d == 0) {
        const unsigned long long th = __builtin_readcyclecounter();
        vh_depth_limit_wave(E, lo, hi, kb, heap_el);
        if (dp && lane == 0) atomicAdd(dp + 7, __builtin_readcyclecounter() - th);
      } else {
        const int cut = vh_partition_wave(E, Bs, lo, hi, dp);
        if (cut >= 0) {
          const int l0 = cut - lo, l1 = hi - cut;
          const bool left_small = l0 <= l1;
          const int sl = left_small ? lo : cut, sn = left_small ? l0 : l1;  // smaller part: now
          const int bl_ = left_small ? cut : lo, bn = left_small ? l1 : l0;  // larger: pending
          if (sn > SS_THRESHOLD) {  // the smaller part now, the larger one listed or kept
            if (bn > SS_THRESHOLD) {
              int s = VH_ROOTS;
              if (bn > VH_SHARE && lane == 0 &&
                  __hip_atomic_load(&C->nroot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < VH_ROOTS - 64) {
                // listed for any wave: counted pending before it is visible
                s = atomicAdd(&C->nroot, 1);
                if (s < VH_ROOTS) {
                  atomicAdd(&C->pending, 1);
                  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                  __hip_atomic_store(&roots[s], vh_pack(bl_, bn, d - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
              }
              s = __builtin_amdgcn_readfirstlane(s);
              if (s >= VH_ROOTS) {  // kept by this wave
                if (lane == 0 && top < VH_LIFO) stk[top] = vh_pack(bl_, bn, d - 1);
                ++top;  // (overflow impossible: each kept part is larger than the current one)
              }
              ss_wave_fence();
            }
            cur = vh_pack(sl, sn, d - 1);
            next = false;
          } else if (bn > SS_THRESHOLD) {
            // a degenerate partition (the smaller part needs nothing): the chain goes on on this
            // wave, with no round trip through the list or the LIFO
            cur = vh_pack(bl_, bn, d - 1);
            next = false;
          }
        }
      }
    }
    if (next) {
      if (top == 0) break;
      --top;
      cur = __builtin_amdgcn_readfirstlane(stk[min(top, VH_LIFO - 1)]);
    }
  }
}

// Drain the listed wave subtrees (all waves), then reset the list.  Uniform call.  A wave claims
// list entries in order (a ticket); an entry not yet listed is waited for while some listed
// subtree is unfinished (its partitions may list more: the larger part of a partition over
// VH_SHARE elements), so one wave's deep subtree is shared out.  Entries are zero until listed
// and zeroed when taken (the list starts zeroed, vh_sort).
template <int NT>
__device__ inline void vh_drain(const VhLds& L) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* wa = L.wave + wid * VH_WAVE_W;
  VhCtl* C = L.C;
  unsigned long long* dp = C->dprof;
  if (threadIdx.x == 0) C->pending = min(C->nroot, VH_ROOTS);
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  while (true) {
    int k = 0;
    if (lane == 0) k = atomicAdd(&C->root_take, 1);
    k = __builtin_amdgcn_readfirstlane(k);
    uint32_t item = 0;
    for (uint32_t spins = 0;; ++spins) {
      uint32_t it = 0;
      int pend = 0;
      if (lane == 0) {
        pend = __hip_atomic_load(&C->pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        it = k < VH_ROOTS ? __hip_atomic_load(&L.roots[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
      }
      it = __builtin_amdgcn_readfirstlane(it);
      pend = __builtin_amdgcn_readfirstlane(pend);
      if (it) {
        item = it;
        break;
      }
      if (pend == 0) break;
      if (spins >= vh_spin_limit_g) {  // ran out: the entry's subtree may stay unsorted
        if (lane == 0) atomicOr(&C->err, VH_ERR_SPIN);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!item) break;
    if (lane == 0) L.roots[k] = 0u;
    vh_wave_subtree(L.E, L.Bs, item, wa, &C->heap_el, C, L.roots, dp);
    if (lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // its listings before its end
      atomicSub(&C->pending, 1);
    }
    if (dp && lane == 0) atomicAdd(dp + 8, 1ull);
  }
  if (dp && lane == 0) {
    const unsigned long long b = __builtin_readcyclecounter() - t0;
    atomicAdd(dp + 5, b);
    atomicMax(dp + 6, b);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    L.C->nroot = 0;
    L.C->root_take = 0;
  }
  __syncthreads();
}

// Every segment of one workgroup level [lo, hi) (m > VH_BIG; L.bigl[cur], nb of them) partitioned
// at once: segment s owns threads tstart[s] .. tstart[s + 1] - 1, each classifying c consecutive
// positions (a chunk never crosses a segment) into two bit masks; one block scan of the packed
// counts places every stop of every segment (offsets relative to the scan before the segment's
// first thread), so a level costs four barriers whatever its segment count.  Per segment:
// lv.cut[s], or -1 when fewer than two hot elements lie in it.  Uniform; lv.tstart / c, hot = S = 0
// and cut = INT_MAX set by the caller.
template <int NT, int CH>
__device__ inline void vh_partition_level_c(const VhLds& L, int cur, int nb) {
  constexpr int NW = NT / 64;
  static_assert(CH <= 32, "chunk masks in one word");
  static_assert(NW <= VX_WAVES, "scan scratch");
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  uint32_t* E = L.E;
  VhCtl* C = L.C;
  VhLvl& V = C->lv;
  uint32_t* ws = C->ws;
  const VhLess less;
  const int c = V.c;
  // this thread's segment (nb <= 32: binary search over the thread starts)
  int sg = -1;
  if (tid < V.tstart[nb]) {
    int a = 0, b = nb - 1;
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (V.tstart[mid] <= tid) a = mid;
      else b = mid - 1;
    }
    sg = a;
  }
  int lo = 0, hi = 0, r = 0;
  if (sg >= 0) {
    const uint32_t ent = L.bigl[cur * VH_BIGC + sg];
    lo = (int)(ent & 0x7FFFu);
    hi = (int)(ent >> 15);
    r = tid - V.tstart[sg];
  }
  // __move_median_to_first(lo, lo + 1, mid, hi - 1), computed by every thread of the segment: the
  // classification sees the swap (position mm holds E[lo]), the segment's first thread makes it
  // after the scan's barriers
  uint32_t elo = 0, pe = 0;
  int mm = -1;
  if (sg >= 0) {
    elo = E[lo];
    const int a = lo + 1, b = lo + (hi - lo) / 2, cc = hi - 1;
    const uint32_t ea = E[a], eb = E[b], ec = E[cc];
    if (less(ea, eb)) {
      if (less(eb, ec)) mm = b;
      else if (less(ea, ec)) mm = cc;
      else mm = a;
    } else if (less(ea, ec)) {
      mm = a;
    } else if (less(eb, ec)) {
      mm = cc;
    } else {
      mm = b;
    }
    pe = mm == a ? ea : (mm == b ? eb : ec);
  }
  const uint32_t p = pe >> 16;
  const int b0 = lo + 1 + r * c, e0 = min(b0 + c, hi);  // this thread's positions [b0, e0)
  uint32_t ml = 0, mr = 0;
  int nh = 0;
  uint32_t ev[CH];
#pragma unroll
  for (int u = 0; u < CH; ++u) ev[u] = sg >= 0 ? E[min(b0 + u, hi - 1)] : 0u;  // (clamped: every load issued at once)
#pragma unroll
  for (int u = 0; u < CH; ++u) {
    const int i = b0 + u;
    if (i < e0) {
      const uint32_t e = i == mm ? elo : ev[u];
      const uint32_t k = e >> 16;
      if (!(k < p)) ml |= 1u << u;
      if (!(p < k)) mr |= 1u << u;
      nh += (e & VH_HOT) ? 1 : 0;
    }
  }
  // per-segment sums: one atomic per wave when the wave lies in one segment
  auto seg_add = [&](int* arr, int val) {
    const int s0 = __builtin_amdgcn_readfirstlane(sg);
    if (__ballot(sg != s0) == 0ull) {
      const int t = (int)dpp_wave_sum_u((uint32_t)val);
      if (lane == 0 && t && s0 >= 0) atomicAdd(&arr[s0], t);
    } else if (sg >= 0 && val) {
      atomicAdd(&arr[sg], val);
    }
  };
  seg_add(V.hot, nh);
  const uint32_t v = (uint32_t)__popc(ml) | ((uint32_t)__popc(mr) << 16);  // totals < 2^16
  uint32_t x = dpp_incl_scan_u(v);
  if (lane == 63) ws[wid] = x;
  __syncthreads();
  uint32_t all = 0;
  for (int w = 0; w < NW; ++w) {
    x += w < wid ? ws[w] : 0u;  // inclusive over the block
    all += ws[w];
  }
  uint32_t sbase = 0, send = all;  // the scan before the segment's first thread / after its last
  if (nb > 1) {  // (uniform; one segment: the block's own bounds, no barrier)
    if (sg >= 0 && r == 0) V.base[sg] = x - v;
    if (sg >= 0 && tid == V.tstart[sg + 1] - 1) V.endv[sg] = x;
    __syncthreads();
    if (sg >= 0) {
      sbase = V.base[sg];
      send = V.endv[sg];
    }
  }
  const bool act = sg >= 0 && V.hot[sg] + ((pe & VH_HOT) ? 1 : 0) >= 2;
  if (act && r == 0) {  // the median swap (read by nobody before the next barrier)
    E[lo] = pe;
    E[mm] = elo;
  }
  uint16_t* Bs = L.Bs;
  const int m = hi - lo, KB = (m - 1) / 2, bb = lo >> 1;
  const uint32_t off = act ? x - v - sbase : 0u, tot = act ? send - sbase : 0u;
  const int nr = 1 + (int)(tot >> 16);
  int S = 0;
  if (act) {
    int kl = (int)(off & 0xFFFFu), t = 1 + (int)(off >> 16);  // t: ascending right-stop index
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const bool isl = (ml >> u) & 1u, isr = (mr >> u) & 1u;
      if (isl) {
        ++kl;
        S += kl <= nr - (t + (isr ? 1 : 0)) ? 1 : 0;
      }
      if (isr) {
        if (nr - t <= KB) Bs[bb + nr - t - 1] = (uint16_t)(b0 + u);
        ++t;
      }
    }
    if (r == 0 && nr <= KB) Bs[bb + nr - 1] = (uint16_t)lo;
  }
  seg_add(V.S, S);
  __syncthreads();
  if (act) {  // the swaps (each pair read and written by the thread of its left stop alone) and the cut
    const int Sg = V.S[sg];
    int kl = (int)(off & 0xFFFFu);
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if ((ml >> u) & 1u) {
        ++kl;
        if (kl <= Sg) {
          const int y = Bs[bb + kl - 1];
          const uint32_t t = E[y];
          E[y] = E[b0 + u];
          E[b0 + u] = t;
        }
        if (kl == Sg + 1) atomicMin(&V.cut[sg], b0 + u);
      }
    }
    if (r == 0) atomicMin(&V.cut[sg], Sg >= 1 ? (int)Bs[bb + Sg - 1] : hi);
  }
  if (sg >= 0 && r == 0 && !act) V.cut[sg] = -1;
  __syncthreads();
}
template <int NT>
__device__ inline void vh_partition_level(const VhLds& L, int cur, int nb) {
  const int c = L.C->lv.c;  // positions per thread (<= 31: see vh_level_setup)
  if (c <= 2) vh_partition_level_c<NT, 2>(L, cur, nb);
  else if (c <= 4) vh_partition_level_c<NT, 4>(L, cur, nb);
  else if (c <= 8) vh_partition_level_c<NT, 8>(L, cur, nb);
  else if (c <= 16) vh_partition_level_c<NT, 16>(L, cur, nb);
  else vh_partition_level_c<NT, 32>(L, cur, nb);
}

// Thread shares of one level (wave 0; the caller's barrier follows): the least c with
// sum over segments of ceil((m - 1) / c) <= NT (c <= 31 for n <= VH_MAX_N: with at most 30
// segments over 1024, c = 31 gives at most 30720 / 31 + 30 < 1024 threads)
template <int NT>
__device__ inline void vh_level_setup(const VhLds& L, int cur, int nb) {
  const int lane = threadIdx.x & 63;
  VhLvl& V = L.C->lv;
  int len = 0;
  if (lane < nb) {
    const uint32_t ent = L.bigl[cur * VH_BIGC + lane];
    len = (int)(ent >> 15) - (int)(ent & 0x7FFFu) - 1;
  }
  const int tot = (int)dpp_wave_sum_u((uint32_t)len);
  int c = max(1, (tot + NT - 1) / NT);
  int th = 0;
  for (;; ++c) {
    th = lane < nb ? (len + c - 1) / c : 0;
    if ((int)dpp_wave_sum_u((uint32_t)th) <= NT) break;
  }
  const uint32_t incl = dpp_incl_scan_u((uint32_t)th);
  if (lane < nb) {
    V.tstart[lane] = (int)(incl - th);
    V.hot[lane] = 0;
    V.S[lane] = 0;
    V.cut[lane] = 0x7FFFFFFF;
  }
  if (lane == nb - 1) V.tstart[nb] = (int)incl;
  if (lane == 0) V.c = c;
}

// A depth-limit segment of the workgroup: the dup check on a bitmap of slots (in the Bs area,
// free between partitions), then, if two members of one hot voxel lie in it, the literal heap sort
template <int NT>
__device__ inline void vh_depth_limit_wg(const VhLds& L, int n, int lo, int hi) {
  const int tid = threadIdx.x;
  uint32_t* bm = reinterpret_cast<uint32_t*>(L.Bs);
  const int nw = (n >> 5) + 1;  // slot < n
  for (int w = tid; w < nw; w += NT) bm[w] = 0u;
  if (tid == 0) L.C->dup = 0x7FFFFFFF;  // the smallest shared hot key (none)
  __syncthreads();
  int kd = 0x7FFFFFFF;
  for (int i = lo + tid; i < hi; i += NT) {
    const uint32_t e = L.E[i];
    if (e & VH_HOT) {
      const uint32_t s = e >> 16, bit = 1u << (s & 31u);
      if ((atomicOr(&bm[s >> 5], bit) & bit) != 0u) kd = min(kd, (int)s);  // its second member seen
    }
  }
  kd = wave_min_i(kd);
  if (kd != 0x7FFFFFFF && (tid & 63) == 0) atomicMin(&L.C->dup, kd);
  __syncthreads();
  const int kmin = L.C->dup;
  if (kmin != 0x7FFFFFFF && tid < 64) {
    const int pops = vh_pops_needed(L.E, lo, hi, (uint32_t)kmin);
    if (tid == 0) L.C->heap_el += pops;
    vh_heap_sort_wave(L.E, lo, hi, pops);
  }
  __syncthreads();
}

// Phase 2: the pruned emulation over the n points (n <= VH_MAX_N; all NT threads), then
// H.fpos[i] for every hot point i.  *err |= VH_ERR_ROOTS on a list overflow (cannot happen).
// prof (optional, diagnostics): [0] elements heap-sorted literally; [1..4] cycles of the setup, the
// workgroup partitions (and depth-limit segments), the wave subtrees, the positions
// part (vh_sort_big): the n elements are a part of a larger sort, W[0 .. n) (slot << 32 | hot << 31 |
// point), whose depth budget is d0 and whose first position is pos0 (the point ids in E are then
// local: k, with W[k] holding the point)
template <int NT>
__device__ inline int vh_sort(uint32_t* lds, int n, const VxHot& H, int* err, unsigned long long* prof = nullptr,
                               unsigned long long* dprof = nullptr, const uint64_t* part = nullptr, int d0 = -1,
                               uint32_t pos0 = 0) {
  const int tid = threadIdx.x;
  unsigned long long tp = __builtin_readcyclecounter(), t_drain = 0;
  const VhLds L = vh_layout<NT>(lds, n);
  VhCtl* C = L.C;
  for (int i0 = tid; i0 < n; i0 += 8 * NT) {  // 8 loads in flight per thread
    uint32_t r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * NT;
      if (part) {
        const uint64_t w = i < n ? part[i] : 0ull;
        r[u] = ((uint32_t)(w >> 32) << 1) | (uint32_t)((w >> 31) & 1ull);
      } else {
        r[u] = i < n ? H.rk[i] : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * NT;
      if (i < n) L.E[i] = ((r[u] >> 1) << 16) | ((r[u] & 1u) << 15) | (uint32_t)i;
    }
  }
  for (int i = tid; i < VH_ROOTS; i += NT) L.roots[i] = 0u;
  __syncthreads();  // (the entries are zero until listed: tid 0 lists below)
  const int D0 = d0 >= 0 ? d0 : n > 1 ? 2 * (31 - __clz(n)) : 0;  // 2 * __lg(n)
  if (tid == 0) {
    C->nbig[0] = C->nbig[1] = 0;
    C->nroot = C->root_take = 0;
    C->err = 0;
    C->heap_el = 0;
    C->dprof = dprof;
    if (n > SS_THRESHOLD) {
      if (n > VH_BIG) {
        L.bigl[0] = (uint32_t)n << 15;
        C->nbig[0] = 1;
      } else {
        L.roots[0] = vh_pack(0, n, D0);
        C->nroot = 1;
      }
    }
  }
  __syncthreads();
  vx_phase(prof ? prof + 1 : nullptr, 0, &tp);
  for (int lev = 0;; ++lev) {
    const int cur = lev & 1, nxt = cur ^ 1;
    const int nb = min(C->nbig[cur], VH_BIGC);
    if (nb == 0) break;
    const int d = D0 - lev;
    if (d == 0) {
      for (int t = 0; t < nb; ++t) {
        const uint32_t ent = L.bigl[cur * VH_BIGC + t];
        vh_depth_limit_wg<NT>(L, n, (int)(ent & 0x7FFFu), (int)(ent >> 15));
      }
    } else {
      if (tid < 64) vh_level_setup<NT>(L, cur, nb);
      __syncthreads();
      vh_partition_level<NT>(L, cur, nb);
      if (tid < nb) {  // one thread per segment lists its parts
        const uint32_t ent = L.bigl[cur * VH_BIGC + tid];
        const int lo = (int)(ent & 0x7FFFu), hi = (int)(ent >> 15), cut = C->lv.cut[tid];
        if (cut >= 0) {
          const int parts[2][2] = {{lo, cut}, {cut, hi}};
          for (int q = 0; q < 2; ++q) {
            const int a = parts[q][0], b = parts[q][1];
            if (b - a > VH_BIG) {
              const int s = atomicAdd(&C->nbig[nxt], 1);
              if (s < VH_BIGC) L.bigl[nxt * VH_BIGC + s] = (uint32_t)a | ((uint32_t)b << 15);
              else atomicOr(&C->err, VH_ERR_ROOTS);
            } else if (b - a > SS_THRESHOLD) {
              const int s = atomicAdd(&C->nroot, 1);
              if (s < VH_ROOTS) L.roots[s] = vh_pack(a, b - a, d - 1);
              else atomicOr(&C->err, VH_ERR_ROOTS);
            }
          }
        }
      }
    }
    __syncthreads();
    // (nbig[cur] is next read two levels on; nroot is not written before the drain)
    const bool drain = C->nroot > VH_ROOTS - 2 * VH_BIGC;
    if (tid == 0) C->nbig[cur] = 0;
    if (drain) {
      const unsigned long long t0 = __builtin_readcyclecounter();
      vh_drain<NT>(L);
      t_drain += __builtin_readcyclecounter() - t0;
    }
  }
  if (prof && tid == 0) {  // the workgroup levels without the drains inside them
    const unsigned long long now = __builtin_readcyclecounter();
    atomicAdd(prof + 2, now - tp - t_drain);
    atomicAdd(prof + 3, t_drain);
    tp = now;
  }
  vh_drain<NT>(L);
  vx_phase(prof ? prof + 3 : nullptr, 0, &tp);
  if (tid == 0 && C->err) atomicOr(err, C->err);
  const int heap_el = C->heap_el;
  if (tid == 0 && prof) atomicAdd(prof, (unsigned long long)heap_el);
  for (int q = tid; q < n; q += NT) {
    const uint32_t e = L.E[q];
    if (e & VH_HOT) {
      const uint32_t k = e & 0x7FFFu;
      H.fpos[part ? (uint32_t)part[k] & 0x7FFFFFFFu : k] = pos0 + (uint32_t)q;
    }
  }
  __syncthreads();
  vx_phase(prof ? prof + 4 : nullptr, 0, &tp);
  return heap_el;
}

// Sorts of more than VH_MAX_N points (up to VH_BIG_N; the LDS holds only VH_MAX_N): libstdc++'s
// first partition of the whole array runs in global memory (H.w: slot << 32 | hot << 31 | point),
// exactly: __move_median_to_first(first, first + 1, mid, last - 1), then __unguarded_partition with
// the k-th left stop (key not below the pivot, ascending) swapped with the k-th right stop (not
// above, descending) while l_k < r_k, cut = min(l_{S+1}, r_S) (the rank form of the scanning
// loop); each part then runs the LDS emulation with depth budget 2 lg n - 1 (vh_fixup).  Stop
// positions: H.rk (consumed when W is built) and H.fpos (written only after the partition).
// Returns the cut, or -1 when a part is still over VH_MAX_N (the caller then sorts in global
// memory).  All NT threads.
constexpr int VH_BIG_N = 40000;  // hot member lists of vh_centroids fit the LDS (n + 64 words)
template <int NT>
__device__ inline int vh_big_partition(uint32_t* ws, int n, const VxHot& H) {
  const int tid = threadIdx.x;
  uint64_t* W = H.w;
  uint32_t* Lp = H.rk;
  uint32_t* Rp = H.fpos;
  for (int i = tid; i < n; i += NT) {
    const uint32_t r = H.rk[i];
    W[i] = ((uint64_t)(r >> 1) << 32) | ((uint64_t)(r & 1u) << 31) | (uint64_t)i;
  }
  __syncthreads();
  if (tid == 0) {  // the median of positions 1, n / 2, n - 1 to position 0
    const int a = 1, b = n / 2, c = n - 1;
    const uint64_t wa = W[a], wb = W[b], wc = W[c];
    const uint32_t ka = (uint32_t)(wa >> 32), kb = (uint32_t)(wb >> 32), kc = (uint32_t)(wc >> 32);
    int m;
    if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
    else m = ka < kc ? a : (kb < kc ? c : b);
    const uint64_t w0 = W[0], wm = m == a ? wa : (m == b ? wb : wc);
    W[0] = wm;
    W[m] = w0;
  }
  __syncthreads();
  const uint32_t p = (uint32_t)(W[0] >> 32);
  // stops of positions 1 .. n - 1: thread t owns [1 + t C, 1 + (t + 1) C)
  const int C = (n - 1 + NT - 1) / NT;
  const int b0 = 1 + tid * C, b1 = min(n, b0 + C);
  uint32_t cl = 0, cr = 0;
  for (int i = b0; i < b1; ++i) {
    const uint32_t k = (uint32_t)(W[i] >> 32);
    cl += k < p ? 0u : 1u;
    cr += p < k ? 0u : 1u;
  }
  uint32_t totl, totr;
  const uint32_t pl = vx_block_scan_t<NT>(cl, ws, &totl);
  const uint32_t pr = vx_block_scan_t<NT>(cr, ws, &totr);
  {
    uint32_t jl = pl, jr = totr - pr;  // (descending rank of the chunk's last right stop) + 1
    for (int i = b0; i < b1; ++i) {
      const uint32_t k = (uint32_t)(W[i] >> 32);
      if (!(k < p)) Lp[jl++] = (uint32_t)i;
      if (!(p < k)) Rp[--jr] = (uint32_t)i;
    }
  }
  __syncthreads();
  uint32_t sc = 0;  // pairs l_k < r_k (a prefix of k)
  const uint32_t kmax = min(totl, totr);
  for (uint32_t k = tid; k < kmax; k += NT) sc += Lp[k] < Rp[k] ? 1u : 0u;
  uint32_t S;
  (void)vx_block_scan_t<NT>(sc, ws, &S);
  for (uint32_t k = tid; k < S; k += NT) {
    const uint32_t a = Lp[k], b = Rp[k];
    const uint64_t wa = W[a], wb = W[b];
    W[a] = wb;
    W[b] = wa;
  }
  const int cut = (int)min(S < totl ? Lp[S] : (uint32_t)n, S >= 1 ? Rp[S - 1] : (uint32_t)n);
  __syncthreads();
  return (cut > VH_MAX_N || n - cut > VH_MAX_N) ? -1 : cut;
}

// Phase 3: every hot voxel's centroid from its members in position order -> out[slot].  The
// members' (position << 16 | point) go to LDS (lds[0 .. list length)), each voxel's run is
// sorted (one thread up to VH_SMALL members, else one wave by rank), then summed in that order
// from 0 in float (PCL's CentroidPoint), divided by (float)count.  Returns whether some centroid
// left its voxel (then the filter's output is not a VoxelGrid fixed point).  All NT threads;
// M.hot_n / hot_l from phase 1.
template <int NT, typename PF>
__device__ inline bool vh_centroids(const PF& P, float4* out, const VxHot& H, const VxGeom& g, uint32_t* lds,
                                    uint32_t lds_words, VxMisc& M, int* err) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t nh = min(M.hot_n, H.cap_h), nl = M.hot_l;
  uint32_t* Lh = lds;
  uint32_t* big = lds + nl;  // the voxels left to the waves
  if (nl + 64 > lds_words) {  // cannot happen: nl <= n <= VH_BIG_N
    if (tid == 0) atomicOr(err, VH_ERR_LIST);
    return true;
  }
  const uint32_t big_cap = lds_words - nl;
  for (uint32_t j0 = tid; j0 < nl; j0 += 8 * NT) {  // 8 gathers in flight per thread
    uint32_t ii[8], fp[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) ii[u] = j0 + u * NT < nl ? H.hl[j0 + u * NT] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u) fp[u] = j0 + u * NT < nl ? H.fpos[ii[u]] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + u * NT < nl) Lh[j0 + u * NT] = (fp[u] << 16) | ii[u];
  }
  if (tid == 0) {
    M.nbig = 0;
    M.moved = 0;
  }
  __syncthreads();
  bool moved = false;
  auto finish = [&](uint32_t slot, float sx, float sy, float sz, float si, uint32_t n, uint32_t i0) {
    const float fn = (float)n;
    const float4 cc = make_float4(sx / fn, sy / fn, sz / fn, si / fn);
    out[slot] = cc;
    moved |= vx_key(g, cc) != vx_key(g, P(i0));
  };
  for (uint32_t h = tid; h < nh; h += NT) {
    const uint32_t slot = H.hv[3 * h], st = H.hv[3 * h + 1], cnt = H.hv[3 * h + 2];
    if (cnt > (uint32_t)VH_SMALL) {
      const uint32_t e = atomicAdd(&M.nbig, 1u);
      if (e < big_cap) big[e] = h;
      continue;
    }
    for (uint32_t a = 1; a < cnt; ++a) {
      const uint32_t x = Lh[st + a];
      uint32_t b = a;
      while (b > 0 && Lh[st + b - 1] > x) {
        Lh[st + b] = Lh[st + b - 1];
        --b;
      }
      Lh[st + b] = x;
    }
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    for (uint32_t a = 0; a < cnt; a += 4) {
      float4 pp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < cnt) pp[u] = P(Lh[st + a + u] & 0xFFFFu);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a + u < cnt) {
          sx += pp[u].x; sy += pp[u].y; sz += pp[u].z; si += pp[u].w;
        }
    }
    finish(slot, sx, sy, sz, si, cnt, Lh[st] & 0xFFFFu);
  }
  __syncthreads();
  const uint32_t nbig = min(M.nbig, big_cap);
  for (uint32_t q = wid; q < nbig; q += NT / 64) {
    const uint32_t h = big[q];
    const uint32_t slot = H.hv[3 * h], st = H.hv[3 * h + 1], cnt = H.hv[3 * h + 2];
    if (cnt <= 64u * VH_REG) {  // rank sort: positions are distinct
      uint32_t v[VH_REG], r[VH_REG];
#pragma unroll
      for (int u = 0; u < VH_REG; ++u) {
        const uint32_t a = lane + 64u * u;
        v[u] = a < cnt ? Lh[st + a] : 0u;
        r[u] = 0;
      }
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t y = Lh[st + j];
#pragma unroll
        for (int u = 0; u < VH_REG; ++u) r[u] += y < v[u] ? 1u : 0u;
      }
      ss_wave_fence();
#pragma unroll
      for (int u = 0; u < VH_REG; ++u)
        if (lane + 64u * u < cnt) Lh[st + r[u]] = v[u];
      ss_wave_fence();
    } else if (lane == 0) {  // (larger voxels: one lane)
      for (uint32_t a = 1; a < cnt; ++a) {
        const uint32_t x = Lh[st + a];
        uint32_t b = a;
        while (b > 0 && Lh[st + b - 1] > x) {
          Lh[st + b] = Lh[st + b - 1];
          --b;
        }
        Lh[st + b] = x;
      }
    }
    ss_wave_fence();
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;  // every lane keeps the same running sum
    for (uint32_t a = 0; a < cnt; a += 64) {
      float4 pp = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a + lane < cnt) pp = P(Lh[st + a + lane] & 0xFFFFu);
      const uint32_t mm = min(64u, cnt - a);
      for (uint32_t l = 0; l < mm; ++l) {
        sx += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pp.x), (int)l));
        sy += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pp.y), (int)l));
        sz += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pp.z), (int)l));
        si += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pp.w), (int)l));
      }
    }
    if (lane == 0) finish(slot, sx, sy, sz, si, cnt, Lh[st] & 0xFFFFu);
  }
  if (moved) M.moved = 1;
  __syncthreads();
  return M.moved != 0;
}

// After phase 1 (voxel_segment or vx_merge_fixed_point<.., HOT> with S.hot = H, on the n points
// P(0 .. n), n <= VH_MAX_N; output slots relative to out + M.sbase[1]): when a voxel has 3 or more
// members, the pruned emulation and those voxels' centroids.  The stable token phase 1 wrote
// (cold voxels) is cleared when a hot centroid left its voxel.  All NT threads; uniform.
// prof (optional, diagnostics): [0] cycles of the emulated sort, [1] of the hot centroids, [2]
// filters with a hot voxel; sprof: vh_sort's (literal heap elements, setup, workgroup levels,
// wave subtrees, positions).  Returns the elements heap-sorted at the depth limit (0 without a
// hot voxel; diagnostics), or -1 when n > VH_MAX_N and the first partition left a part over
// VH_MAX_N (vh_sort_big: nothing written; the caller sorts in global memory).
template <int NT, typename PF>
__device__ __attribute__((always_inline)) inline int vh_fixup(const PF& P, int n, float4* out, const VxHot& H, uint32_t* lds, uint32_t lds_words,
                                VxMisc& M, uint32_t* stable_out, int* err, unsigned long long* prof = nullptr,
                                unsigned long long* sprof = nullptr, unsigned long long* dprof = nullptr) {
  __syncthreads();
  if (M.hot_n == 0) return 0;
  const VxGeom g = M.g;
  float4* o = out + M.sbase[1];
  const unsigned long long t0 = __builtin_readcyclecounter();
  int heap_el = 0;
  // the whole sort, or (more than VH_MAX_N points: callers pass at most VH_BIG_N, with H.w) the two
  // parts of its first partition; one call site of vh_sort (inlined)
  int nparts = 1, cut = n, d0 = -1;
  const uint64_t* W = nullptr;
  if (n > VH_MAX_N) {
    cut = vh_big_partition<NT>(lds, n, H);
    if (cut < 0) return -1;
    nparts = 2;
    W = H.w;
    d0 = 2 * (31 - __clz(n)) - 1;
  }
  for (int q = 0; q < nparts; ++q) {
    const int lo = q ? cut : 0, len = q ? n - cut : cut;
    bool run = true;
    if (W) {  // a part of at most 16 elements, or with fewer than two hot ones, keeps its positions
      uint32_t nh = 0;
      for (int i = threadIdx.x; i < len; i += NT) nh += (uint32_t)(W[lo + i] >> 31) & 1u;
      uint32_t tot;
      (void)vx_block_scan_t<NT>(nh, lds, &tot);
      run = len > SS_THRESHOLD && tot >= 2;
      if (!run) {
        for (int i = threadIdx.x; i < len; i += NT) {
          const uint64_t w = W[lo + i];
          if ((w >> 31) & 1ull) H.fpos[(uint32_t)w & 0x7FFFFFFFu] = (uint32_t)(lo + i);
        }
        __syncthreads();
      }
    }
    if (run) heap_el += vh_sort<NT>(lds, len, H, err, sprof, dprof, W ? W + lo : nullptr, d0, (uint32_t)lo);
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  const bool mv = vh_centroids<NT>(P, o, H, g, lds, lds_words, M, err);
  if (mv && threadIdx.x == 0 && stable_out) *stable_out = 0u;
  if (prof && threadIdx.x == 0) {
    atomicAdd(prof, t1 - t0);
    atomicAdd(prof + 1, __builtin_readcyclecounter() - t1);
    atomicAdd(prof + 2, 1ull);
  }
  __syncthreads();
  return heap_el;
}

}  // namespace loam
