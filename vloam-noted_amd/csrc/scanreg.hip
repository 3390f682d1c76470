// scanreg.hip — ScanRegistration::input (scan_registration.cpp:144-513) on MI355X.
//
// Kernels (one frame per call; all buffers HBM-resident, outputs stay on the device for the
// odometry / mapping stages):
//   k_sr_valid      NaN + minimum-range filter (:168-176, :107-141); first/last valid index
//                   -> startOri / endOri (:185-197)
//   k_sr_ring       elevation -> scanID (:217-259), azimuth branch-1 test; the halfPassed
//                   latch (:265-292) = first ring-valid point whose branch-1 azimuth passes
//                   startOri + pi (atomicMin); per-block ring histograms
//   k_sr_ring_scan  exclusive scan of the (ring, block) histogram -> stable counting sort
//                   offsets = laserCloudScans concatenation (:308-315)
//   k_sr_scatter    stable scatter into the ring-major cloud, intensity = scanID + 0.1*relTime
//   k_sr_curv       11-tap curvature over the concatenated cloud (:323-346), crossing rings
//   k_sr_ring_features  one workgroup per ring, two phases in one 160 KiB LDS:
//                   selection: the 6 sectors sorted by curvature at once (one wave per sector,
//                   register bitonic), then the greedy sharp / lessSharp / flat picks with +-5
//                   neighbour suppression (:352-493), one wave per sector with 64-wide ballots,
//                   sectors concurrently and a rerun where a border's inherited flags matter;
//                   then VoxelGrid 0.2 m of the ring's lessFlat candidates (:497-503), in PCL's
//                   summation order (voxel.h + voxel_hot.h: std::sort's order only where a
//                   voxel has 3+ members)
//   k_sr_gather     concatenation of the per-ring outputs in ring order
// The reference sorts each sector with std::sort (unstable).  The bitonic sort by (curvature,
// index) is std::sort's order whenever a sector's curvatures are distinct; a sector with a tie
// is re-sorted by the exact libstdc++ permutation (stdsort.h) before the picks.  Azimuths and
// elevations use glibc's atan2f / atanf restated (libm_f32.h), so ring ids and intensity carry
// the reference's bits.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "libm_f32.h"
#include "stdsort.h"
#include "voxel.h"
#include "voxel_hot.h"

namespace loam {

constexpr int SR_MAX_RINGS = 64;
constexpr int SR_BLOCK = 256;
constexpr int SR_RING_CAP = 16384;  // points per ring handled in LDS
constexpr int SR_SECT_CAP = 4096;   // points per sector (bitonic in LDS)
constexpr int SR_SHARP = 2, SR_LESS_SHARP = 20, SR_FLAT = 4;
constexpr int SR_ERR_RING = 1, SR_ERR_VOXEL = 2, SR_ERR_SORT = 4;

struct SrFrame {
  int n_in;
  int first, last;  // first / last valid raw index
  int latch;        // raw index of the halfPassed latch (INT_MAX: never)
  float start_ori, end_ori;
  int n_cloud;
  int ring_off[SR_MAX_RINGS + 1];
  int ring_cnt[SR_MAX_RINGS];
  int n_sharp[SR_MAX_RINGS], n_less_sharp[SR_MAX_RINGS], n_flat[SR_MAX_RINGS];
  int n_less_flat_scan[SR_MAX_RINGS];
  uint32_t n_less_flat[SR_MAX_RINGS];
  int out_n[5];
  int err;
};

struct SrDev {
  int cap;  // max input points
  int n_in;  // this frame's input points (k_sr_init)
  int n_scans;
  float min_range;
  int stride;
  const float* xyz;      // raw input (stride floats per point)
  SrFrame* fr;
  int* ring_of;          // [cap] scanID per raw point (-1 dropped)
  int* blk_hist;         // [SR_MAX_RINGS][nblocks]
  int* blk_off;          // [SR_MAX_RINGS][nblocks]
  int* blk_aux;          // [3][nblocks]: per block first / last valid index, first latch index
  float4* cloud;         // [cap] laserCloud
  float* curv;           // [cap]
  int* sort_ind;         // [cap] debug: label per point
  int* label;            // [cap]
  int* ring_sharp;       // [SR_MAX_RINGS][6*SR_SHARP] cloud indices
  int* ring_less_sharp;  // [SR_MAX_RINGS][6*SR_LESS_SHARP]
  int* ring_flat;        // [SR_MAX_RINGS][6*SR_FLAT]
  float4* less_flat_scan;  // [cap] ring-local regions
  float4* less_flat_ds;    // [cap]
  float4* vx_pts;
  int* vx_idx;
  float4* out[5];        // laserCloud alias, sharp, lessSharp, flat, lessFlat
  // std::sort emulation scratch for sectors / rings too long for LDS, indexed by cloud position
  uint64_t* ss_e;
  uint32_t* ss_a;
  uint32_t* ss_b;
  uint64_t* ss_s;
  int* ss_seg;  // [ring][2][3 * SR_SS_GSEG] level lists of the long-sector path (one sector of a ring at a time;
               // every ring's workgroup has its own area: the rings run concurrently)
  unsigned long long* dbg;  // [LOAM_SR_DEBUG_COUNTERS] (loam_scanreg_debug_counters)
  unsigned long long* pdbg;  // dbg when LOAM_PHASE_COUNTERS=1 at create, else null (no cycle counting)
};

// scan_registration.cpp:217-259 (float atan/sqrt like the reference's float overloads)
__device__ inline int sr_scan_id(float x, float y, float z, int n_scans) {
  // float atan(float) * 180 -> float, / M_PI -> double, stored as float
  const float angle = (float)((double)(glibc_atanf(z / sqrtf(x * x + y * y)) * 180) / M_PI);
  int scanID = 0;
  if (n_scans == 16) {
    scanID = int((angle + 15) / 2 + 0.5);
    if (scanID > (n_scans - 1) || scanID < 0) return -1;
  } else if (n_scans == 32) {
    scanID = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
    if (scanID > (n_scans - 1) || scanID < 0) return -1;
  } else {
    if (angle >= -8.83) scanID = int((2 - angle) * 3.0 + 0.5);
    else scanID = n_scans / 2 + int((-8.83 - angle) * 2.0 + 0.5);
    if (angle > 2 || angle < -24.33 || scanID > 50 || scanID < 0) return -1;
  }
  return scanID;
}

// the frame record's initial state, written on the device (a pageable host-to-device copy of it
// cost the stream a staging round trip per frame)
__global__ void __launch_bounds__(256) k_sr_init(const SrDev* __restrict__ Ds) {
  SrFrame* F = Ds[blockIdx.y].fr;
  const int n_in = Ds[blockIdx.y].n_in;
  uint32_t* w = reinterpret_cast<uint32_t*>(F);
  for (int k = threadIdx.x; k < (int)(sizeof(SrFrame) / 4); k += 256) w[k] = 0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    F->n_in = n_in;
    F->first = 0x7FFFFFFF;
    F->last = -1;
    F->latch = 0x7FFFFFFF;
  }
}

// one point per thread; every block leaves its first / last valid index in blk_aux (one
// contended device-scope atomic per block or wave cost ~100 us per frame)
__global__ void __launch_bounds__(SR_BLOCK) k_sr_valid(const SrDev* __restrict__ Ds, int nblocks) {
  const SrDev D = Ds[blockIdx.y];  // this launch's frame y (loam_scanreg_input_batch)
  __shared__ int wf[SR_BLOCK / 64], wl[SR_BLOCK / 64];
  SrFrame& F = *D.fr;
  const float thr2 = D.min_range * D.min_range;
  const int i = blockIdx.x * SR_BLOCK + threadIdx.x, w = threadIdx.x >> 6;
  bool ok = false;
  if (i < F.n_in) {
    const float x = D.xyz[(size_t)i * D.stride], y = D.xyz[(size_t)i * D.stride + 1],
                z = D.xyz[(size_t)i * D.stride + 2];
    ok = isfinite(x) && isfinite(y) && isfinite(z) && !(x * x + y * y + z * z < thr2);
    D.ring_of[i] = ok ? 0 : -2;  // -2: removed before the ring rule
  }
  const uint64_t b = __ballot(ok);
  const int i0 = i - (threadIdx.x & 63);
  if ((threadIdx.x & 63) == 0) {
    wf[w] = b ? i0 + __ffsll((unsigned long long)b) - 1 : 0x7FFFFFFF;
    wl[w] = b ? i0 + 63 - __clzll((unsigned long long)b) : -1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int f = 0x7FFFFFFF, l = -1;
    for (int k = 0; k < SR_BLOCK / 64; ++k) {
      f = min(f, wf[k]);
      l = max(l, wl[k]);
    }
    D.blk_aux[blockIdx.x] = f;
    D.blk_aux[nblocks + blockIdx.x] = l;
  }
}

__device__ inline float sr_ori_branch1(float ori, float startOri) {
  if (ori < startOri - M_PI / 2) ori += 2 * M_PI;
  else if (ori > startOri + M_PI * 3 / 2) ori -= 2 * M_PI;
  return ori;
}

// per raw point: ring (or -1), branch-1 latch test; per-block ring histogram
__global__ void __launch_bounds__(SR_BLOCK) k_sr_ring(const SrDev* __restrict__ Ds, int nblocks) {
  const SrDev D = Ds[blockIdx.y];  // this launch's frame y (loam_scanreg_input_batch)
  __shared__ int hist[SR_MAX_RINGS];
  SrFrame& F = *D.fr;
  for (int r = threadIdx.x; r < SR_MAX_RINGS; r += SR_BLOCK) hist[r] = 0;
  __syncthreads();
  const int i = blockIdx.x * SR_BLOCK + threadIdx.x;
  bool past = false;  // past the halfPassed latch candidate
  if (i < F.n_in && D.ring_of[i] == 0) {
    const float x = D.xyz[(size_t)i * D.stride], y = D.xyz[(size_t)i * D.stride + 1],
                z = D.xyz[(size_t)i * D.stride + 2];
    const int sid = sr_scan_id(x, y, z, D.n_scans);
    D.ring_of[i] = sid;
    if (sid >= 0) {
      atomicAdd(&hist[sid], 1);
      const float ori = sr_ori_branch1(-glibc_atan2f(y, x), F.start_ori);
      past = ori - F.start_ori > M_PI;
    }
  }
  // the latch is the lowest such index: per block (lanes hold consecutive indices), reduced
  // over the blocks in k_sr_ring_scan
  __shared__ int wlat[SR_BLOCK / 64];
  const uint64_t pb = __ballot(past);
  if ((threadIdx.x & 63) == 0)
    wlat[threadIdx.x >> 6] = pb ? i - (threadIdx.x & 63) + __ffsll((unsigned long long)pb) - 1 : 0x7FFFFFFF;
  __syncthreads();
  if (threadIdx.x == 0) {
    int lt = 0x7FFFFFFF;
    for (int k = 0; k < SR_BLOCK / 64; ++k) lt = min(lt, wlat[k]);
    D.blk_aux[2 * nblocks + blockIdx.x] = lt;
  }
  for (int r = threadIdx.x; r < SR_MAX_RINGS; r += SR_BLOCK) D.blk_hist[r * nblocks + blockIdx.x] = hist[r];
}

__global__ void __launch_bounds__(1024) k_sr_oris(const SrDev* __restrict__ Ds, int nblocks) {
  const SrDev D = Ds[blockIdx.y];  // this launch's frame y (loam_scanreg_input_batch)
  __shared__ int wf[16], wl[16];
  SrFrame& F = *D.fr;
  int f = 0x7FFFFFFF, l = -1;
  for (int k = threadIdx.x; k < nblocks; k += 1024) {
    f = min(f, D.blk_aux[k]);
    l = max(l, D.blk_aux[nblocks + k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    f = min(f, __shfl_xor(f, o, 64));
    l = max(l, __shfl_xor(l, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    wf[threadIdx.x >> 6] = f;
    wl[threadIdx.x >> 6] = l;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int k = 0; k < 16; ++k) {
    f = min(f, wf[k]);
    l = max(l, wl[k]);
  }
  F.first = f;
  F.last = l;
  // startOri / endOri (scan_registration.cpp:185-197)
  if (F.first > F.last) return;
  const float* p0 = D.xyz + (size_t)F.first * D.stride;
  const float* p1 = D.xyz + (size_t)F.last * D.stride;
  float startOri = -glibc_atan2f(p0[1], p0[0]);
  float endOri = (float)(-glibc_atan2f(p1[1], p1[0]) + 2 * M_PI);
  if (endOri - startOri > 3 * M_PI) endOri = (float)(endOri - 2 * M_PI);
  else if (endOri - startOri < M_PI) endOri = (float)(endOri + 2 * M_PI);
  F.start_ori = startOri;
  F.end_ori = endOri;
}

// exclusive scan of blk_hist in ring-major order (one 1024-thread workgroup)
__global__ void __launch_bounds__(1024) k_sr_ring_scan(const SrDev* __restrict__ Ds, int nblocks) {
  const SrDev D = Ds[blockIdx.y];  // this launch's frame y (loam_scanreg_input_batch)
  __shared__ uint32_t ws[VX_WAVES + 1];
  __shared__ int ring_tot[SR_MAX_RINGS];
  __shared__ int wl[16];
  SrFrame& F = *D.fr;
  const int total = SR_MAX_RINGS * nblocks;
  {  // the halfPassed latch: the lowest of the blocks' first indices past startOri + pi
    int lt = 0x7FFFFFFF;
    for (int k = threadIdx.x; k < nblocks; k += 1024) lt = min(lt, D.blk_aux[2 * nblocks + k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lt = min(lt, __shfl_xor(lt, o, 64));
    if ((threadIdx.x & 63) == 0) wl[threadIdx.x >> 6] = lt;
    __syncthreads();
    if (threadIdx.x == 0) {  // one plain store (this workgroup is the only writer): 16 contended
      for (int k = 0; k < 16; ++k) lt = min(lt, wl[k]);  // device atomics cost ~7 us
      F.latch = lt;
    }
  }
  // exclusive scan of the flattened [ring][block] histogram: thread t holds RS_PER consecutive
  // entries in registers (all its loads in flight at once: the pass is one memory latency, not
  // one per 64-entry step), one block scan of the thread sums, then the thread writes its
  // prefixes; a ring starts at the prefix of its block 0
  constexpr int RS_PER = 32;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t carry = 0;
  for (int r0 = 0; r0 < total; r0 += 1024 * RS_PER) {
    const int e0 = r0 + threadIdx.x * RS_PER;
    uint32_t v[RS_PER];
    if (e0 + RS_PER <= total) {
      const int4* src = reinterpret_cast<const int4*>(D.blk_hist + e0);  // e0 % 4 == 0: 16-byte aligned
#pragma unroll
      for (int j = 0; j < RS_PER / 4; ++j) {
        const int4 q = src[j];
        v[4 * j] = (uint32_t)q.x;
        v[4 * j + 1] = (uint32_t)q.y;
        v[4 * j + 2] = (uint32_t)q.z;
        v[4 * j + 3] = (uint32_t)q.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < RS_PER; ++j) v[j] = e0 + j < total ? (uint32_t)D.blk_hist[e0 + j] : 0u;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < RS_PER; ++j) sum += v[j];
    const uint32_t inc = wave_incl_scan_u(sum);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    uint32_t pre = carry + inc - sum, tot_r = 0;
    for (int k = 0; k < 16; ++k) {
      const uint32_t w = ws[k];
      pre += k < wid ? w : 0u;
      tot_r += w;
    }
    if (e0 < total) {
      int nxt = ((e0 + nblocks - 1) / nblocks) * nblocks;  // the first ring start at or after e0
      uint32_t o[RS_PER];
#pragma unroll
      for (int j = 0; j < RS_PER; ++j) {
        o[j] = pre;
        if (e0 + j == nxt) {
          ring_tot[nxt / nblocks] = (int)pre;
          nxt += nblocks;
        }
        pre += v[j];
      }
      if (e0 + RS_PER <= total) {
        int4* dst = reinterpret_cast<int4*>(D.blk_off + e0);
#pragma unroll
        for (int j = 0; j < RS_PER / 4; ++j)
          dst[j] = make_int4((int)o[4 * j], (int)o[4 * j + 1], (int)o[4 * j + 2], (int)o[4 * j + 3]);
      } else {
#pragma unroll
        for (int j = 0; j < RS_PER; ++j)
          if (e0 + j < total) D.blk_off[e0 + j] = (int)o[j];
      }
    }
    carry += tot_r;
    __syncthreads();  // ws is rewritten by the next round
  }
  const uint32_t tot = carry;
  __syncthreads();
  if (threadIdx.x <= SR_MAX_RINGS) {
    const int r = threadIdx.x;
    const int start = r < SR_MAX_RINGS ? ring_tot[r] : (int)tot;
    F.ring_off[r] = start;
    if (r < SR_MAX_RINGS) F.ring_cnt[r] = (r + 1 < SR_MAX_RINGS ? ring_tot[r + 1] : (int)tot) - start;
    if (r == SR_MAX_RINGS) F.n_cloud = (int)tot;
  }
}

// stable scatter: rank within the block by wave peeling, intensity = scanID + 0.1 * relTime
__global__ void __launch_bounds__(SR_BLOCK) k_sr_scatter(const SrDev* __restrict__ Ds, int nblocks) {
  const SrDev D = Ds[blockIdx.y];  // this launch's frame y (loam_scanreg_input_batch)
  __shared__ int wcnt[SR_BLOCK / 64][SR_MAX_RINGS];
  const SrFrame& F = *D.fr;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  for (int k = tid; k < (SR_BLOCK / 64) * SR_MAX_RINGS; k += SR_BLOCK) (&wcnt[0][0])[k] = 0;
  __syncthreads();
  const int i = blockIdx.x * SR_BLOCK + tid;
  const int sid = (i < F.n_in) ? D.ring_of[i] : -1;
  // wave-local stable rank among equal rings
  uint64_t active = __ballot(sid >= 0);
  int rank = 0;
  while (active) {
    const int leader = __ffsll((long long)active) - 1;
    const int r = __shfl(sid, leader, 64);
    const uint64_t mask = __ballot(sid == r);
    if (sid == r) rank = __popcll(mask & lanemask_lt());
    if (lane == leader) wcnt[wid][r] = __popcll(mask);
    active &= ~mask;
  }
  __syncthreads();
  if (sid < 0) return;
  int before = 0;
  for (int w = 0; w < wid; ++w) before += wcnt[w][sid];
  const int pos = D.blk_off[sid * nblocks + blockIdx.x] + before + rank;
  const float x = D.xyz[(size_t)i * D.stride], y = D.xyz[(size_t)i * D.stride + 1],
              z = D.xyz[(size_t)i * D.stride + 2];
  float ori = -glibc_atan2f(y, x);
  const float startOri = F.start_ori, endOri = F.end_ori;
  if (i <= F.latch) {
    ori = sr_ori_branch1(ori, startOri);
  } else {
    ori = (float)(ori + 2 * M_PI);
    if (ori < endOri - M_PI * 3 / 2) ori = (float)(ori + 2 * M_PI);
    else if (ori > endOri + M_PI / 2) ori = (float)(ori - 2 * M_PI);
  }
  const float relTime = (ori - startOri) / (endOri - startOri);
  const float intensity = (float)(sid + 0.1 * relTime);
  D.cloud[pos] = make_float4(x, y, z, intensity);
}

__global__ void k_sr_curv(const SrDev* __restrict__ Ds) {
  const SrDev D = Ds[blockIdx.y];
  const SrFrame& F = *D.fr;
  const int n = F.n_cloud;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    D.label[i] = 0;
    if (i < 5 || i >= n - 5) {
      D.curv[i] = 0.f;
      continue;
    }
    const float4* L = D.cloud;
    float dx = L[i - 5].x + L[i - 4].x + L[i - 3].x + L[i - 2].x + L[i - 1].x - 10 * L[i].x +
               L[i + 1].x + L[i + 2].x + L[i + 3].x + L[i + 4].x + L[i + 5].x;
    float dy = L[i - 5].y + L[i - 4].y + L[i - 3].y + L[i - 2].y + L[i - 1].y - 10 * L[i].y +
               L[i + 1].y + L[i + 2].y + L[i + 3].y + L[i + 4].y + L[i + 5].y;
    float dz = L[i - 5].z + L[i - 4].z + L[i - 3].z + L[i - 2].z + L[i - 1].z - 10 * L[i].z +
               L[i + 1].z + L[i + 2].z + L[i + 3].z + L[i + 4].z + L[i + 5].z;
    D.curv[i] = dx * dx + dy * dy + dz * dz;
  }
}

// +-5 neighbour suppression while consecutive squared gaps stay <= 0.05 (:406-429)
// +-5 neighbour suppression of a pick (scan_registration.cpp:402-429): the reference walks
// outwards while consecutive points are within sqrt(0.05); gapok[k] holds that test for the
// pair (k, k + 1) of the ring (ring-local indices), precomputed in parallel.
// The reference's neighbour suppression after a pick at ring position i (:389-404): up to 5
// points on each side are marked picked, each side stopping at the first squared gap > 0.05
// (gapok[k]: the gap k -> k+1 is not).  nf / nb: the chain lengths ahead and behind (0..5).
__device__ inline void sr_chain(const uint8_t* gapok, int i, int& nf, int& nb) {
  uint32_t f = 0, b = 0;
#pragma unroll
  for (int l = 0; l < 5; ++l) {
    f |= (uint32_t)(gapok[i + l] != 0) << l;
    b |= (uint32_t)(gapok[i - 1 - l] != 0) << l;
  }
  nf = __builtin_ctz((~f & 31u) | 32u);
  nb = __builtin_ctz((~b & 31u) | 32u);
}

// One wave sorts one sector in registers: E * 64 keys (curvature bits << 32 | index), bitonic,
// partners within a lane's registers swapped directly and partners in other lanes by
// shuffles (no barriers); padding keys are ~0 and end last.
template <int E>
__device__ inline void sr_wave_sort(const float* curv, int sp, int len, uint64_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = e * 64 + lane;
    v[e] = i < len ? (((uint64_t)__float_as_uint(curv[sp + i]) << 32) | (uint32_t)(sp + i)) : ~0ull;
  }
#pragma unroll
  for (int k = 2; k <= E * 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int ej = j >> 6;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int f = e ^ ej;
          if (f > e) {
            const int i = e * 64 + lane;
            const uint64_t a = v[e], b = v[f];
            const bool asc = (i & k) == 0;
            v[e] = asc ? (a < b ? a : b) : (a < b ? b : a);
            v[f] = asc ? (a < b ? b : a) : (a < b ? a : b);
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = e * 64 + lane;
          const uint64_t p = __shfl_xor(v[e], j, 64);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) out[e * 64 + lane] = v[e];
}

constexpr int SR_WSORT_MAX = 1024;  // register sort (one wave per sector) up to this length
constexpr int SR_SS_LDS = 512;      // tied sectors re-sorted in LDS up to this length (else global)
constexpr int SR_SS_SEG = SR_WSORT_MAX / 17 + 2;  // level list of one wave-sorted sector
constexpr int SR_SS_GSEG = 6 * SR_WSORT_MAX / 17 + 2;  // long sectors: global level lists

struct SrCurvLess {  // the reference's comparator: cloudCurvature[i] < cloudCurvature[j]
  static constexpr int free_run = 1;  // tied curvatures: the order picks the features
  __device__ bool operator()(uint64_t a, uint64_t b) const {
    return __uint_as_float((uint32_t)(a >> 32)) < __uint_as_float((uint32_t)(b >> 32));
  }
};

// K[0, len): one sector's keys (curvature bits << 32 | cloud index) sorted by (curvature,
// index).  If two curvatures are equal, std::sort's order differs from that one: the wave
// recomputes the exact libstdc++ permutation of the sector (cloudSortInd[sp..ep] starts as
// the identity, :341) into K.  One wave; E/A/B in LDS for short sectors, else the global
// scratch at the sector's cloud positions.
__device__ inline void sr_exact_sector(const SrDev& D, int sp, int len, uint64_t* K, uint64_t* lE, uint32_t* lA,
                                       uint32_t* lB, SsLevels* lev, int* seg0, int* seg1, int cap) {
  const int lane = threadIdx.x & 63;
  ss_wave_fence();
  bool tie = false;
  for (int k = lane; k + 1 < len; k += 64) tie |= (uint32_t)(K[k] >> 32) == (uint32_t)(K[k + 1] >> 32);
  if (!__ballot(tie)) return;
  const bool lds = len <= SR_SS_LDS;
  uint64_t* E = lds ? lE : D.ss_e + sp;
  uint32_t* A = lds ? lA : D.ss_a + sp;
  uint32_t* B = lds ? lB : D.ss_b + sp;
  for (int k = lane; k < len; k += 64)
    E[k] = ((uint64_t)__float_as_uint(D.curv[sp + k]) << 32) | (uint32_t)(sp + k);
  if (lane == 0) ss_levels_init(lev, len, seg0, seg1, cap);
  const SrCurvLess less;
  ss_levels<false>(E, A, B, lev, 0, 1, less, seg0, seg1, nullptr);
  ss_final(E, A, B, len, K, lane, 64, less);
  if (lane == 0 && lev->err) atomicOr(&D.fr->err, SR_ERR_SORT);
  ss_wave_fence();
}

// One sector's picks (LDS), in pick order, and what the sector's run leaves at its borders.
struct SrSect {
  int sh[SR_SHARP], ls[SR_LESS_SHARP], fl[SR_FLAT];
  int nsh, nls, nfl;
  uint32_t spill;  // (concurrent runs) suppression past the sector's end: bit b = ring index hi + 1 + b
  uint32_t head;   // picks among the sector's first 5 points: bit b = ring index lo + b
};

// sharp / lessSharp (descending curvature, :371-431) and flat (ascending, :439-483) picks of
// one sector [lo, hi] (ring-local) from its sorted keys K[0, len): one wave.  A window of 64
// sorted candidates is loaded with its picked flags and each candidate's suppression chains
// (sr_chain); a pick then costs no LDS read: the candidates its suppression covers (cloud index
// within the chains) drop out of the window's mask by one ballot, and picked[] is written for
// the later windows.  The reference's next candidate is the first unpicked one behind the pick.
// conc (the sectors of a ring run concurrently, sr_greedy_ring): picked[] is written only inside
// [lo, hi]; suppression past hi goes to `spill` instead, suppression before lo is dropped (the
// sectors before are done with their picks in the reference's order, and lessFlat reads labels,
// not picked flags).
template <bool SHARP>
__device__ inline void sr_greedy_pass(int base, int lo, int hi, bool conc, const uint64_t* K, int len,
                                      uint8_t* picked, int8_t* lab, const uint8_t* gapok, SrSect& S, int& nsh,
                                      int& nls, int& nfl, uint32_t& spill, uint32_t& head) {
  const int lane = threadIdx.x & 63;
  int count = 0;
  for (int w = 0; w < len; w += 64) {
    const int k = SHARP ? len - 1 - w - lane : w + lane;
    bool cand = false;
    int ind = base, nf = 0, nb = 0;
    if (k >= 0 && k < len) {
      const uint64_t key = K[k];
      ind = (int)(key & 0xFFFFFFFFu);
      const double c = (double)__uint_as_float((uint32_t)(key >> 32));
      // the reference compares the float curvature with the double literal 0.1 (:381, :443): a
      // curvature of exactly 0.1f (> 0.1) is an edge candidate
      cand = SHARP ? c > 0.1 : c < 0.1;
    }
    // every curvature after the first non-candidate fails the test too (sorted order)
    const uint64_t bx = __ballot(k >= 0 && k < len && !cand);
    const int fx = bx ? __ffsll((long long)bx) - 1 : 64;
    bool avl = cand && lane < fx && picked[ind - base] == 0;
    if (avl) sr_chain(gapok, ind - base, nf, nb);
    uint64_t avail = __ballot(avl);
    while (avail) {
      const int fc = __ffsll((long long)avail) - 1;
      const int pind = __builtin_amdgcn_readlane(ind, fc) - base;
      const int pf = __builtin_amdgcn_readlane(nf, fc), pb = __builtin_amdgcn_readlane(nb, fc);
      count++;
      if (SHARP && count > SR_LESS_SHARP) return;
      if (pind - lo < 5) head |= 1u << (pind - lo);  // (the 4th flat pick too: it is a pick)
      if (SHARP) {
        if (lane == 0) {
          if (count <= SR_SHARP) {
            lab[pind] = 2;
            S.sh[nsh] = pind + base;
          } else {
            lab[pind] = 1;
          }
          S.ls[nls] = pind + base;
        }
        nsh += count <= SR_SHARP;
        nls++;
      } else {
        if (lane == 0) {
          lab[pind] = -1;
          S.fl[nfl] = pind + base;
        }
        nfl++;
        if (count >= SR_FLAT) return;
      }
      if (lane == 0) picked[pind] = 1;
      const int q = lane < pf ? pind + 1 + lane : (lane >= 5 && lane - 5 < pb) ? pind - (lane - 4) : -1;
      if (q >= 0 && (!conc || (q >= lo && q <= hi))) picked[q] = 1;
      if (conc && pind + pf > hi)
        for (int l = hi + 1 - pind; l <= pf; ++l) spill |= 1u << (pind + l - hi - 1);
      const int rel = ind - base;
      avail &= ~__ballot(rel >= pind - pb && rel <= pind + pf);  // the pick and its suppressed neighbours
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the window's writes before the next reads
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (fx < 64) return;
  }
}

// one sector's two passes (sharp first, :371-431, then flat, :439-483) on one wave; the counts,
// spill and head go to S
__device__ inline void sr_greedy_sector(int base, int lo, int hi, bool conc, const uint64_t* K, int len,
                                        uint8_t* picked, int8_t* lab, const uint8_t* gapok, SrSect& S) {
  int nsh = 0, nls = 0, nfl = 0;
  uint32_t spill = 0, head = 0;
  sr_greedy_pass<true>(base, lo, hi, conc, K, len, picked, lab, gapok, S, nsh, nls, nfl, spill, head);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  sr_greedy_pass<false>(base, lo, hi, conc, K, len, picked, lab, gapok, S, nsh, nls, nfl, spill, head);
  if ((threadIdx.x & 63) == 0) {
    S.nsh = nsh;
    S.nls = nls;
    S.nfl = nfl;
    S.spill = spill;
    S.head = head;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int SR_CONC_MIN = 8;  // sectors run concurrently when each holds at least this many points

// The six sectors' greedy picks, concurrently (one wave each), in the reference's sequential
// result.  The reference runs sector j after sector j - 1, so the only state sector j inherits is
// the picked flags that j - 1's last picks spread into j's first (at most 5) points.  Sector j ran
// without them; its picks are still the reference's unless it picked one of those points (a flag
// on a point the run never picked changes no availability test the run's choices depended on).
// Wave 0 then walks the borders in order and reruns such a sector with the inherited flags (its
// own spill can change, so the next border is checked against the rerun's).
__device__ inline void sr_greedy_ring(int base, const int* lo, const int* hi, const uint64_t* keys, const int* len,
                                      uint8_t* picked, int8_t* lab, const uint8_t* gapok, SrSect* sect,
                                      unsigned long long* dbg) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wid < 6) sr_greedy_sector(base, lo[wid], hi[wid], true, keys + wid * SR_WSORT_MAX, len[wid], picked, lab, gapok,
                                sect[wid]);
  __syncthreads();
  if (wid == 0) {
    for (int j = 1; j < 6; ++j) {
      const uint32_t inh = sect[j - 1].spill;
      if (!(inh & sect[j].head)) continue;
      for (int k = lo[j] + lane; k <= hi[j]; k += 64) {
        picked[k] = (k - lo[j] < 5 && ((inh >> (k - lo[j])) & 1u)) ? 1 : 0;
        lab[k] = 0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      sr_greedy_sector(base, lo[j], hi[j], true, keys + j * SR_WSORT_MAX, len[j], picked, lab, gapok, sect[j]);
      if (lane == 0 && dbg) atomicAdd(dbg + 21, 1ull);  // (debug counter 21: sector reruns)
    }
  }
  __syncthreads();
}

// LDS of one ring's feature selection (carved from the ring workgroup's 160 KiB)
struct SrSelLds {
  uint64_t* keys;    // [6][SR_WSORT_MAX] the sorted sectors
  uint64_t* ssE;     // [6][SR_SS_LDS] exact re-sort of tied sectors (one wave each)
  uint32_t* ssA;     // [6][SR_SS_LDS]
  uint32_t* ssB;     // [6][SR_SS_LDS]
  uint8_t* picked;   // [SR_RING_CAP]
  int8_t* lab;       // [SR_RING_CAP]
  uint8_t* gapok;    // [SR_RING_CAP]
  int* ssSeg;        // [6][2][3 * SR_SS_SEG]
  SsLevels* ssLev;   // [6]
  SrSect* sect;      // [6]
  uint32_t* ws;      // [VX_WAVES]
};

constexpr size_t sr_align16(size_t b) { return (b + 15) & ~(size_t)15; }
constexpr size_t SR_SEL_LDS_BYTES =
    sr_align16(6 * SR_WSORT_MAX * 8) + sr_align16(6 * SR_SS_LDS * 8) + 2 * sr_align16(6 * SR_SS_LDS * 4) +
    3 * sr_align16(SR_RING_CAP) + sr_align16(6 * 2 * 3 * SR_SS_SEG * 4) + sr_align16(6 * sizeof(SsLevels)) +
    sr_align16(6 * sizeof(SrSect)) + sr_align16(VX_WAVES * 4);
static_assert(SR_SEL_LDS_BYTES <= (size_t)VX_LDS_WORDS * 4, "the ring's selection fits the workgroup's LDS");

__device__ inline SrSelLds sr_sel_carve(uint32_t* lds) {
  uint8_t* p = reinterpret_cast<uint8_t*>(lds);
  SrSelLds L;
  auto take = [&p](size_t b) {
    uint8_t* q = p;
    p += sr_align16(b);
    return q;
  };
  L.keys = reinterpret_cast<uint64_t*>(take(6 * SR_WSORT_MAX * 8));
  L.ssE = reinterpret_cast<uint64_t*>(take(6 * SR_SS_LDS * 8));
  L.ssA = reinterpret_cast<uint32_t*>(take(6 * SR_SS_LDS * 4));
  L.ssB = reinterpret_cast<uint32_t*>(take(6 * SR_SS_LDS * 4));
  L.picked = take(SR_RING_CAP);
  L.lab = reinterpret_cast<int8_t*>(take(SR_RING_CAP));
  L.gapok = take(SR_RING_CAP);
  L.ssSeg = reinterpret_cast<int*>(take(6 * 2 * 3 * SR_SS_SEG * 4));
  L.ssLev = reinterpret_cast<SsLevels*>(take(6 * sizeof(SsLevels)));
  L.sect = reinterpret_cast<SrSect*>(take(6 * sizeof(SrSect)));
  L.ws = reinterpret_cast<uint32_t*>(take(VX_WAVES * 4));
  return L;
}

// Feature selection of ring r (:352-493) by the whole workgroup (NT threads): the 6 sectors
// sorted by curvature at once (one wave per sector, register bitonic; a sector with tied
// curvatures re-sorted in libstdc++'s order), the greedy picks (sr_greedy_ring), the ring's pick
// lists and labels, and its lessFlat candidates compacted in index order into the ring's region
// of less_flat_scan.  Returns their number (0 for a ring too short to select from).
template <int NT>
__device__ inline int sr_select_ring(const SrDev& D, int r, const SrSelLds& M) {
  SrFrame& F = *D.fr;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int base = F.ring_off[r], n = F.ring_cnt[r];
  const int s = base + 5, e = base + n - 6;
  if (e - s < 6) {  // :355-356
    if (tid == 0) F.n_sharp[r] = F.n_less_sharp[r] = F.n_flat[r] = F.n_less_flat_scan[r] = 0;
    return 0;
  }
  if (n > SR_RING_CAP) {
    if (tid == 0) {
      F.n_sharp[r] = F.n_less_sharp[r] = F.n_flat[r] = F.n_less_flat_scan[r] = 0;
      atomicOr(&F.err, SR_ERR_RING);
    }
    return 0;
  }
  uint64_t* keys = M.keys;
  uint8_t* picked = M.picked;
  int8_t* lab = M.lab;
  const float4* L = D.cloud;
  for (int k = tid; k < n; k += NT) {
    picked[k] = 0;
    lab[k] = 0;
    uint8_t ok = 0;
    if (k + 1 < n) {  // the reference's float test, (dX^2 + dY^2 + dZ^2) > 0.05 in double
      const float4 a = L[base + k], b = L[base + k + 1];
      const float dX = b.x - a.x, dY = b.y - a.y, dZ = b.z - a.z;
      ok = (dX * dX + dY * dY + dZ * dZ > 0.05) ? 0 : 1;
    }
    M.gapok[k] = ok;
  }
  // sectors (:361-365); with all 6 short enough, wave j sorts sector j in registers
  int sp[6], len[6], lo[6], hi[6], maxlen = 0, minlen = 1 << 30;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    sp[j] = s + (e - s) * j / 6;
    len[j] = (s + (e - s) * (j + 1) / 6 - 1) - sp[j] + 1;
    lo[j] = sp[j] - base;
    hi[j] = lo[j] + len[j] - 1;
    maxlen = max(maxlen, len[j]);
    minlen = min(minlen, len[j]);
  }
  const bool fast = maxlen <= SR_WSORT_MAX;
  unsigned long long* prof = D.pdbg;  // (diagnostics: [13] sector sorts, [14] greedy, [15] slowest ring)
  const unsigned long long t0 = prof ? __builtin_readcyclecounter() : 0ull;
  if (!fast && maxlen > 6 * SR_WSORT_MAX) {
    if (tid == 0) {
      F.n_sharp[r] = F.n_less_sharp[r] = F.n_flat[r] = F.n_less_flat_scan[r] = 0;
      atomicOr(&F.err, SR_ERR_RING);
    }
    return 0;
  }
  if (fast && wid < 6) {
    uint64_t* K = keys + wid * SR_WSORT_MAX;
    if (maxlen <= 512) sr_wave_sort<8>(D.curv, sp[wid], len[wid], K);
    else sr_wave_sort<16>(D.curv, sp[wid], len[wid], K);
    sr_exact_sector(D, sp[wid], len[wid], K, M.ssE + wid * SR_SS_LDS, M.ssA + wid * SR_SS_LDS,
                    M.ssB + wid * SR_SS_LDS, &M.ssLev[wid], M.ssSeg + wid * 6 * SR_SS_SEG,
                    M.ssSeg + wid * 6 * SR_SS_SEG + 3 * SR_SS_SEG, SR_SS_SEG);
  }
  __syncthreads();
  const unsigned long long t1 = prof ? __builtin_readcyclecounter() : 0ull;
  if (fast && minlen >= SR_CONC_MIN) {
    sr_greedy_ring(base, lo, hi, keys, len, picked, lab, M.gapok, M.sect, D.dbg);
    if (tid == 0 && D.dbg) atomicAdd(D.dbg + 22, 1ull);  // (debug counter 22: rings with concurrent sectors)
  } else {
    // sequential sectors (a ring with a sector over SR_WSORT_MAX points, or one shorter than
    // SR_CONC_MIN): every suppression flag written where the reference writes it
    for (int j = 0; j < 6; j++) {
      const uint64_t* K = keys + j * SR_WSORT_MAX;
      if (!fast) {  // long sectors: block bitonic in LDS, one sector at a time
        K = keys;
        int pad = 1;
        while (pad < len[j]) pad <<= 1;
        for (int k = tid; k < pad; k += NT)
          keys[k] = k < len[j] ? (((uint64_t)__float_as_uint(D.curv[sp[j] + k]) << 32) | (uint32_t)(sp[j] + k))
                               : 0xFFFFFFFFFFFFFFFFull;
        __syncthreads();
        for (int kk = 2; kk <= pad; kk <<= 1) {
          for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            for (int i = tid; i < pad; i += NT) {
              const int ixj = i ^ jj;
              if (ixj > i) {
                const uint64_t a = keys[i], b = keys[ixj];
                const bool asc = (i & kk) == 0;
                if ((a > b) == asc) {
                  keys[i] = b;
                  keys[ixj] = a;
                }
              }
            }
            __syncthreads();
          }
        }
        if (wid == 0)
          sr_exact_sector(D, sp[j], len[j], keys, nullptr, nullptr, nullptr, &M.ssLev[0],
                          D.ss_seg + r * 6 * SR_SS_GSEG, D.ss_seg + r * 6 * SR_SS_GSEG + 3 * SR_SS_GSEG, SR_SS_GSEG);
        __syncthreads();
      }
      if (wid == 0) sr_greedy_sector(base, lo[j], hi[j], false, K, len[j], picked, lab, M.gapok, M.sect[j]);
      if (!fast) __syncthreads();
    }
    __syncthreads();
  }
  if (prof && tid == 0) {
    const unsigned long long t2 = __builtin_readcyclecounter();
    atomicAdd(prof + 13, t1 - t0);
    atomicAdd(prof + 14, t2 - t1);
    atomicMax(prof + 15, t2 - t0);
    atomicMax(prof + 19, t1 - t0);
    atomicMax(prof + 20, t2 - t1);
  }
  // the ring's pick lists, sectors in order (the reference appends them sector by sector)
  if (wid == 0) {
    int osh = 0, ols = 0, ofl = 0;
    for (int j = 0; j < 6; ++j) {
      const SrSect& S = M.sect[j];
      if (lane < S.nsh) D.ring_sharp[r * 6 * SR_SHARP + osh + lane] = S.sh[lane];
      if (lane < S.nls) D.ring_less_sharp[r * 6 * SR_LESS_SHARP + ols + lane] = S.ls[lane];
      if (lane < S.nfl) D.ring_flat[r * 6 * SR_FLAT + ofl + lane] = S.fl[lane];
      osh += S.nsh;
      ols += S.nls;
      ofl += S.nfl;
    }
    if (lane == 0) {
      F.n_sharp[r] = osh;
      F.n_less_sharp[r] = ols;
      F.n_flat[r] = ofl;
    }
  }
  // lessFlat candidates: label <= 0 in index order (:486-493) over [s, e), the 6 sectors
  // back to back; stable block compaction
  int nlf = 0;
  for (int c = s; c < e; c += NT) {
    const int k = c + tid;
    const bool pred = k < e && lab[k - base] <= 0;
    const uint64_t bal = __ballot(pred);
    const uint32_t pre = __popcll(bal & lanemask_lt());
    if (lane == 0) M.ws[wid] = __popcll(bal);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < NT / 64; ++w) {
      if (w < wid) off += M.ws[w];
      tot += M.ws[w];
    }
    if (pred) D.less_flat_scan[base + nlf + off + pre] = L[k];
    nlf += tot;
    __syncthreads();
  }
  for (int k = tid; k < n; k += NT) D.label[base + k] = lab[k];
  if (tid == 0) F.n_less_flat_scan[r] = nlf;
  return nlf;
}

// PCL VoxelGrid of one ring's lessFlat candidates (scan_registration.cpp:497-501) in PCL's
// summation order: the input-order filter (voxel.h) sums every voxel of at most 2 members
// (order-free) and records the others, then voxel_hot.h runs the pruned std::sort emulation in
// LDS and sums those voxels in its order.  Scratch: the ring's region of the sector sort's
// arrays (the ring's selection is done with them).
constexpr int SRV_THREADS = VX_THREADS;
static_assert(SR_RING_CAP <= VH_MAX_N, "a ring's lessFlat cloud fits the LDS emulation");

__device__ inline void sr_ringvox(const SrDev& D, int r, int n, uint32_t* lds) {
  SrFrame& F = *D.fr;
  const int base = F.ring_off[r];
  VoxSeg S{};
  S.src0 = D.less_flat_scan + base;
  S.n0 = n;
  S.leaf = 0.2f;
  S.out = D.less_flat_ds + base;
  S.cap = (uint32_t)n;
  S.res_cnt = &F.n_less_flat[r];
  S.scratch_idx = reinterpret_cast<int*>(D.ss_b + base);
  S.scratch_cap = (uint32_t)n;
  S.err = &F.err;
  S.hot.rk = D.ss_a + base;
  S.hot.hl = reinterpret_cast<uint32_t*>(D.ss_e + base);
  S.hot.hv = S.hot.hl + n;  // 3 words per hot voxel, at most n / 3 of them: within the ring's 2 n
  S.hot.fpos = reinterpret_cast<uint32_t*>(D.ss_s + base);
  S.hot.cap_h = (uint32_t)n / 3;
  unsigned long long* prof = D.pdbg;
  const unsigned long long t0 = __builtin_readcyclecounter();
  voxel_segment(S, lds);
  const unsigned long long t1 = __builtin_readcyclecounter();
  const int heap_el = vh_fixup<SRV_THREADS>(VxSrc{S.src0, n, nullptr}, n, S.out, S.hot, lds, VX_LDS_WORDS - 256,
                                            *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192), nullptr, &F.err,
                                            prof, prof ? prof + 8 : nullptr);
  if (prof && threadIdx.x == 0) {  // (diagnostics: include/loam_core.h LOAM_SR_DEBUG_COUNTERS)
    const unsigned long long t2 = __builtin_readcyclecounter();
    atomicAdd(prof + 4, t1 - t0);
    atomicAdd(prof + 5, (unsigned long long)n);
    atomicMax(prof + 6, (unsigned long long)n);
    atomicMax(prof + 7, (unsigned long long)heap_el);
    // the slowest ring: its cycles in the high bits, then its heap-sorted elements and points
    atomicMax(prof + 3, t2 - t0);
    atomicMax(prof + 16, ((t2 - t0) << 32) | ((unsigned long long)heap_el << 16) | (unsigned long long)n);
    atomicMax(prof + 18, ((t2 - t0) << 32) | (t2 - t1));
  }
}

// A ring's selection and then its lessFlat VoxelGrid in one workgroup: the ring's VoxelGrid
// starts when its own picks are done, not when the slowest ring's are, and both phases share
// the 160 KiB.  Inlined into the kernel (as a called function its frame spilled 464 B per lane
// to scratch; 84 inlined).
__device__ __attribute__((always_inline)) inline void sr_ring_features(const SrDev* __restrict__ Ds) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  const SrDev D = Ds[blockIdx.y];
  const int r = blockIdx.x;
  const int nlf = sr_select_ring<SRV_THREADS>(D, r, sr_sel_carve(lds));
  __syncthreads();  // (the ring's lessFlat points were written by this workgroup: same CU)
  sr_ringvox(D, r, nlf, lds);
}

__global__ void __launch_bounds__(SRV_THREADS) k_sr_ring_features(const SrDev* __restrict__ Ds) {
  sr_ring_features(Ds);
}

// concatenation of the per-ring outputs in ring order
__global__ void k_sr_gather(const SrDev* __restrict__ Ds) {
  const SrDev D = Ds[blockIdx.y];
  const int r = blockIdx.x;
  SrFrame& F = *D.fr;
  int o1 = 0, o2 = 0, o3 = 0, o4 = 0;
  for (int q = 0; q < r; ++q) {
    o1 += F.n_sharp[q];
    o2 += F.n_less_sharp[q];
    o3 += F.n_flat[q];
    o4 += (int)F.n_less_flat[q];
  }
  const float4* L = D.cloud;
  for (int k = threadIdx.x; k < F.n_sharp[r]; k += blockDim.x)
    D.out[1][o1 + k] = L[D.ring_sharp[r * 6 * SR_SHARP + k]];
  for (int k = threadIdx.x; k < F.n_less_sharp[r]; k += blockDim.x)
    D.out[2][o2 + k] = L[D.ring_less_sharp[r * 6 * SR_LESS_SHARP + k]];
  for (int k = threadIdx.x; k < F.n_flat[r]; k += blockDim.x)
    D.out[3][o3 + k] = L[D.ring_flat[r * 6 * SR_FLAT + k]];
  const int base = F.ring_off[r];
  for (int k = threadIdx.x; k < (int)F.n_less_flat[r]; k += blockDim.x)
    D.out[4][o4 + k] = D.less_flat_ds[base + k];
  if (r == SR_MAX_RINGS - 1 && threadIdx.x == 0) {
    F.out_n[0] = F.n_cloud;
    F.out_n[1] = o1 + F.n_sharp[r];
    F.out_n[2] = o2 + F.n_less_sharp[r];
    F.out_n[3] = o3 + F.n_flat[r];
    F.out_n[4] = o4 + (int)F.n_less_flat[r];
  }
}

}  // namespace loam

using namespace loam;

struct loam_scanreg {
  loam_params P;
  int dev = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // frames per launch sequence (loam_scanreg_create_batch; 1 for loam_scanreg_create): every
  // per-frame buffer exists nb times, Dv[f] points at frame f's; D is frame 0's (the single-frame
  // calls)
  int nb = 1;
  std::vector<SrDev> Dv;
  SrDev D{};
  SrDev* d_Ds = nullptr;      // [nb] the launch's frame views (kernel argument arrays)
  SrDev* h_Ds = nullptr;      // [nb] page-locked staging of d_Ds
  int nf = 0;                 // frames of the last launch
  std::vector<SrFrame> hfv;   // [nb] their records after the wait
  SrFrame hf{};               // frame 0's
  float* d_in = nullptr;      // [nb][cap][4] staging of host input
  float* h_pinned = nullptr;  // loam_scanreg_host_buffer: page-locked ingest buffer (cap x 4 floats)
  SrFrame* hf_pinned = nullptr;  // [nb] D2H target of the frame records (page-locked: the copy stays async)
  int pending = 0;            // loam_scanreg_input_async launched, loam_scanreg_wait not yet called
  int pending_stride = 4;
  const float* pending_xyz = nullptr;
  std::vector<void*> allocs;
  float ms = 0.f;
};

namespace {
template <typename T>
int32_t sralloc(loam_scanreg* h, T** p, size_t n) {
  void* q = nullptr;
  LOAM_HIP(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)));
  // zero on the handle's own (non-blocking) stream: a null-stream memset is not ordered
  // before this stream's kernels; create() synchronizes the stream before returning
  LOAM_HIP(hipMemsetAsync(q, 0, std::max<size_t>(n, 1) * sizeof(T), h->st));
  h->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return LOAM_OK;
}
void sr_free(loam_scanreg* h) {
  if (h->st) (void)hipStreamSynchronize(h->st);  // an input_async still in flight
  if (h->h_pinned) (void)hipHostFree(h->h_pinned);
  if (h->hf_pinned) (void)hipHostFree(h->hf_pinned);
  if (h->h_Ds) (void)hipHostFree(h->h_Ds);
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->st) (void)hipStreamDestroy(h->st);
}
}  // namespace

extern "C" {

int32_t loam_scanreg_create(const loam_params* p, int32_t device, loam_scanreg** out) {
  return loam_scanreg_create_batch(p, device, 1, out);
}

int32_t loam_scanreg_create_batch(const loam_params* p, int32_t device, int32_t max_frames, loam_scanreg** out) {
  if (!out || max_frames < 1) return LOAM_ERR_ARG;
  *out = nullptr;
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  vh_spin_limit_from_env(device);
  auto* h = new loam_scanreg;
  if (p) h->P = *p; else loam_params_default(&h->P);
  if (h->P.scan_line != 16 && h->P.scan_line != 32 && h->P.scan_line != 64) {
    delete h;
    set_error("only support velodyne with 16, 32 or 64 scan line (scan_registration.cpp:58-61)");
    return LOAM_ERR_ARG;
  }
  h->dev = device;
  h->nb = max_frames;
  const int nb = max_frames;
  h->Dv.assign(nb, SrDev{});
  h->hfv.assign(nb, SrFrame{});
  const int cap = h->P.max_input_points;
  SrDev& D = h->D;
  D.cap = cap;
  D.n_scans = h->P.scan_line;
  D.min_range = (float)h->P.minimum_range;
  const int nblocks = (cap + SR_BLOCK - 1) / SR_BLOCK;
  auto fail = [&](int32_t r) {
    sr_free(h);
    delete h;
    return r;
  };
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) return fail(LOAM_ERR_HIP);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(LOAM_ERR_HIP);
  // every per-frame buffer: one allocation of nb copies, frame f's at f * n
#define SRA(field, n)                                                      \
  do {                                                                     \
    const size_t n_ = (n);                                                 \
    if ((rc = sralloc(h, &D.field, n_ * nb)) != LOAM_OK) return fail(rc);  \
    for (int f = 0; f < nb; ++f) h->Dv[f].field = D.field + f * n_;        \
  } while (0)
  if ((rc = sralloc(h, &h->d_in, (size_t)cap * 4 * nb)) != LOAM_OK) return fail(rc);
  SRA(fr, 1);
  SRA(ring_of, cap);
  SRA(blk_hist, (size_t)SR_MAX_RINGS * nblocks);
  SRA(blk_off, (size_t)SR_MAX_RINGS * nblocks);
  SRA(blk_aux, (size_t)3 * nblocks);
  SRA(cloud, cap);
  SRA(curv, cap);
  SRA(label, cap);
  SRA(ring_sharp, SR_MAX_RINGS * 6 * SR_SHARP);
  SRA(ring_less_sharp, SR_MAX_RINGS * 6 * SR_LESS_SHARP);
  SRA(ring_flat, SR_MAX_RINGS * 6 * SR_FLAT);
  SRA(less_flat_scan, cap);
  SRA(less_flat_ds, cap);
  SRA(vx_pts, cap);
  SRA(vx_idx, cap);
  for (int k = 1; k < 5; ++k) SRA(out[k], cap);
  SRA(ss_e, cap);
  SRA(ss_a, cap);
  SRA(ss_b, cap);
  SRA(ss_s, cap);
  SRA(ss_seg, (size_t)SR_MAX_RINGS * 6 * SR_SS_GSEG);
  if ((rc = sralloc(h, &D.dbg, LOAM_SR_DEBUG_COUNTERS)) != LOAM_OK) return fail(rc);  // shared by the frames
  {
    const char* penv = std::getenv("LOAM_PHASE_COUNTERS");
    D.pdbg = (penv && std::atoi(penv) > 0) ? D.dbg : nullptr;
  }
#undef SRA
  if ((rc = sralloc(h, &h->d_Ds, nb)) != LOAM_OK) return fail(rc);
  if (hipHostMalloc(reinterpret_cast<void**>(&h->h_Ds), sizeof(SrDev) * nb, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&h->hf_pinned), sizeof(SrFrame) * nb, hipHostMallocDefault) != hipSuccess)
    return fail(LOAM_ERR_HIP);
  D.out[0] = D.cloud;
  D.sort_ind = nullptr;
  for (int f = 0; f < nb; ++f) {  // the scalars and the shared pointers
    SrDev& V = h->Dv[f];
    V.cap = D.cap;
    V.n_scans = D.n_scans;
    V.min_range = D.min_range;
    V.dbg = D.dbg;
    V.pdbg = D.pdbg;
    V.out[0] = V.cloud;
    V.sort_ind = nullptr;
  }
  h->Dv[0] = D;
  if (hipStreamSynchronize(h->st) != hipSuccess) return fail(LOAM_ERR_HIP);
  *out = h;
  return LOAM_OK;
}

int32_t loam_scanreg_destroy(loam_scanreg* h) {
  if (!h) return LOAM_ERR_ARG;
  (void)hipSetDevice(h->dev);
  sr_free(h);
  delete h;
  return LOAM_OK;
}

static int32_t sr_finish(loam_scanreg* h);

// enqueue nf frames (H2D when host memory, then every kernel, frame f in grid row y = f, and the
// D2H of the frame records) on the handle's stream; sr_finish waits for them
static int32_t sr_launch_frames(loam_scanreg* h, int nf, const float* const* xyz, const int32_t* n, int32_t stride,
                                bool on_device) {
  if (!h || nf < 1 || nf > h->nb || !xyz || !n || stride < 3) {
    set_error("loam_scanreg_input: bad arguments");
    return LOAM_ERR_ARG;
  }
  int nmax = 0;
  for (int f = 0; f < nf; ++f) {
    if (n[f] < 0 || (n[f] > 0 && !xyz[f])) {
      set_error("loam_scanreg_input: bad arguments");
      return LOAM_ERR_ARG;
    }
    if (n[f] > h->D.cap) {
      set_error("loam_scanreg_input: more points than max_input_points");
      return LOAM_ERR_CAPACITY;
    }
    nmax = std::max(nmax, (int)n[f]);
  }
  if (!on_device && stride != 4)
    for (int f = 0; f < nf; ++f)
      if ((size_t)n[f] * stride > (size_t)h->D.cap * 4) {
        set_error("loam_scanreg_input: stride too large for the staging buffer");
        return LOAM_ERR_CAPACITY;
      }
  LOAM_HIP(hipSetDevice(h->dev));
  hipStream_t st = h->st;
  for (int f = 0; f < nf; ++f) {  // (the previous launch's copy of h_Ds is done: sr_finish came first)
    SrDev D = h->Dv[f];
    D.stride = stride;
    D.n_in = n[f];
    if (on_device) {
      D.xyz = xyz[f];
    } else {
      float* stage = h->d_in + (size_t)f * h->D.cap * 4;
      if (n[f]) LOAM_HIP(hipMemcpyAsync(stage, xyz[f], sizeof(float) * (size_t)n[f] * stride, hipMemcpyHostToDevice, st));
      D.xyz = stage;
    }
    h->h_Ds[f] = D;
  }
  LOAM_HIP(hipMemcpyAsync(h->d_Ds, h->h_Ds, sizeof(SrDev) * nf, hipMemcpyHostToDevice, st));
  static_assert(sizeof(SrFrame) % 4 == 0, "k_sr_init writes the record by words");
  LOAM_HIP(hipEventRecord(h->ev[0], st));
  const SrDev* Ds = h->d_Ds;
  k_sr_init<<<dim3(1, nf), 256, 0, st>>>(Ds);
  const int nblocks = std::max(1, (nmax + SR_BLOCK - 1) / SR_BLOCK);
  if (nmax > 0) {
    k_sr_valid<<<dim3(nblocks, nf), SR_BLOCK, 0, st>>>(Ds, nblocks);
    k_sr_oris<<<dim3(1, nf), 1024, 0, st>>>(Ds, nblocks);
    k_sr_ring<<<dim3(nblocks, nf), SR_BLOCK, 0, st>>>(Ds, nblocks);
    k_sr_ring_scan<<<dim3(1, nf), 1024, 0, st>>>(Ds, nblocks);
    k_sr_scatter<<<dim3(nblocks, nf), SR_BLOCK, 0, st>>>(Ds, nblocks);
    k_sr_curv<<<dim3(std::min(nblocks, 1024), nf), SR_BLOCK, 0, st>>>(Ds);
    k_sr_ring_features<<<dim3(SR_MAX_RINGS, nf), SRV_THREADS, 0, st>>>(Ds);
    k_sr_gather<<<dim3(SR_MAX_RINGS, nf), 256, 0, st>>>(Ds);
    LOAM_HIP(hipGetLastError());
  }
  LOAM_HIP(hipEventRecord(h->ev[1], st));
  LOAM_HIP(hipMemcpyAsync(h->hf_pinned, h->Dv[0].fr, sizeof(SrFrame) * nf, hipMemcpyDeviceToHost, st));
  h->pending = 1;
  h->nf = nf;
  h->pending_xyz = h->h_Ds[0].xyz;
  h->pending_stride = stride;
  return LOAM_OK;
}

static int32_t sr_launch(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride, bool on_device) {
  if (!h) return LOAM_ERR_ARG;
  return sr_launch_frames(h, 1, &xyz, &n, stride, on_device);
}

static int32_t sr_finish(loam_scanreg* h) {
  if (!h->pending) return LOAM_OK;
  h->pending = 0;
  LOAM_HIP(hipSetDevice(h->dev));
  LOAM_HIP(hipStreamSynchronize(h->st));
  for (int f = 0; f < h->nf; ++f) h->hfv[f] = h->hf_pinned[f];
  h->hf = h->hfv[0];
  LOAM_HIP(hipEventElapsedTime(&h->ms, h->ev[0], h->ev[1]));
  h->D.xyz = h->pending_xyz;
  h->D.stride = h->pending_stride;
  int e = 0, ef = 0;
  for (int f = 0; f < h->nf && !e; ++f)
    if (h->hfv[f].err) {
      e = h->hfv[f].err;
      ef = f;
    }
  if (e) {
    set_error(std::string("loam_scanreg_input: frame ") + std::to_string(ef) + ": " +
              ((e & VH_ERR_SPIN) ? "ring VoxelGrid sort: a wave's wait for a listed subtree ran out"
               : (e & SR_ERR_SORT) ? "std::sort emulation level list overflow"
                                   : "ring or sector larger than the LDS capacity") +
              " (err " + std::to_string(e) + ")");
    return (e & VH_ERR_SPIN) ? LOAM_ERR_SYNC : LOAM_ERR_CAPACITY;
  }
  return LOAM_OK;
}

static int32_t sr_run(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride, bool on_device) {
  if (h && h->pending) TRY(sr_finish(h));
  TRY(sr_launch(h, xyz, n, stride, on_device));
  return sr_finish(h);
}

int32_t loam_scanreg_input(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride) {
  return sr_run(h, xyz, n, stride, false);
}

int32_t loam_scanreg_input_device(loam_scanreg* h, const float* d_xyz, int32_t n, int32_t stride) {
  return sr_run(h, d_xyz, n, stride, true);
}

int32_t loam_scanreg_host_buffer(loam_scanreg* h, float** ptr, int32_t* cap_points) {
  if (!h || !ptr) return LOAM_ERR_ARG;
  if (!h->h_pinned) {
    LOAM_HIP(hipSetDevice(h->dev));
    LOAM_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->h_pinned), sizeof(float) * 4 * (size_t)h->D.cap,
                           hipHostMallocDefault));
  }
  *ptr = h->h_pinned;
  if (cap_points) *cap_points = h->D.cap;
  return LOAM_OK;
}

int32_t loam_scanreg_input_async(loam_scanreg* h, const float* xyz, int32_t n, int32_t stride) {
  if (h && h->pending) TRY(sr_finish(h));
  return sr_launch(h, xyz, n, stride, false);
}

int32_t loam_scanreg_wait(loam_scanreg* h) {
  if (!h) return LOAM_ERR_ARG;
  return sr_finish(h);
}

int32_t loam_scanreg_counts(loam_scanreg* h, int32_t* counts) {
  if (!h || !counts) return LOAM_ERR_ARG;
  TRY(sr_finish(h));  // an input_async in flight completes first
  for (int k = 0; k < 5; ++k) counts[k] = h->hf.n_in > 0 ? h->hf.out_n[k] : 0;
  return LOAM_OK;
}

int32_t loam_scanreg_copy(loam_scanreg* h, int32_t which, float* out, int32_t cap) {
  if (!h || which < 0 || which > 4 || (cap > 0 && !out)) return LOAM_ERR_ARG;
  TRY(sr_finish(h));  // an input_async in flight completes first
  LOAM_HIP(hipSetDevice(h->dev));
  const int n = h->hf.n_in > 0 ? h->hf.out_n[which] : 0;
  if (n > cap) {
    set_error("loam_scanreg_copy: output buffer too small");
    return LOAM_ERR_CAPACITY;
  }
  if (n) LOAM_HIP(hipMemcpy(out, h->D.out[which], sizeof(float4) * n, hipMemcpyDeviceToHost));
  return n;
}

int32_t loam_scanreg_device_ptr(loam_scanreg* h, int32_t which, const float** ptr) {
  if (!h || which < 0 || which > 4 || !ptr) return LOAM_ERR_ARG;
  TRY(sr_finish(h));  // an input_async in flight completes first
  *ptr = reinterpret_cast<const float*>(h->D.out[which]);
  return h->hf.n_in > 0 ? h->hf.out_n[which] : 0;
}

int32_t loam_scanreg_curvature(loam_scanreg* h, float* curv, int32_t* label, int32_t cap) {
  if (!h || (cap > 0 && (!curv || !label))) return LOAM_ERR_ARG;
  TRY(sr_finish(h));  // an input_async in flight completes first
  LOAM_HIP(hipSetDevice(h->dev));
  const int n = h->hf.n_in > 0 ? h->hf.n_cloud : 0;
  if (n > cap) return LOAM_ERR_CAPACITY;
  if (n) {
    LOAM_HIP(hipMemcpy(curv, h->D.curv, sizeof(float) * n, hipMemcpyDeviceToHost));
    LOAM_HIP(hipMemcpy(label, h->D.label, sizeof(int) * n, hipMemcpyDeviceToHost));
  }
  return n;
}

double loam_scanreg_ms(loam_scanreg* h) { return h ? (double)h->ms : 0.0; }

int32_t loam_scanreg_input_batch(loam_scanreg* h, int32_t n_frames, const uint64_t* xyz, const int32_t* n,
                                 int32_t stride, int32_t on_device) {
  if (!h || n_frames < 1 || n_frames > h->nb || !xyz || !n) {
    set_error("loam_scanreg_input_batch: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (h->pending) TRY(sr_finish(h));
  std::vector<const float*> p(n_frames);
  for (int f = 0; f < n_frames; ++f) p[f] = reinterpret_cast<const float*>(xyz[f]);
  TRY(sr_launch_frames(h, n_frames, p.data(), n, stride, on_device != 0));
  return sr_finish(h);
}

static int32_t sr_frame_ok(loam_scanreg* h, int32_t frame) {
  if (!h || frame < 0) return LOAM_ERR_ARG;
  TRY(sr_finish(h));  // an input_async in flight completes first
  if (frame >= std::max(h->nf, 1)) {
    set_error("loam_scanreg: frame index past the last launch's frames");
    return LOAM_ERR_ARG;
  }
  return LOAM_OK;
}

int32_t loam_scanreg_frame_counts(loam_scanreg* h, int32_t frame, int32_t* counts) {
  if (!counts) return LOAM_ERR_ARG;
  TRY(sr_frame_ok(h, frame));
  const SrFrame& F = h->hfv[frame];
  for (int k = 0; k < 5; ++k) counts[k] = F.n_in > 0 ? F.out_n[k] : 0;
  return LOAM_OK;
}

int32_t loam_scanreg_frame_device_ptr(loam_scanreg* h, int32_t frame, int32_t which, const float** ptr) {
  if (which < 0 || which > 4 || !ptr) return LOAM_ERR_ARG;
  TRY(sr_frame_ok(h, frame));
  *ptr = reinterpret_cast<const float*>(h->Dv[frame].out[which]);
  return h->hfv[frame].n_in > 0 ? h->hfv[frame].out_n[which] : 0;
}

int32_t loam_scanreg_frame_copy(loam_scanreg* h, int32_t frame, int32_t which, float* out, int32_t cap) {
  if (which < 0 || which > 4 || (cap > 0 && !out)) return LOAM_ERR_ARG;
  TRY(sr_frame_ok(h, frame));
  LOAM_HIP(hipSetDevice(h->dev));
  const int n = h->hfv[frame].n_in > 0 ? h->hfv[frame].out_n[which] : 0;
  if (n > cap) {
    set_error("loam_scanreg_frame_copy: output buffer too small");
    return LOAM_ERR_CAPACITY;
  }
  if (n) LOAM_HIP(hipMemcpy(out, h->Dv[frame].out[which], sizeof(float4) * n, hipMemcpyDeviceToHost));
  return n;
}

int32_t loam_scanreg_debug_counters(loam_scanreg* h, uint64_t* out, int32_t n, int32_t reset) {
  if (!h || !out || n < 0) return set_error("loam_scanreg_debug_counters: bad argument"), LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  LOAM_HIP(hipStreamSynchronize(h->st));
  const int k = std::min<int>(n, LOAM_SR_DEBUG_COUNTERS);
  LOAM_HIP(hipMemcpy(out, h->D.dbg, sizeof(uint64_t) * k, hipMemcpyDeviceToHost));
  if (reset) LOAM_HIP(hipMemset(h->D.dbg, 0, sizeof(uint64_t) * LOAM_SR_DEBUG_COUNTERS));
  return LOAM_OK;
}

}  // extern "C"
