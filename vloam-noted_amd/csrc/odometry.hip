// odometry.hip — LaserOdometry::solveLO (laser_odometry.cpp:199-584) on MI355X.
//
// One handle = B independent odometry streams; every launch covers all of them.  Per frame:
//   2 x { k_od_corr   one wave per query (cornerPointsSharp, surfPointsFlat): TransformToStart
//                     (:152-173, s = 1), exact 1-NN in the last cloud (KdTreeFLANN, d2 < 25,
//                     :292/:398) over a 2 m cell grid, then the second / third point by the
//                     reference's own linear scans of the last cloud from the 1-NN
//                     (:309-355 corner, :407-456 surf), 64 points per wave step
//                     -> factor records (LidarEdgeFactor / LidarPlaneFactor)
//         k_od_lm     Ceres TR-LM on the records (lm.h, one launch per round) }
//   k_od_build        laserCloudCornerLast / SurfLast <- lessSharp / lessFlat (:559-569) and
//                     their 2 m cell tables (replaces kdtree->setInputCloud, :571-572)
// The pose composition t_w += q_w t_lc, q_w = q_w q_lc (:524-527) runs on the host with the
// oracle's operation order.
//
// The ring scans are restated literally, not as a ring-filtered nearest search: int(intensity)
// is not monotone along a last cloud (points before the halfPassed latch with relTime < 0 carry
// scanID - 1, scan_registration.cpp:263-296; the lessSharp picks follow curvature order and
// lessFlat voxel order), and the reference's `continue` / `break` tests (:312-317, :337-342,
// :410, :436) decide which points are visited.  A wave steps 64 consecutive points at a time;
// the first lane whose point triggers the `break` ends the scan, the lanes before it are the
// visited points.  Each lane keeps its own running minimum under strict '<' (its points come
// in scan order), and the lanes' minima are merged with the scan order as the tie rule: the
// forward scan's earliest j, then the backward scan's latest j, the backward one only if
// strictly nearer (minPointSqDis2 / 3 carry over from the forward loop).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "device_math.h"
#include "lm.h"

namespace loam {

constexpr int OD_TAB = 16384;        // cell table slots per last cloud (LDS-built)
constexpr float OD_INV_CELL = 0.5f;  // 2 m cells
constexpr float OD_CELL = 2.0f;
constexpr int OD_ORIGIN = 256;       // cell coordinates offset: +-512 m around the sensor
constexpr float OD_THR = 25.0f;      // DISTANCE_SQ_THRESHOLD (laser_odometry.h:90)
constexpr int OD_QBLK_MAX = 1024;   // query workgroups per stream (at most; one wave per query)
constexpr int OD_QTHREADS = 256;
constexpr int OD_LM_THREADS = 256;
constexpr int OD_BUILD_THREADS = 1024;
constexpr uint32_t OD_EMPTY = 0xFFFFFFFFu;
constexpr int OD_ERR_CAPACITY = 1, OD_ERR_TABLE = 2, OD_ERR_LM_SYNC = 4;
constexpr int OD_MAXQ = 16384;       // sharp + flat queries per stream
constexpr int VX_WAVES_OD = OD_BUILD_THREADS / 64;
constexpr int OD_PBLK = 32;          // LM partials per stream (workgroups per stream <= this)

struct OdomFrame {
  double x[7];  // para_q (xyzw) + para_t: q_last_curr / t_last_curr, in/out
  int active;   // received an input this call
  int inited;   // systemInited (a last cloud exists)
  int n_in[4];  // sharp, lessSharp, flat, lessFlat
  const float4* in_ptr[4];
  int n_last[2];  // cornerLast, surfLast
  int corr[4];    // corner / plane correspondences, rounds 0 and 1
  int err;
  int has_prior;   // !detach_VO_LO: every outer round starts from `prior` (laser_odometry.cpp:237-250)
  double prior[7];
  LmState lm[2];
};

struct OdomDev {
  int* corr_part;  // [B][2 rounds][OD_QBLK_MAX][2] per-workgroup correspondence counts of k_od_corr
  int B, cap;
  OdomFrame* fr;
  float4* stage[4];    // [B][cap] host-input staging
  float4* last[2];     // [B][cap] last clouds, reference order
  float4* lsort[2];    // [B][cap] cell-sorted copy (w = intensity)
  int* lsidx[2];       // [B][cap] original index of lsort entries
  uint4* ltab[2];      // [B][OD_TAB] {key, start, count, -}
  uint32_t* scratch;   // [B][2][cap] slot << 16 | rank (build)
  int* r_type;         // records [B][OD_MAXQ]
  float *r_px, *r_py, *r_pz;
  double* r_a[3];
  double* r_b[3];
  double* partials;    // [B][OD_PBLK][LM_NACC]
  uint32_t* lm_sync;   // [B][2][LM_SYNC_WORDS] (lm.h)
  double* lm_xpub;     // [B][2][8]
};

__device__ inline int od_cell(float v) {
  const int c = (int)floorf(v * OD_INV_CELL) + OD_ORIGIN;
  return min(max(c, 0), 511);
}
__device__ inline uint32_t od_key(int x, int y, int z) {
  return (uint32_t)x | ((uint32_t)y << 9) | ((uint32_t)z << 18);
}
__device__ inline uint32_t od_hash(uint32_t k) {
  uint32_t h = k * 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h & (OD_TAB - 1);
}
__device__ inline uint4 od_find(const uint4* tab, uint32_t key) {
  uint32_t h = od_hash(key);
  for (int p = 0; p < OD_TAB; ++p) {
    const uint4 e = tab[h];
    if (e.x == key) return e;
    if (e.x == OD_EMPTY) break;
    h = (h + 1) & (OD_TAB - 1);
  }
  return make_uint4(OD_EMPTY, 0, 0, 0);
}
// squared distance from q to cell (x, y, z) (0 inside)
__device__ inline float od_gap2(float qx, float qy, float qz, int x, int y, int z) {
  auto g = [](float q, int c) {
    const float lo = (float)(c - OD_ORIGIN) * OD_CELL, hi = lo + OD_CELL;
    return q < lo ? lo - q : (q > hi ? q - hi : 0.0f);
  };
  const float gx = g(qx, x), gy = g(qy, y), gz = g(qz, z);
  return gx * gx + gy * gy + gz * gz;
}

// ---------------------------------------------------------------------------------------
// last clouds <- lessSharp / lessFlat, and their cell tables: one workgroup per (stream,
// cloud); LDS open-addressing table of the 2 m cells, counting sort of the points by cell
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(OD_BUILD_THREADS) k_od_build(OdomDev D) {
  __shared__ uint32_t lkey[OD_TAB];
  __shared__ uint32_t lcnt[OD_TAB];
  __shared__ uint32_t ws[VX_WAVES_OD + 1];
  const int s = blockIdx.x >> 1, c = blockIdx.x & 1;
  OdomFrame& F = D.fr[s];
  if (!F.active) return;
  const int tid = threadIdx.x;
  const int n = min(F.n_in[c == 0 ? 1 : 3], D.cap);  // lessSharp -> cornerLast, lessFlat -> surfLast
  const float4* src = F.in_ptr[c == 0 ? 1 : 3];
  const size_t base = (size_t)s * D.cap;
  float4* last = D.last[c] + base;
  float4* srt = D.lsort[c] + base;
  int* sidx = D.lsidx[c] + base;
  uint32_t* sc = D.scratch + ((size_t)s * 2 + c) * D.cap;
  uint4* tab = D.ltab[c] + (size_t)s * OD_TAB;
  for (int i = tid; i < OD_TAB; i += OD_BUILD_THREADS) {
    lkey[i] = OD_EMPTY;
    lcnt[i] = 0;
  }
  __syncthreads();
  bool full = false;
  for (int i = tid; i < n; i += OD_BUILD_THREADS) {
    const float4 p = src[i];
    last[i] = p;
    const uint32_t key = od_key(od_cell(p.x), od_cell(p.y), od_cell(p.z));
    uint32_t h = od_hash(key);
    int probe = 0;
    for (; probe < OD_TAB; ++probe) {
      const uint32_t old = atomicCAS(&lkey[h], OD_EMPTY, key);
      if (old == OD_EMPTY || old == key) break;
      h = (h + 1) & (OD_TAB - 1);
    }
    if (probe == OD_TAB) {
      full = true;
      sc[i] = 0xFFFFFFFFu;
      continue;
    }
    sc[i] = (h << 16) | (atomicAdd(&lcnt[h], 1u) & 0xFFFFu);
  }
  if (full) atomicOr(&F.err, OD_ERR_TABLE);
  __syncthreads();
  // exclusive scan of the slot counts (16 slots per thread) -> starts; table to global
  constexpr int PER = OD_TAB / OD_BUILD_THREADS;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    v[k] = lcnt[tid * PER + k];
    sum += v[k];
  }
  const int wid = tid >> 6, lane = tid & 63;
  uint32_t inc = wave_incl_scan_u(sum);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < VX_WAVES_OD; ++w) {
      const uint32_t t = ws[w];
      ws[w] = acc;
      acc += t;
    }
  }
  __syncthreads();
  uint32_t pre = ws[wid] + inc - sum;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int sl = tid * PER + k;
    tab[sl] = make_uint4(lkey[sl], pre, v[k], 0);
    lcnt[sl] = pre;  // start
    pre += v[k];
  }
  __syncthreads();
  for (int i = tid; i < n; i += OD_BUILD_THREADS) {
    const uint32_t e = sc[i];
    if (e == 0xFFFFFFFFu) continue;
    const uint32_t pos = lcnt[e >> 16] + (e & 0xFFFFu);
    srt[pos] = last[i];
    sidx[pos] = i;
  }
  if (tid == 0) F.n_last[c] = n;
}

// ---------------------------------------------------------------------------------------
// correspondences of one round -> factor records
// ---------------------------------------------------------------------------------------
struct OdNear {  // running minimum of (d2, order)
  float d;
  uint32_t ord;
  int j;
};
__device__ inline void od_offer(OdNear& b, float d, uint32_t ord, int j) {
  if (d < b.d || (d == b.d && ord < b.ord)) {
    b.d = d;
    b.ord = ord;
    b.j = j;
  }
}

// wave-wide minimum of (d2, order): every lane ends with the same candidate
__device__ inline OdNear od_wave_min(OdNear b) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float d = __shfl_xor(b.d, o, 64);
    const uint32_t ord = __shfl_xor(b.ord, o, 64);
    const int j = __shfl_xor(b.j, o, 64);
    if (d < b.d || (d == b.d && ord < b.ord)) {
      b.d = d;
      b.ord = ord;
      b.j = j;
    }
  }
  return b;
}

// One wave per query: visit the cells around q nearest-shell first (every lane the same
// cell), the lanes split each cell's points, f(entry) evaluates them and returns the new
// (wave-uniform) bound.  Stops once the next shell is farther than the bound (squared, with
// a rounding margin); cells farther than the bound are skipped.  The minimum of (d2, order)
// does not depend on the visiting order, so the result is the sequential search's.
template <typename F>
__device__ inline void od_visit(const uint4* tab, float qx, float qy, float qz, float bound, F&& f) {
  const int cx = od_cell(qx), cy = od_cell(qy), cz = od_cell(qz);
  for (int k = 0; k <= 3; ++k) {
    const float shell_gap = (float)(k > 0 ? k - 1 : 0) * OD_CELL;  // cells of shell k are >= this far
    if (k > 0 && shell_gap * shell_gap > bound) break;
    for (int dz = -k; dz <= k; ++dz)
      for (int dy = -k; dy <= k; ++dy)
        for (int dx = -k; dx <= k; ++dx) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != k) continue;
          const int x = cx + dx, y = cy + dy, z = cz + dz;
          if (x < 0 || y < 0 || z < 0 || x > 511 || y > 511 || z > 511) continue;
          if (od_gap2(qx, qy, qz, x, y, z) > bound) continue;
          const uint4 e = od_find(tab, od_key(x, y, z));
          if (e.x != OD_EMPTY && e.z > 0) bound = f(e);
        }
  }
}

// squared distance of the reference's scans (laser_odometry.cpp:319-322): float differences,
// float products and sums, widened to double only for the comparison (same outcome)
__device__ inline float od_scan_d2(const float4& p, const float4& q) {
  const float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
  return dx * dx + dy * dy + dz * dz;
}

// lanes' running minima -> the wave's (every lane ends with it); `later` = larger j wins a
// tie (the backward scan meets larger j first)
__device__ inline OdNear od_merge_lanes(OdNear b, bool later) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float d = __shfl_xor(b.d, o, 64);
    const int j = __shfl_xor(b.j, o, 64);
    const bool take = j >= 0 && (b.j < 0 || d < b.d || (d == b.d && (later ? j > b.j : j < b.j)));
    if (take) {
      b.d = d;
      b.j = j;
    }
  }
  return b;
}

// The second (corner) / second and third (surf) points: the reference's forward scan
// j = cl+1 .. n-1 and backward scan j = cl-1 .. 0 over the last cloud in its own order.
//   corner (:309-355): skip int(I) <= cid (fwd) / >= cid (bwd); stop at int(I) > cid + 2 (fwd)
//                      / < cid - 2 (bwd); nearest under '<' starting from 25
//   surf   (:407-456): stop at int(I) > cid + 2 (fwd) / < cid - 2 (bwd); int(I) <= cid (fwd) /
//                      >= cid (bwd) -> minPointInd2, else -> minPointInd3
// b2 / b3: j = -1 when none (d < 25 never met).
__device__ inline void od_ring_scans(const float4* last, int nl, int cl, int cid, int c, const float4& sel, int lane,
                                     OdNear& b2, OdNear& b3) {
  OdNear f2{OD_THR, 0, -1}, f3{OD_THR, 0, -1};
  for (int j0 = cl + 1; j0 < nl; j0 += 64) {  // forward
    const int j = j0 + lane;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < nl) p = last[j];
    const int r = (int)p.w;
    const uint64_t brk = __ballot(j < nl && r > cid + 2);
    const int stop = brk ? __ffsll((long long)brk) - 1 : 64;
    if (j < nl && lane < stop) {
      const float d = od_scan_d2(p, sel);
      if (c == 0) {
        if (r > cid && d < f2.d) f2 = OdNear{d, 0, j};
      } else if (r <= cid) {
        if (d < f2.d) f2 = OdNear{d, 0, j};
      } else if (d < f3.d) {
        f3 = OdNear{d, 0, j};
      }
    }
    if (brk) break;
  }
  OdNear k2{OD_THR, 0, -1}, k3{OD_THR, 0, -1};
  for (int j0 = cl - 1; j0 >= 0; j0 -= 64) {  // backward
    const int j = j0 - lane;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j >= 0) p = last[j];
    const int r = (int)p.w;
    const uint64_t brk = __ballot(j >= 0 && r < cid - 2);
    const int stop = brk ? __ffsll((long long)brk) - 1 : 64;
    if (j >= 0 && lane < stop) {
      const float d = od_scan_d2(p, sel);
      if (c == 0) {
        if (r < cid && d < k2.d) k2 = OdNear{d, 0, j};
      } else if (r >= cid) {
        if (d < k2.d) k2 = OdNear{d, 0, j};
      } else if (d < k3.d) {
        k3 = OdNear{d, 0, j};
      }
    }
    if (brk) break;
  }
  f2 = od_merge_lanes(f2, false);
  k2 = od_merge_lanes(k2, true);
  b2 = (k2.j >= 0 && (f2.j < 0 || k2.d < f2.d)) ? k2 : f2;
  if (c == 1) {
    f3 = od_merge_lanes(f3, false);
    k3 = od_merge_lanes(k3, true);
    b3 = (k3.j >= 0 && (f3.j < 0 || k3.d < f3.d)) ? k3 : f3;
  } else {
    b3 = OdNear{OD_THR, 0, -1};
  }
}

constexpr int OD_QWAVES = OD_QTHREADS / 64;  // queries in flight per workgroup (one per wave)

__global__ void __launch_bounds__(OD_QTHREADS) k_od_corr(OdomDev D, int round, int qblk) {
  const int s = blockIdx.x / qblk, blk = blockIdx.x % qblk;
  OdomFrame& F = D.fr[s];
  if (!F.active || !F.inited) return;
  // para_q / para_t at the start of the round: the VO prior when coupled (:237-250), else the
  // previous frame's (round 0) or round 0's result (round 1)
  const double* x0 = F.has_prior ? F.prior : F.x;
  double X[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) X[i] = x0[i];
  if (blk == 0 && threadIdx.x < LM_SYNC_WORDS) D.lm_sync[((size_t)s * 2 + round) * LM_SYNC_WORDS + threadIdx.x] = 0;
  if (blk == 0 && threadIdx.x == 0) lm_init(F.lm[round], X, 4, true);
  const int ns = F.n_in[0], nf = F.n_in[2];
  const size_t rb = (size_t)s * OD_MAXQ;
  const size_t cb = (size_t)s * D.cap;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t n_edge = 0, n_plane = 0;
  for (int q = blk * OD_QWAVES + wid; q < ns + nf; q += qblk * OD_QWAVES) {
    const int c = q < ns ? 0 : 1;  // 0: sharp vs cornerLast, 1: flat vs surfLast
    const float4 cp = c == 0 ? F.in_ptr[0][q] : F.in_ptr[2][q - ns];
    const float4 sel = to_map(X, cp);  // TransformToStart, s = 1: same double transform
    const uint4* tab = D.ltab[c] + (size_t)s * OD_TAB;
    const float4* srt = D.lsort[c] + cb;
    const int* sidx = D.lsidx[c] + cb;
    const float4* last = D.last[c] + cb;
    int type = 0;
    double a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
    // 1-NN (FLANN L2_Simple<float>, ties by index)
    OdNear n1{INFINITY, 0xFFFFFFFFu, -1};
    od_visit(tab, sel.x, sel.y, sel.z, OD_THR * 1.01f + 1e-5f, [&](const uint4& e) {
      for (uint32_t k = lane; k < e.z; k += 64) {
        const float4 p = srt[e.y + k];
        const int j = sidx[e.y + k];
        od_offer(n1, fdist2(sel.x, sel.y, sel.z, p.x, p.y, p.z), (uint32_t)j, j);
      }
      n1 = od_wave_min(n1);
      return fminf(n1.d, OD_THR) * 1.01f + 1e-5f;
    });
    if (n1.j >= 0 && n1.d < OD_THR) {
      const int cl = n1.j;
      const int cid = (int)last[cl].w;  // closestPointScanID = int(intensity)
      const int nl = F.n_last[c];
      OdNear b2, b3;
      od_ring_scans(last, nl, cl, cid, c, sel, lane, b2, b3);
      const float4 pa = last[cl];
      if (c == 0 && b2.j >= 0) {
        // LidarEdgeFactor(curr, a = last[cl], b = last[ind2]): r = (lp - a) x e, e = (a - b)/|a - b|
        const float4 pb = last[b2.j];
        const d3 de{(double)pa.x - (double)pb.x, (double)pa.y - (double)pb.y, (double)pa.z - (double)pb.z};
        const double dn = sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
        type = 1;
        a[0] = pa.x; a[1] = pa.y; a[2] = pa.z;
        b[0] = de.x / dn; b[1] = de.y / dn; b[2] = de.z / dn;
        n_edge += lane == 0;
      } else if (c == 1 && b2.j >= 0 && b3.j >= 0) {
        // LidarPlaneFactor ctor (lidarFactor.hpp:73-74): ljm = normalize((j - l) x (j - m))
        const float4 pl = last[b2.j], pm = last[b3.j];
        const d3 jv{(double)pa.x, (double)pa.y, (double)pa.z};
        d3 nv = cross3(d3{jv.x - pl.x, jv.y - pl.y, jv.z - pl.z}, d3{jv.x - pm.x, jv.y - pm.y, jv.z - pm.z});
        const double nn = sqrt(nv.x * nv.x + nv.y * nv.y + nv.z * nv.z);
        if (nn > 0) nv = {nv.x / nn, nv.y / nn, nv.z / nn};
        type = 2;
        a[0] = jv.x; a[1] = jv.y; a[2] = jv.z;
        b[0] = nv.x; b[1] = nv.y; b[2] = nv.z;
        n_plane += lane == 0;
      }
    }
    if (lane == 0) {
      D.r_type[rb + q] = type;
      D.r_px[rb + q] = cp.x;
      D.r_py[rb + q] = cp.y;
      D.r_pz[rb + q] = cp.z;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        D.r_a[k][rb + q] = a[k];
        D.r_b[k][rb + q] = b[k];
      }
    }
  }
  // the workgroup's counts go to its own slot (k_od_lm adds the slots): thousands of atomics on
  // the stream's two counters serialise in the memory system
  __shared__ uint32_t wsum[OD_QWAVES][2];
  uint32_t we = n_edge, wp = n_plane;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    we += __shfl_xor(we, o, 64);
    wp += __shfl_xor(wp, o, 64);
  }
  if (lane == 0) {
    wsum[wid][0] = we;
    wsum[wid][1] = wp;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t t = 0;
    for (int w = 0; w < OD_QWAVES; ++w) t += wsum[w][threadIdx.x];
    D.corr_part[(((size_t)s * 2 + round) * OD_QBLK_MAX + blk) * 2 + threadIdx.x] = (int)t;
  }
}

__global__ void __launch_bounds__(OD_LM_THREADS) k_od_lm(OdomDev D, int round, int G, int qblk) {
  // block b -> stream b % Bp, member b / Bp: a stream's blocks share an XCD (lm.h lm_padded)
  const int Bp = lm_padded(D.B), s = blockIdx.x % Bp, g = blockIdx.x / Bp;
  if (s >= D.B) return;
  OdomFrame& F = D.fr[s];
  if (!F.active || !F.inited) return;
  if (g == 0 && threadIdx.x < 64) {  // the round's correspondence counts (k_od_corr slots)
    const int c = threadIdx.x & 1;
    uint32_t t = 0;
    for (int b = threadIdx.x >> 1; b < qblk; b += 32)
      t += (uint32_t)D.corr_part[(((size_t)s * 2 + round) * OD_QBLK_MAX + b) * 2 + c];
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
    if (threadIdx.x < 2) F.corr[round * 2 + c] = (int)t;
  }
  const size_t rb = (size_t)s * OD_MAXQ;
  LmJob J;
  J.S = &F.lm[round];
  J.R = LmRecView{D.r_type + rb, D.r_px + rb, D.r_py + rb, D.r_pz + rb, D.r_a[0] + rb, D.r_a[1] + rb,
                  D.r_a[2] + rb, D.r_b[0] + rb, D.r_b[1] + rb, D.r_b[2] + rb};
  J.nrec = F.n_in[0] + F.n_in[2];
  J.part = D.partials + (size_t)s * OD_PBLK * LM_NACC;
  J.sync = D.lm_sync + ((size_t)s * 2 + round) * LM_SYNC_WORDS;
  J.xpub = D.lm_xpub + ((size_t)s * 2 + round) * 8;
  J.best_out = F.x;
  J.err = &F.err;
  J.err_code = OD_ERR_LM_SYNC;
  lm_round_device<OD_LM_THREADS>(J, g, G);
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct OdomHost {
  double q_w[4] = {0, 0, 0, 1}, t_w[3] = {0, 0, 0};
  int frame_count = 0;
  bool pending = false;
  bool prior_set = false;  // loam_odometry_set_prior for the next solve
  double prior[7] = {0, 0, 0, 1, 0, 0, 0};
  loam_odom_stats st{};
};

}  // namespace loam

using namespace loam;

struct loam_odometry {
  int dev = 0;
  int B = 0;
  int G = 1;
  loam_params P{};
  OdomDev D{};
  std::vector<OdomFrame> hf;
  OdomFrame* hf_pin = nullptr;  // page-locked staging of hf: the per-solve copies stay DMA copies
  std::vector<OdomHost> hs;
  std::vector<void*> allocs;
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
};

namespace {

template <typename T>
int32_t od_alloc(loam_odometry* h, T** p, size_t n) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  LOAM_HIP(hipMalloc(&q, bytes));
  LOAM_HIP(hipMemsetAsync(q, 0, bytes, h->st));  // on the handle's stream (ordered)
  h->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return LOAM_OK;
}

void od_free(loam_odometry* h) {
  if (h->st) (void)hipStreamSynchronize(h->st);
  if (h->hf_pin) (void)hipHostFree(h->hf_pin);
  h->hf_pin = nullptr;
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->st) (void)hipStreamDestroy(h->st);
}

int32_t od_check(loam_odometry* h, int32_t s) {
  if (!h || s < 0 || s >= h->B) {
    set_error("loam_odometry: bad handle or stream");
    return LOAM_ERR_ARG;
  }
  return LOAM_OK;
}

}  // namespace

extern "C" {

int32_t loam_odometry_create(const loam_params* p, int32_t device, int32_t n_streams, loam_odometry** out) {
  if (!out || n_streams <= 0) {
    set_error("loam_odometry_create: bad arguments");
    return LOAM_ERR_ARG;
  }
  *out = nullptr;
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  auto* h = new loam_odometry;
  if (p) h->P = *p; else loam_params_default(&h->P);
  if (h->P.mapping_skip_frame < 1) h->P.mapping_skip_frame = 1;
  h->dev = device;
  h->B = n_streams;
  auto fail = [&](int32_t r) {
    od_free(h);
    delete h;
    return r;
  };
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) return fail(LOAM_ERR_HIP);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(LOAM_ERR_HIP);
  OdomDev& D = h->D;
  D.B = n_streams;
  D.cap = std::min(h->P.max_input_points, 65535);  // 16-bit ranks in the build
  const size_t B = n_streams, cap = D.cap;
#define OA(ptr, n) \
  if ((rc = od_alloc(h, &(ptr), (n))) != LOAM_OK) return fail(rc)
  OA(D.fr, B);
  for (int k = 0; k < 4; ++k) OA(D.stage[k], B * cap);
  for (int c = 0; c < 2; ++c) {
    OA(D.last[c], B * cap);
    OA(D.lsort[c], B * cap);
    OA(D.lsidx[c], B * cap);
    OA(D.ltab[c], B * (size_t)OD_TAB);
  }
  OA(D.scratch, B * 2 * cap);
  OA(D.r_type, B * (size_t)OD_MAXQ);
  OA(D.r_px, B * (size_t)OD_MAXQ);
  OA(D.r_py, B * (size_t)OD_MAXQ);
  OA(D.r_pz, B * (size_t)OD_MAXQ);
  for (int k = 0; k < 3; ++k) {
    OA(D.r_a[k], B * (size_t)OD_MAXQ);
    OA(D.r_b[k], B * (size_t)OD_MAXQ);
  }
  OA(D.partials, B * (size_t)OD_PBLK * LM_NACC);
  OA(D.corr_part, B * 2 * (size_t)OD_QBLK_MAX * 2);
  OA(D.lm_sync, B * 2 * LM_SYNC_WORDS);
  OA(D.lm_xpub, B * 2 * 8);
#undef OA
  {  // workgroups per stream of the LM round (lm.h: shares are claimed by whichever workgroups
     // run, so residency is a speed matter only): one block per CU (256 VGPRs) when they fit
    int occ = 0, cus = 0;
    h->G = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_od_lm, OD_LM_THREADS, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess)
      h->G = std::max(1, std::min(OD_PBLK, std::min(4, std::min(occ, 1) * cus / n_streams)));
  }
  h->hf.assign(B, OdomFrame{});
  h->hs.assign(B, OdomHost{});
  for (auto& F : h->hf) F.x[3] = 1.0;
  if (hipHostMalloc(reinterpret_cast<void**>(&h->hf_pin), sizeof(OdomFrame) * B, hipHostMallocDefault) != hipSuccess)
    return fail(LOAM_ERR_HIP);
  if (hipStreamSynchronize(h->st) != hipSuccess) return fail(LOAM_ERR_HIP);
  *out = h;
  return LOAM_OK;
}

int32_t loam_odometry_destroy(loam_odometry* h) {
  if (!h) return LOAM_ERR_ARG;
  (void)hipSetDevice(h->dev);
  od_free(h);
  delete h;
  return LOAM_OK;
}

int32_t loam_odometry_reset(loam_odometry* h) {
  if (!h) return LOAM_ERR_ARG;
  for (auto& F : h->hf) {
    F = OdomFrame{};
    F.x[3] = 1.0;
  }
  for (auto& H : h->hs) H = OdomHost{};
  return LOAM_OK;
}

static int32_t od_input(loam_odometry* h, int32_t s, const float* const* clouds, const int32_t* n, bool device) {
  TRY(od_check(h, s));
  for (int k = 0; k < 4; ++k) {
    if (n[k] < 0 || (n[k] > 0 && !clouds[k])) {
      set_error("loam_odometry_input: bad cloud");
      return LOAM_ERR_ARG;
    }
    if (n[k] > h->D.cap) {
      set_error("loam_odometry_input: cloud larger than the capacity");
      return LOAM_ERR_CAPACITY;
    }
  }
  if (n[0] + n[2] > OD_MAXQ) {
    set_error("loam_odometry_input: more sharp + flat points than OD_MAXQ");
    return LOAM_ERR_CAPACITY;
  }
  LOAM_HIP(hipSetDevice(h->dev));
  OdomFrame& F = h->hf[s];
  for (int k = 0; k < 4; ++k) {
    F.n_in[k] = n[k];
    if (device) {
      F.in_ptr[k] = reinterpret_cast<const float4*>(clouds[k]);
    } else {
      float4* dst = h->D.stage[k] + (size_t)s * h->D.cap;
      if (n[k]) LOAM_HIP(hipMemcpyAsync(dst, clouds[k], sizeof(float4) * n[k], hipMemcpyHostToDevice, h->st));
      F.in_ptr[k] = dst;
    }
  }
  F.active = 1;
  h->hs[s].pending = true;
  if (!device) LOAM_HIP(hipStreamSynchronize(h->st));  // caller's host buffers are free after return
  return LOAM_OK;
}

int32_t loam_odometry_input(loam_odometry* h, int32_t s, const float* sharp, int32_t n_sharp,
                            const float* less_sharp, int32_t n_less_sharp, const float* flat, int32_t n_flat,
                            const float* less_flat, int32_t n_less_flat) {
  const float* c[4] = {sharp, less_sharp, flat, less_flat};
  const int32_t n[4] = {n_sharp, n_less_sharp, n_flat, n_less_flat};
  return od_input(h, s, c, n, false);
}

int32_t loam_odometry_input_device(loam_odometry* h, int32_t s, const float* sharp, int32_t n_sharp,
                                   const float* less_sharp, int32_t n_less_sharp, const float* flat,
                                   int32_t n_flat, const float* less_flat, int32_t n_less_flat) {
  const float* c[4] = {sharp, less_sharp, flat, less_flat};
  const int32_t n[4] = {n_sharp, n_less_sharp, n_flat, n_less_flat};
  return od_input(h, s, c, n, true);
}

int32_t loam_odometry_solve(loam_odometry* h) {
  if (!h) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  const int B = h->B;
  bool any = false, any_inited = false;
  for (int s = 0; s < B; ++s) {
    OdomFrame& F = h->hf[s];
    OdomHost& H = h->hs[s];
    if (H.pending && F.inited && !h->P.detach_vo_lo && !H.prior_set) {
      set_error("loam_odometry_solve: detach_vo_lo = 0 needs loam_odometry_set_prior for every stream with an "
                "input (laser_odometry.cpp:237-250)");
      return LOAM_ERR_STATE;
    }
  }
  for (int s = 0; s < B; ++s) {
    OdomFrame& F = h->hf[s];
    OdomHost& H = h->hs[s];
    F.active = H.pending ? 1 : 0;
    F.has_prior = (F.active && H.prior_set) ? 1 : 0;
    for (int i = 0; i < 7; ++i) F.prior[i] = H.prior[i];
    F.err = 0;
    for (int k = 0; k < 4; ++k) F.corr[k] = 0;
    any |= F.active != 0;
    any_inited |= F.active && F.inited;
  }
  if (!any) return LOAM_OK;
  hipStream_t st = h->st;
  OdomDev& D = h->D;
  std::memcpy(h->hf_pin, h->hf.data(), sizeof(OdomFrame) * B);  // the stream is idle (synchronized below)
  LOAM_HIP(hipEventRecord(h->ev[0], st));
  LOAM_HIP(hipMemcpyAsync(D.fr, h->hf_pin, sizeof(OdomFrame) * B, hipMemcpyHostToDevice, st));
  if (any_inited) {
    // one wave per query: enough workgroups per stream for the largest query count
    int maxq = 1;
    for (int s = 0; s < B; ++s)
      if (h->hf[s].active) maxq = std::max(maxq, h->hf[s].n_in[0] + h->hf[s].n_in[2]);
    const int qblk = std::min(OD_QBLK_MAX, (maxq + OD_QWAVES - 1) / OD_QWAVES);
    for (int round = 0; round < 2; ++round) {
      k_od_corr<<<B * qblk, OD_QTHREADS, 0, st>>>(D, round, qblk);
      k_od_lm<<<lm_padded(B) * h->G, OD_LM_THREADS, 0, st>>>(D, round, h->G, qblk);
    }
  }
  k_od_build<<<B * 2, OD_BUILD_THREADS, 0, st>>>(D);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipEventRecord(h->ev[1], st));
  LOAM_HIP(hipMemcpyAsync(h->hf_pin, D.fr, sizeof(OdomFrame) * B, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipStreamSynchronize(st));
  std::memcpy(h->hf.data(), h->hf_pin, sizeof(OdomFrame) * B);
  float ms = 0.f;
  LOAM_HIP(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
  int err = 0;
  for (int s = 0; s < B; ++s) {
    OdomFrame& F = h->hf[s];
    OdomHost& H = h->hs[s];
    if (!F.active) continue;
    err |= F.err;
    loam_odom_stats& S = H.st;
    S = loam_odom_stats{};
    if (F.inited) {
      // laser_odometry.cpp:524-527: t_w += q_w * t_lc ; q_w = q_w * q_lc
      const dq qw{H.q_w[0], H.q_w[1], H.q_w[2], H.q_w[3]};
      const d3 tr = qrot(qw, d3{F.x[4], F.x[5], F.x[6]});
      H.t_w[0] += tr.x;
      H.t_w[1] += tr.y;
      H.t_w[2] += tr.z;
      const dq qn = qmul(qw, dq{F.x[0], F.x[1], F.x[2], F.x[3]});
      H.q_w[0] = qn.x; H.q_w[1] = qn.y; H.q_w[2] = qn.z; H.q_w[3] = qn.w;
      for (int r = 0; r < 2; ++r) {
        S.corner_num[r] = F.corr[2 * r];
        S.surf_num[r] = F.corr[2 * r + 1];
        S.lm[r].iterations = F.lm[r].iteration;
        S.lm[r].successful = F.lm[r].successful;
        S.lm[r].invalid = F.lm[r].invalid;
        S.lm[r].termination = F.lm[r].term;
        S.lm[r].initial_cost = F.lm[r].initial_cost;
        S.lm[r].final_cost = F.lm[r].min_cost;
      }
    }
    F.inited = 1;
    H.frame_count++;
    H.pending = false;
    H.prior_set = false;  // velo_last_VOT_velo_curr is the VO estimate of this frame pair only
    F.active = 0;
    S.n_corner_last = F.n_last[0];
    S.n_surf_last = F.n_last[1];
    S.ms = ms;
  }
  if (err & OD_ERR_LM_SYNC) {
    set_error("loam_odometry_solve: the LM round's workgroup hand-off timed out (lm.h spin bound; flags " +
              std::to_string(err) + ")");
    return LOAM_ERR_SYNC;
  }
  if (err) {
    set_error(std::string("loam_odometry_solve: ") +
              ((err & OD_ERR_TABLE) ? "last-cloud cell table full" : "device capacity exceeded") + " (flags " +
              std::to_string(err) + ")");
    return LOAM_ERR_CAPACITY;
  }
  return LOAM_OK;
}

int32_t loam_odometry_set_prior(loam_odometry* h, int32_t s, const double* q_xyzw, const double* t_xyz) {
  TRY(od_check(h, s));
  if (h->P.detach_vo_lo) {
    set_error("loam_odometry_set_prior: detach_vo_lo = 1 (the reference ignores the VO prior, "
              "laser_odometry.cpp:237)");
    return LOAM_ERR_STATE;
  }
  OdomHost& H = h->hs[s];
  if (!q_xyzw || !t_xyz) {
    H.prior_set = false;
    return LOAM_OK;
  }
  for (int i = 0; i < 4; ++i) H.prior[i] = q_xyzw[i];
  for (int i = 0; i < 3; ++i) H.prior[4 + i] = t_xyz[i];
  H.prior_set = true;
  return LOAM_OK;
}

int32_t loam_odometry_output(loam_odometry* h, int32_t s, double* q_w, double* t_w, double* q_lc, double* t_lc,
                             int32_t* skip_frame) {
  TRY(od_check(h, s));
  const OdomHost& H = h->hs[s];
  const OdomFrame& F = h->hf[s];
  if (q_w) for (int i = 0; i < 4; ++i) q_w[i] = H.q_w[i];
  if (t_w) for (int i = 0; i < 3; ++i) t_w[i] = H.t_w[i];
  if (q_lc) for (int i = 0; i < 4; ++i) q_lc[i] = F.x[i];
  if (t_lc) for (int i = 0; i < 3; ++i) t_lc[i] = F.x[4 + i];
  // laser_odometry.cpp:668-678
  if (skip_frame) *skip_frame = (H.frame_count % h->P.mapping_skip_frame == 0) ? 0 : 1;
  return LOAM_OK;
}

int32_t loam_odometry_last_cloud(loam_odometry* h, int32_t s, int32_t which, const float** d_ptr) {
  TRY(od_check(h, s));
  if (which < 0 || which > 1 || !d_ptr) return LOAM_ERR_ARG;
  *d_ptr = reinterpret_cast<const float*>(h->D.last[which] + (size_t)s * h->D.cap);
  return h->hf[s].n_last[which];
}

int32_t loam_odometry_copy_last(loam_odometry* h, int32_t s, int32_t which, float* out, int32_t cap) {
  const float* p = nullptr;
  const int32_t n = loam_odometry_last_cloud(h, s, which, &p);
  if (n < 0) return n;
  if (!out || cap < n) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  if (n) LOAM_HIP(hipMemcpy(out, p, sizeof(float4) * n, hipMemcpyDeviceToHost));
  return n;
}

int32_t loam_odometry_stats(loam_odometry* h, int32_t s, loam_odom_stats* st) {
  TRY(od_check(h, s));
  if (!st) return LOAM_ERR_ARG;
  *st = h->hs[s].st;
  return LOAM_OK;
}

}  // extern "C"
