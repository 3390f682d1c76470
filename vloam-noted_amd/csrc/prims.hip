// prims.hip — standalone entry points of the kernels behind the stages (include/loam_core.h):
// the device LM engine on an explicit factor list, the VoxelGrid workgroup routine on one
// cloud, and the radius-bounded kNN over the 1 m cell hash.  They share the kernels' code
// with the stage pipelines and exist so that each kernel can be parity-tested on its own.
#include <cmath>
#include <vector>

#include "cellhash.h"
#include "common.h"
#include "lm.h"
#include "voxel.h"
#include "voxel_hot.h"
#include "voxel_pcl.h"

namespace loam {

constexpr int P_LM_THREADS = 256;
constexpr int P_LM_PER_THREAD = 4;
constexpr int P_LM_CHUNK = P_LM_THREADS * P_LM_PER_THREAD;

struct LmRecDev {
  int* type;
  float *px, *py, *pz;
  double *a0, *a1, *a2, *b0, *b1, *b2;
};

__global__ void __launch_bounds__(P_LM_THREADS) k_lm_eval_single(LmRecDev R, int nrec, const LmState* S,
                                                                 double* partials) {
  const LmRecView V{R.type, R.px, R.py, R.pz, R.a0, R.a1, R.a2, R.b0, R.b1, R.b2};
  lm_eval_block<P_LM_THREADS>(V, nrec, *S, blockIdx.x, gridDim.x, partials + (size_t)blockIdx.x * LM_NACC);
}

__global__ void __launch_bounds__(64) k_lm_step_single(const double* partials, int nblk, LmState* S) {
  lm_step_wave(partials, nblk, *S);
}

// one evaluation at x: partial sums per workgroup (no state machine)
__global__ void __launch_bounds__(P_LM_THREADS)
    k_lm_eval(LmRecDev R, int nrec, const double* x, double* partials) {
  __shared__ double red[P_LM_THREADS / 64][LM_NACC];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  double X[7], Rm[9];
  for (int i = 0; i < 7; ++i) X[i] = x[i];
  lm_rotmat(X, Rm);
  double acc[LM_NACC];
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) acc[i] = 0.0;
  for (int it = 0; it < P_LM_PER_THREAD; ++it) {
    const int r = blockIdx.x * P_LM_CHUNK + it * P_LM_THREADS + tid;
    if (r < nrec && R.type[r] != 0)
      lm_accum(R.type[r], R.px[r], R.py[r], R.pz[r], R.a0[r], R.a1[r], R.a2[r], R.b0[r], R.b1[r],
               R.b2[r], Rm, X, acc);
  }
#pragma unroll
  for (int i = 0; i < LM_NACC; ++i) {
    double v = wave_sum_d(acc[i]);
    if (lane == 0) red[wid][i] = v;
  }
  __syncthreads();
  if (tid < LM_NACC) {
    double v = 0.0;
    for (int w = 0; w < P_LM_THREADS / 64; ++w) v += red[w][tid];
    partials[(size_t)blockIdx.x * LM_NACC + tid] = v;
  }
}

__global__ void __launch_bounds__(VX_THREADS) k_voxel_one(VoxSeg S) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  voxel_segment(S, lds);
}

// re-VoxelGrid of fixed-point content + new points (the map update path); *merged = 1 if the
// merge path ran, 0 if it fell back to the full filter
// PCL-order VoxelGrid (voxel_pcl.h) of one cloud in global scratch (any size)
constexpr int P_PCL_THREADS = 1024;
inline int ss_cap(int n) { return n / (SS_THRESHOLD + 1) + 2; }
__global__ void __launch_bounds__(P_PCL_THREADS) k_voxel_pcl_one(const float4* src, int n, float leaf, float4* out,
                                                                 uint32_t* out_n, uint64_t* E, uint32_t* A,
                                                                 uint32_t* B, uint64_t* S, int* seg, int cap,
                                                                 int* err) {
  __shared__ SsLevels lev;
  __shared__ VxMisc M;
  __shared__ uint32_t ws[P_PCL_THREADS / 64 + 1];
  const VxPclScratch X{E, A, B, S, &lev, {seg, seg + 3 * cap}, cap};
  VxPclOut O;
  O.out = out;
  O.res_cnt = out_n;
  voxel_grid_pcl<P_PCL_THREADS>(VxPtrSrc{src}, n, leaf, O, X, M, ws, err);
}

// PCL-order VoxelGrid of one cloud of at most VH_MAX_N points the way the mapper runs it
// (exact_voxel_order): the input-order filter for the voxels of at most 2 members, the pruned
// std::sort emulation for the others (voxel_hot.h)
__global__ void __launch_bounds__(VX_THREADS) k_voxel_hot_one(VoxSeg S, int* err) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  voxel_segment(S, lds);
  vh_fixup<VX_THREADS>(VxSrc{S.src0, S.n0, nullptr}, S.n0, S.out, S.hot, lds, VX_LDS_WORDS - 256,
                       *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192), nullptr, err);
}

struct PKeyLess {
  static constexpr int free_run = 1;  // the permutation itself: every tie order is visible
  __device__ bool operator()(uint64_t a, uint64_t b) const { return (uint32_t)(a >> 32) < (uint32_t)(b >> 32); }
};

// std::sort permutation of (keys[i], i) by key (stdsort.h), NT threads cooperating
__global__ void __launch_bounds__(P_PCL_THREADS) k_sort_perm(const uint32_t* keys, int n, int32_t* perm, uint64_t* E,
                                                             uint32_t* A, uint32_t* B, uint64_t* S, int* seg, int cap,
                                                             int nwaves, int* err) {
  __shared__ SsLevels lev;
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += P_PCL_THREADS) E[i] = ((uint64_t)keys[i] << 32) | (uint32_t)i;
  if (tid == 0) ss_levels_init(&lev, n, seg, seg + 3 * cap, cap);
  const PKeyLess less;
  ss_levels<true, P_PCL_THREADS>(E, A, B, &lev, tid >> 6, nwaves, less, seg, seg + 3 * cap, nullptr);
  __syncthreads();
  if (tid == 0 && lev.err) err[0] = lev.err;
  ss_final(E, A, B, n, S, tid, P_PCL_THREADS, less);
  __syncthreads();
  for (int i = tid; i < n; i += P_PCL_THREADS) perm[i] = (int32_t)(uint32_t)S[i];
}

__global__ void __launch_bounds__(VX_THREADS) k_voxel_merge(VoxSeg S, int* merged) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  if (S.n1 > 0 && (uint32_t)S.n1 <= VX_MERGE_CAP && S.n0 > 0 && vx_merge_fixed_point(S, lds)) {
    if (threadIdx.x == 0) *merged = 1;
    return;
  }
  __syncthreads();
  if (threadIdx.x == 0) *merged = 0;
  voxel_segment(S, lds);
}

// standalone cell hash (one point set)
__global__ void k_hash_insert(const float4* pts, int n, const int* origin, unsigned long long* hk,
                              unsigned long long* hc, uint32_t mask, uint32_t epoch, uint32_t* ps,
                              uint32_t* pr, int* err) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float4 p = pts[i];
    uint32_t slot, rank;
    if (!hash_claim_rank(hk, hc, mask, epoch, cell_key_rel(p.x, p.y, p.z, origin), &slot, &rank)) {
      atomicOr(err, 1);
      pr[i] = 0xFFFFFFFFu;
      continue;
    }
    ps[i] = slot;
    pr[i] = rank;
  }
}

__global__ void k_hash_alloc(int n, const unsigned long long* hk, const unsigned long long* hc,
                             uint32_t epoch, uint32_t* hs, uint4* qt, const uint32_t* ps,
                             const uint32_t* pr, uint32_t* cursor) {
  for (int b0 = blockIdx.x * blockDim.x; b0 < n; b0 += gridDim.x * blockDim.x) {  // whole waves
    const int i = b0 + threadIdx.x;
    const bool first = i < n && pr[i] == 0;
    hash_alloc_cell(first, first ? ps[i] : 0u, hk, hc, epoch, hs, qt, cursor);
  }
}

__global__ void k_hash_scatter(const float4* pts, int n, const uint32_t* hs, const uint32_t* ps,
                               const uint32_t* pr, float4* sp) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (pr[i] == 0xFFFFFFFFu) continue;
    const float4 p = pts[i];
    sp[hs[ps[i]] + pr[i]] = make_float4(p.x, p.y, p.z, __int_as_float(i));
  }
}

__global__ void k_knn_query(const float4* q, int nq, int k, float radius2, const int* origin,
                            const uint4* qt, const float4* sp, uint32_t mask, uint32_t epoch,
                            int* idx, float* d2) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += gridDim.x * blockDim.x) {
    Top5 T;
    knn5_hash(q[i], origin, qt, sp, mask, epoch, radius2, T);
    for (int j = 0; j < k; ++j) {
      const bool ok = T.d[j] < radius2;
      idx[(size_t)i * k + j] = ok ? T.id[j] : -1;
      d2[(size_t)i * k + j] = ok ? T.d[j] : INFINITY;
    }
  }
}

// host helpers
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

template <typename T>
hipError_t dmalloc(DevBuf& b, size_t n) {
  hipError_t e = hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(T));
  if (e == hipSuccess) e = hipMemset(b.p, 0, std::max<size_t>(n, 1) * sizeof(T));
  return e;
}

struct LmHostRecs {
  DevBuf type, px, py, pz, a0, a1, a2, b0, b1, b2;
  LmRecDev view() {
    return LmRecDev{(int*)type.p, (float*)px.p, (float*)py.p, (float*)pz.p, (double*)a0.p,
                    (double*)a1.p, (double*)a2.p, (double*)b0.p, (double*)b1.p, (double*)b2.p};
  }
};

// factor rows (10 doubles) -> device SoA records (edge: a, unit (a-b)/|a-b|)
int32_t upload_factors(const double* f, int n, LmHostRecs& R) {
  std::vector<int> type(n);
  std::vector<float> px(n), py(n), pz(n);
  std::vector<double> A[3], Bv[3];
  for (int k = 0; k < 3; ++k) {
    A[k].resize(n);
    Bv[k].resize(n);
  }
  for (int i = 0; i < n; ++i) {
    const double* r = f + (size_t)i * 10;
    type[i] = (int)r[0];
    px[i] = (float)r[1];
    py[i] = (float)r[2];
    pz[i] = (float)r[3];
    if (type[i] == 1) {
      double de[3] = {r[4] - r[7], r[5] - r[8], r[6] - r[9]};
      double dn = std::sqrt(de[0] * de[0] + de[1] * de[1] + de[2] * de[2]);
      for (int k = 0; k < 3; ++k) {
        A[k][i] = r[4 + k];
        Bv[k][i] = de[k] / dn;
      }
    } else {
      for (int k = 0; k < 3; ++k) {
        A[k][i] = r[4 + k];
        Bv[k][i] = r[7 + k];
      }
    }
  }
  LOAM_HIP(dmalloc<int>(R.type, n));
  LOAM_HIP(dmalloc<float>(R.px, n));
  LOAM_HIP(dmalloc<float>(R.py, n));
  LOAM_HIP(dmalloc<float>(R.pz, n));
  LOAM_HIP(dmalloc<double>(R.a0, n));
  LOAM_HIP(dmalloc<double>(R.a1, n));
  LOAM_HIP(dmalloc<double>(R.a2, n));
  LOAM_HIP(dmalloc<double>(R.b0, n));
  LOAM_HIP(dmalloc<double>(R.b1, n));
  LOAM_HIP(dmalloc<double>(R.b2, n));
  if (n) {
    LOAM_HIP(hipMemcpy(R.type.p, type.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.px.p, px.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.py.p, py.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.pz.p, pz.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.a0.p, A[0].data(), sizeof(double) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.a1.p, A[1].data(), sizeof(double) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.a2.p, A[2].data(), sizeof(double) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.b0.p, Bv[0].data(), sizeof(double) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.b1.p, Bv[1].data(), sizeof(double) * n, hipMemcpyHostToDevice));
    LOAM_HIP(hipMemcpy(R.b2.p, Bv[2].data(), sizeof(double) * n, hipMemcpyHostToDevice));
  }
  return LOAM_OK;
}

}  // namespace loam

using namespace loam;

extern "C" {

int32_t loam_lm_solve(int32_t device, const double* factors, int32_t n, double* x, int32_t max_it,
                      loam_lm_stats* st) {
  if (n < 0 || !x || (n > 0 && !factors) || max_it < 0) {
    set_error("loam_lm_solve: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  LmHostRecs R;
  rc = upload_factors(factors, n, R);
  if (rc != LOAM_OK) return rc;
  const int nblk = 32;
  LmState hS;
  lm_init(hS, x, max_it, true);
  DevBuf dS, dpart;
  LOAM_HIP(dmalloc<LmState>(dS, 1));
  LOAM_HIP(dmalloc<double>(dpart, (size_t)nblk * LM_NACC));
  LOAM_HIP(hipMemcpy(dS.p, &hS, sizeof(LmState), hipMemcpyHostToDevice));
  for (int it = 0; it <= max_it; ++it) {
    k_lm_eval_single<<<nblk, P_LM_THREADS>>>(R.view(), n, (const LmState*)dS.p, (double*)dpart.p);
    k_lm_step_single<<<1, 64>>>((const double*)dpart.p, nblk, (LmState*)dS.p);
  }
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipMemcpy(&hS, dS.p, sizeof(LmState), hipMemcpyDeviceToHost));
  if (hS.status != LM_DONE) {
    set_error("loam_lm_solve: state machine did not terminate");
    return LOAM_ERR_STATE;
  }
  for (int i = 0; i < 7; ++i) x[i] = hS.best[i];
  if (st) {
    st->iterations = hS.iteration;
    st->successful = hS.successful;
    st->invalid = hS.invalid;
    st->termination = hS.term;
    st->initial_cost = hS.initial_cost;
    st->final_cost = hS.min_cost;
  }
  return LOAM_OK;
}

int32_t loam_lm_normal_equations(int32_t device, const double* factors, int32_t n, const double* x,
                                 double* cost, double* jtj, double* jtr) {
  if (n < 0 || !x || !cost || !jtj || !jtr || (n > 0 && !factors)) {
    set_error("loam_lm_normal_equations: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  LmHostRecs R;
  rc = upload_factors(factors, n, R);
  if (rc != LOAM_OK) return rc;
  const int nchunks = std::max(1, (n + P_LM_CHUNK - 1) / P_LM_CHUNK);
  DevBuf dx, dpart;
  LOAM_HIP(dmalloc<double>(dx, 7));
  LOAM_HIP(dmalloc<double>(dpart, (size_t)nchunks * LM_NACC));
  LOAM_HIP(hipMemcpy(dx.p, x, sizeof(double) * 7, hipMemcpyHostToDevice));
  k_lm_eval<<<nchunks, P_LM_THREADS>>>(R.view(), n, (const double*)dx.p, (double*)dpart.p);
  LOAM_HIP(hipGetLastError());
  std::vector<double> part((size_t)nchunks * LM_NACC);
  LOAM_HIP(hipMemcpy(part.data(), dpart.p, sizeof(double) * part.size(), hipMemcpyDeviceToHost));
  double red[LM_NACC] = {0};
  for (int c = 0; c < nchunks; ++c)
    for (int i = 0; i < LM_NACC; ++i) red[i] += part[(size_t)c * LM_NACC + i];
  *cost = red[27];
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c) jtj[r * 6 + c] = red[ut_index(r < c ? r : c, r < c ? c : r)];
  for (int i = 0; i < 6; ++i) jtr[i] = red[21 + i];
  return (int32_t)red[28];
}

int32_t loam_voxel_grid(int32_t device, const float* in, int32_t n, float leaf, float* out, int32_t* n_out) {
  if (n < 0 || (n > 0 && (!in || !out)) || !n_out || !(leaf > 0.f)) {
    set_error("loam_voxel_grid: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  DevBuf din, dout, dsp, dsi, dcnt, derr;
  LOAM_HIP(dmalloc<float4>(din, n));
  LOAM_HIP(dmalloc<float4>(dout, n));
  LOAM_HIP(dmalloc<float4>(dsp, n));
  LOAM_HIP(dmalloc<int>(dsi, n));
  LOAM_HIP(dmalloc<uint32_t>(dcnt, 1));
  LOAM_HIP(dmalloc<int>(derr, 1));
  if (n) LOAM_HIP(hipMemcpy(din.p, in, sizeof(float4) * n, hipMemcpyHostToDevice));
  VoxSeg S{};
  S.src0 = (const float4*)din.p;
  S.n0 = n;
  S.leaf = leaf;
  S.out = (float4*)dout.p;
  S.cap = (uint32_t)n;
  S.res_cnt = (uint32_t*)dcnt.p;
  S.scratch_pts = (float4*)dsp.p;
  S.scratch_idx = (int*)dsi.p;
  S.scratch_cap = (uint32_t)n;
  S.err = (int*)derr.p;
  k_voxel_one<<<1, VX_THREADS>>>(S);
  LOAM_HIP(hipGetLastError());
  uint32_t cnt = 0;
  int err = 0;
  LOAM_HIP(hipMemcpy(&cnt, dcnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    set_error("loam_voxel_grid: more unique voxels than the LDS capacity");
    return LOAM_ERR_CAPACITY;
  }
  if (cnt) LOAM_HIP(hipMemcpy(out, dout.p, sizeof(float4) * cnt, hipMemcpyDeviceToHost));
  *n_out = (int32_t)cnt;
  return LOAM_OK;
}

int32_t loam_voxel_grid_pcl(int32_t device, const float* in, int32_t n, float leaf, float* out, int32_t* n_out) {
  if (n < 0 || (n > 0 && (!in || !out)) || !n_out || !(leaf > 0.f)) {
    set_error("loam_voxel_grid_pcl: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  vh_spin_limit_from_env(device);
  if (n <= VH_MAX_N) {
    DevBuf din, dout, drk, dhl, dhv, dfp, didx, dcnt, derr;
    const size_t m = std::max(n, 1);
    LOAM_HIP(dmalloc<float4>(din, m));
    LOAM_HIP(dmalloc<float4>(dout, m));
    LOAM_HIP(dmalloc<uint32_t>(drk, m));
    LOAM_HIP(dmalloc<uint32_t>(dhl, m));
    LOAM_HIP(dmalloc<uint32_t>(dhv, m + 3));
    LOAM_HIP(dmalloc<uint32_t>(dfp, m));
    LOAM_HIP(dmalloc<int>(didx, m));
    LOAM_HIP(dmalloc<uint32_t>(dcnt, 1));
    LOAM_HIP(dmalloc<int>(derr, 1));
    LOAM_HIP(hipMemset(dcnt.p, 0, sizeof(uint32_t)));
    LOAM_HIP(hipMemset(derr.p, 0, sizeof(int)));
    if (n) LOAM_HIP(hipMemcpy(din.p, in, sizeof(float4) * n, hipMemcpyHostToDevice));
    VoxSeg S{};
    S.src0 = (const float4*)din.p;
    S.n0 = n;
    S.leaf = leaf;
    S.out = (float4*)dout.p;
    S.cap = (uint32_t)m;
    S.res_cnt = (uint32_t*)dcnt.p;
    S.scratch_idx = (int*)didx.p;
    S.scratch_cap = (uint32_t)m;
    S.err = (int*)derr.p;
    S.hot.rk = (uint32_t*)drk.p;
    S.hot.hl = (uint32_t*)dhl.p;
    S.hot.hv = (uint32_t*)dhv.p;
    S.hot.fpos = (uint32_t*)dfp.p;
    S.hot.cap_h = (uint32_t)(n / 3 + 1);
    k_voxel_hot_one<<<1, VX_THREADS>>>(S, (int*)derr.p);
    LOAM_HIP(hipGetLastError());
    uint32_t cnt = 0;
    int err = 0;
    LOAM_HIP(hipMemcpy(&cnt, dcnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
    LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
    if (err & VH_ERR_SPIN) {
      set_error("loam_voxel_grid_pcl: sort: a wave's wait for a listed subtree ran out (err " + std::to_string(err) + ")");
      return LOAM_ERR_SYNC;
    }
    if (err) {
      set_error("loam_voxel_grid_pcl: capacity (unique voxels or sort lists)");
      return LOAM_ERR_CAPACITY;
    }
    if (cnt) LOAM_HIP(hipMemcpy(out, dout.p, sizeof(float4) * cnt, hipMemcpyDeviceToHost));
    *n_out = (int32_t)cnt;
    return LOAM_OK;
  }
  DevBuf din, dout, de, da, db, ds, dseg, dcnt, derr;
  const int cap = ss_cap(n);
  LOAM_HIP(dmalloc<int>(dseg, 6 * (size_t)cap));
  LOAM_HIP(dmalloc<float4>(din, n));
  LOAM_HIP(dmalloc<float4>(dout, n));
  LOAM_HIP(dmalloc<uint64_t>(de, n));
  LOAM_HIP(dmalloc<uint32_t>(da, n));
  LOAM_HIP(dmalloc<uint32_t>(db, n));
  LOAM_HIP(dmalloc<uint64_t>(ds, n));
  LOAM_HIP(dmalloc<uint32_t>(dcnt, 1));
  LOAM_HIP(dmalloc<int>(derr, 1));
  if (n) LOAM_HIP(hipMemcpy(din.p, in, sizeof(float4) * n, hipMemcpyHostToDevice));
  k_voxel_pcl_one<<<1, P_PCL_THREADS>>>((const float4*)din.p, n, leaf, (float4*)dout.p, (uint32_t*)dcnt.p,
                                        (uint64_t*)de.p, (uint32_t*)da.p, (uint32_t*)db.p, (uint64_t*)ds.p,
                                        (int*)dseg.p, cap, (int*)derr.p);
  LOAM_HIP(hipGetLastError());
  uint32_t cnt = 0;
  int err = 0;
  LOAM_HIP(hipMemcpy(&cnt, dcnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    set_error("loam_voxel_grid_pcl: std::sort emulation level list overflow");
    return LOAM_ERR_CAPACITY;
  }
  if (cnt) LOAM_HIP(hipMemcpy(out, dout.p, sizeof(float4) * cnt, hipMemcpyDeviceToHost));
  *n_out = (int32_t)cnt;
  return LOAM_OK;
}

int32_t loam_sort_perm(int32_t device, const uint32_t* keys, int32_t n, int32_t n_waves, int32_t* perm) {
  if (n < 0 || (n > 0 && (!keys || !perm)) || n_waves < 1 || n_waves > P_PCL_THREADS / 64) {
    set_error("loam_sort_perm: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  if (n == 0) return LOAM_OK;
  DevBuf dk, dp, de, da, db, ds, dseg, derr;
  const int cap = ss_cap(n);
  LOAM_HIP(dmalloc<int>(dseg, 6 * (size_t)cap));
  LOAM_HIP(dmalloc<uint32_t>(dk, n));
  LOAM_HIP(dmalloc<int32_t>(dp, n));
  LOAM_HIP(dmalloc<uint64_t>(de, n));
  LOAM_HIP(dmalloc<uint32_t>(da, n));
  LOAM_HIP(dmalloc<uint32_t>(db, n));
  LOAM_HIP(dmalloc<uint64_t>(ds, n));
  LOAM_HIP(dmalloc<int>(derr, 1));
  LOAM_HIP(hipMemcpy(dk.p, keys, sizeof(uint32_t) * n, hipMemcpyHostToDevice));
  k_sort_perm<<<1, P_PCL_THREADS>>>((const uint32_t*)dk.p, n, (int32_t*)dp.p, (uint64_t*)de.p, (uint32_t*)da.p,
                                    (uint32_t*)db.p, (uint64_t*)ds.p, (int*)dseg.p, cap, n_waves, (int*)derr.p);
  LOAM_HIP(hipGetLastError());
  int err = 0;
  LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    set_error("loam_sort_perm: std::sort emulation level list overflow");
    return LOAM_ERR_CAPACITY;
  }
  LOAM_HIP(hipMemcpy(perm, dp.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  return LOAM_OK;
}

int32_t loam_voxel_merge(int32_t device, const float* fixed, int32_t n0, const float* added, int32_t n1,
                         float leaf, float* out, int32_t* n_out, int32_t* merged) {
  if (n0 < 0 || n1 < 0 || (n0 > 0 && !fixed) || (n1 > 0 && !added) || !out || !n_out || !(leaf > 0.f)) {
    set_error("loam_voxel_merge: bad arguments");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  const int32_t n = n0 + n1;
  DevBuf dc, da, dout, dsp, dsi, doff, dcnt, derr, dm;
  LOAM_HIP(dmalloc<float4>(dc, n0));
  LOAM_HIP(dmalloc<float4>(da, n1));
  LOAM_HIP(dmalloc<float4>(dout, n));
  LOAM_HIP(dmalloc<float4>(dsp, n));
  LOAM_HIP(dmalloc<int>(dsi, n));
  LOAM_HIP(dmalloc<uint32_t>(doff, 1));
  LOAM_HIP(dmalloc<uint32_t>(dcnt, 1));
  LOAM_HIP(dmalloc<int>(derr, 1));
  LOAM_HIP(dmalloc<int>(dm, 1));
  if (n0) LOAM_HIP(hipMemcpy(dc.p, fixed, sizeof(float4) * n0, hipMemcpyHostToDevice));
  if (n1) LOAM_HIP(hipMemcpy(da.p, added, sizeof(float4) * n1, hipMemcpyHostToDevice));
  VoxSeg S{};
  S.src0 = (const float4*)dc.p;
  S.n0 = n0;
  S.src1 = (const float4*)da.p;
  S.tag1 = nullptr;
  S.n1 = n1;
  S.leaf = leaf;
  S.out = (float4*)dout.p;
  S.cap = (uint32_t)n;
  S.res_off = (uint32_t*)doff.p;
  S.res_cnt = (uint32_t*)dcnt.p;
  S.scratch_pts = (float4*)dsp.p;
  S.scratch_idx = (int*)dsi.p;
  S.scratch_cap = (uint32_t)n;
  S.err = (int*)derr.p;
  k_voxel_merge<<<1, VX_THREADS>>>(S, (int*)dm.p);
  LOAM_HIP(hipGetLastError());
  uint32_t off = 0, cnt = 0;
  int err = 0, m = 0;
  LOAM_HIP(hipMemcpy(&off, doff.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(&cnt, dcnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(&m, dm.p, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    set_error("loam_voxel_merge: capacity");
    return LOAM_ERR_CAPACITY;
  }
  if (cnt) LOAM_HIP(hipMemcpy(out, (float4*)dout.p + off, sizeof(float4) * cnt, hipMemcpyDeviceToHost));
  *n_out = (int32_t)cnt;
  if (merged) *merged = m;
  return LOAM_OK;
}

int32_t loam_knn_radius(int32_t device, const float* pts, int32_t n, const float* queries, int32_t nq,
                        int32_t k, float radius2, int32_t* idx, float* d2) {
  if (n < 0 || nq < 0 || k < 1 || k > 5 || !(radius2 > 0.f) || radius2 > 1.0f ||
      (n > 0 && !pts) || (nq > 0 && (!queries || !idx || !d2))) {
    set_error("loam_knn_radius: bad arguments (k in 1..5, 0 < radius2 <= 1)");
    return LOAM_ERR_ARG;
  }
  int32_t rc = ensure_device(device);
  if (rc != LOAM_OK) return rc;
  LOAM_HIP(hipSetDevice(device));
  // origin: 2-cell margin below the bounding box of points and queries; 9-bit cells
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], pts[i * 4 + a]);
      mx[a] = std::max(mx[a], pts[i * 4 + a]);
    }
  int origin[3];
  for (int a = 0; a < 3; ++a) {
    origin[a] = n ? (int)std::floor(mn[a]) - 2 : 0;
    if (n && std::floor(mx[a]) - origin[a] > 509) {
      set_error("loam_knn_radius: point cloud spans more than 509 m");
      return LOAM_ERR_ARG;
    }
  }
  uint32_t T = 1;
  while (T < (uint32_t)std::max(2 * n, 64)) T <<= 1;
  DevBuf dp, dq, dorig, dhk, dhc, dhs, dqt, dps, dpr, dsp, dcur, derr, didx, dd2;
  LOAM_HIP(dmalloc<float4>(dp, n));
  LOAM_HIP(dmalloc<float4>(dq, nq));
  LOAM_HIP(dmalloc<int>(dorig, 3));
  LOAM_HIP(dmalloc<unsigned long long>(dhk, T));
  LOAM_HIP(dmalloc<unsigned long long>(dhc, T));
  LOAM_HIP(dmalloc<uint32_t>(dhs, T));
  LOAM_HIP(dmalloc<uint4>(dqt, T));
  LOAM_HIP(dmalloc<uint32_t>(dps, n));
  LOAM_HIP(dmalloc<uint32_t>(dpr, n));
  LOAM_HIP(dmalloc<float4>(dsp, n));
  LOAM_HIP(dmalloc<uint32_t>(dcur, 1));
  LOAM_HIP(dmalloc<int>(derr, 1));
  LOAM_HIP(dmalloc<int>(didx, (size_t)nq * k));
  LOAM_HIP(dmalloc<float>(dd2, (size_t)nq * k));
  if (n) LOAM_HIP(hipMemcpy(dp.p, pts, sizeof(float4) * n, hipMemcpyHostToDevice));
  if (nq) LOAM_HIP(hipMemcpy(dq.p, queries, sizeof(float4) * nq, hipMemcpyHostToDevice));
  LOAM_HIP(hipMemcpy(dorig.p, origin, sizeof(origin), hipMemcpyHostToDevice));
  const uint32_t epoch = 1;
  const int blocks = 256;
  k_hash_insert<<<blocks, 256>>>((const float4*)dp.p, n, (const int*)dorig.p, (unsigned long long*)dhk.p,
                                 (unsigned long long*)dhc.p, T - 1, epoch, (uint32_t*)dps.p,
                                 (uint32_t*)dpr.p, (int*)derr.p);
  k_hash_alloc<<<blocks, 256>>>(n, (const unsigned long long*)dhk.p, (const unsigned long long*)dhc.p, epoch,
                                (uint32_t*)dhs.p, (uint4*)dqt.p, (const uint32_t*)dps.p,
                                (const uint32_t*)dpr.p, (uint32_t*)dcur.p);
  k_hash_scatter<<<blocks, 256>>>((const float4*)dp.p, n, (const uint32_t*)dhs.p, (const uint32_t*)dps.p,
                                  (const uint32_t*)dpr.p, (float4*)dsp.p);
  k_knn_query<<<blocks, 256>>>((const float4*)dq.p, nq, k, radius2, (const int*)dorig.p,
                               (const uint4*)dqt.p, (const float4*)dsp.p, T - 1, epoch, (int*)didx.p,
                               (float*)dd2.p);
  LOAM_HIP(hipGetLastError());
  if (nq) {
    LOAM_HIP(hipMemcpy(idx, didx.p, sizeof(int) * (size_t)nq * k, hipMemcpyDeviceToHost));
    LOAM_HIP(hipMemcpy(d2, dd2.p, sizeof(float) * (size_t)nq * k, hipMemcpyDeviceToHost));
  }
  int err = 0;
  LOAM_HIP(hipMemcpy(&err, derr.p, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    set_error("loam_knn_radius: hash table full");
    return LOAM_ERR_CAPACITY;
  }
  return LOAM_OK;
}

}  // extern "C"
