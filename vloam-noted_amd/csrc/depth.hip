// depth.hip — visual-odometry depth association on MI355X.
//
// Reference: src/visual_odometry/src/point_cloud_util.cpp (called per frame from
// visual_odometry.cpp:195-214 and per feature match from :371-372):
//   projectPointCloud    :183-219  [x y z 1] * cam_T_velo^T * rect0_T_cam^T * P_rect0^T, keep
//                                  depth > 0.1, (u, v) = (u', v') * (1 / depth)
//   downsamplePointCloud :256-324  5 px buckets: first point, then b += (p - b) / count in input
//                                  order; point_cloud_2d_dnsp filled from the end in (x, y) order
//   queryDepth           :381-487  5 x 5 buckets around (x, y), >= 10 occupied, inverse-distance
//                                  weighted depth of the 3 nearest
// One handle = B independent streams (cameras / frames); one launch sequence per process():
//   k_dp_project  one thread per point: the 3-matrix chain in float (4-term dot products in
//                 k order, no contraction: -ffp-contract=off), front test, bucket histogram
//                 (atomics), per-chunk front counts
//   k_dp_scan     one workgroup per stream: chunk offsets, bucket starts, the dnsp slot of every
//                 occupied bucket (reverse (x, y) rank)
//   k_dp_scatter  point_cloud_2d in input order (chunk offset + wave ballots); bucket member
//                 lists (front rank of each point)
//   k_dp_bucket   one thread per bucket: members in input order, the reference's running
//                 average, bucket arrays + point_cloud_2d_dnsp
// Queries: k_dp_query, one thread per image point.
// Everything is HBM-resident; a frame (126k points) moves ~2 MB: latency-bound at one stream,
// batched streams fill the chip.
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.h"

namespace loam {

constexpr int DP_THREADS = 256;
constexpr int DP_CHUNK = 4 * DP_THREADS;  // points per projection workgroup (contiguous)
constexpr int DP_SCAN_THREADS = 1024;
constexpr int DP_ERR_CAP = 1;

struct DepthFrame {
  const float* xyz;  // input points (stride floats each)
  int n, stride;
  int active;
  int n_front, n_dnsp;
  int err;
};

struct DepthDev {
  int B, cap, W, H, nchunk;  // nchunk: chunks per stream (cap / DP_CHUNK)
  float grid;
  float A[16], Bm[16], C[12];  // cam_T_velo, rect0_T_cam, P_rect0 (row-major)
  DepthFrame* fr;
  float4* tmp;       // [B][cap] (u, v, depth, bucket as float bits or -1)
  int* chunk_cnt;    // [B][nchunk] front points per chunk -> offsets
  float4* p2d;       // [B][cap] point_cloud_2d (u, v, depth)
  int* bcnt;         // [B][W*H] bucket_count
  int* bstart;       // [B][W*H + 1] member list starts
  int* bfill;        // [B][W*H]
  int* bslot;        // [B][W*H] dnsp slot (occupied buckets)
  int* members;      // [B][cap] front rank of each bucketed point, grouped by bucket
  float* bx;         // [B][W*H]
  float* by;
  float* bd;
  float4* dnsp;      // [B][W*H]
};

// r[j] = sum_k v[k] M[j][k] (row vector times M^T), k in order, no contraction
__device__ inline void dp_mul_t(const float* v, const float* M, int rows, float* r) {
  for (int j = 0; j < rows; ++j) {
    float acc = v[0] * M[j * 4 + 0];
    acc = acc + v[1] * M[j * 4 + 1];
    acc = acc + v[2] * M[j * 4 + 2];
    acc = acc + v[3] * M[j * 4 + 3];
    r[j] = acc;
  }
}

__global__ void __launch_bounds__(DP_THREADS) k_dp_project(DepthDev D) {
  __shared__ int wcnt[DP_THREADS / 64];
  const int s = blockIdx.x / D.nchunk, c = blockIdx.x % D.nchunk;
  const DepthFrame& F = D.fr[s];
  if (!F.active || c * DP_CHUNK >= F.n) return;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int WH = D.W * D.H;
  int front = 0;
  for (int r = 0; r < DP_CHUNK / DP_THREADS; ++r) {
    const int i = c * DP_CHUNK + r * DP_THREADS + tid;
    if (i >= F.n) break;
    const float* p = F.xyz + (size_t)i * F.stride;
    const float v0[4] = {p[0], p[1], p[2], 1.0f};
    float v1[4], v2[4], v3[3];
    dp_mul_t(v0, D.A, 4, v1);
    dp_mul_t(v1, D.Bm, 4, v2);
    dp_mul_t(v2, D.C, 3, v3);
    float4 o = make_float4(0.f, 0.f, 0.f, __int_as_float(-2));  // -2: behind (dropped)
    if (v3[2] > 0.1f) {  // :197-198 (0.1 as float, Eigen's scalar type)
      const float inv = 1.0f / v3[2];
      const float u = v3[0] * inv, v = v3[1] * inv;
      // :275-277: static_cast<int>(x / grid_size), truncation toward zero
      const int ix = static_cast<int>(u / D.grid), iy = static_cast<int>(v / D.grid);
      int b = -1;
      if (ix >= 0 && ix < D.W && iy >= 0 && iy < D.H) {
        b = ix * D.H + iy;
        atomicAdd(&D.bcnt[(size_t)s * WH + b], 1);
      }
      o = make_float4(u, v, v3[2], __int_as_float(b));
      ++front;
    }
    D.tmp[(size_t)s * D.cap + i] = o;
  }
  front = (int)wave_sum_u((uint32_t)front);
  if (lane == 0) wcnt[wid] = front;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int w = 0; w < DP_THREADS / 64; ++w) t += wcnt[w];
    D.chunk_cnt[(size_t)s * D.nchunk + c] = t;
  }
}

// exclusive block scan of one value per thread (DP_SCAN_THREADS), total in *total
__device__ inline int dp_block_scan(int v, int* ws, int* total) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int inc = (int)wave_incl_scan_u((uint32_t)v);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < DP_SCAN_THREADS / 64; ++w) {
      const int t = ws[w];
      ws[w] = acc;
      acc += t;
    }
    ws[DP_SCAN_THREADS / 64] = acc;
  }
  __syncthreads();
  const int ex = ws[wid] + inc - v;
  *total = ws[DP_SCAN_THREADS / 64];
  __syncthreads();
  return ex;
}

__global__ void __launch_bounds__(DP_SCAN_THREADS) k_dp_scan(DepthDev D) {
  __shared__ int ws[DP_SCAN_THREADS / 64 + 1];
  const int s = blockIdx.x;
  DepthFrame& F = D.fr[s];
  if (!F.active) return;
  const int tid = threadIdx.x;
  // chunk offsets of point_cloud_2d
  const int nch = (F.n + DP_CHUNK - 1) / DP_CHUNK;
  int* cc = D.chunk_cnt + (size_t)s * D.nchunk;
  int base = 0;
  for (int c0 = 0; c0 < nch; c0 += DP_SCAN_THREADS) {
    const int c = c0 + tid;
    const int v = c < nch ? cc[c] : 0;
    int tot;
    const int ex = dp_block_scan(v, ws, &tot);
    if (c < nch) cc[c] = base + ex;
    base += tot;
  }
  if (tid == 0) F.n_front = base;
  // bucket member starts and the dnsp slots: occupied buckets in (x, y) order get ranks
  // 0.., slot = n_dnsp - 1 - rank (the reference fills from the end, :311-322)
  const int WH = D.W * D.H;
  const int* bc = D.bcnt + (size_t)s * WH;
  int* bs = D.bstart + (size_t)s * (WH + 1);
  int* sl = D.bslot + (size_t)s * WH;
  constexpr int PER = 32;  // consecutive buckets per thread and pass
  int mbase = 0, obase = 0;
  for (int b0 = 0; b0 < WH; b0 += PER * DP_SCAN_THREADS) {
    const int lo = b0 + tid * PER;
    int m = 0, o = 0;
    for (int k = 0; k < PER; ++k)
      if (lo + k < WH) {
        const int v = bc[lo + k];
        m += v;
        o += v > 0;
      }
    int mt, ot;
    int mex = dp_block_scan(m, ws, &mt);
    int oex = dp_block_scan(o, ws, &ot);
    mex += mbase;
    oex += obase;
    for (int k = 0; k < PER; ++k)
      if (lo + k < WH) {
        const int v = bc[lo + k];
        bs[lo + k] = mex;
        sl[lo + k] = v > 0 ? oex : -1;  // rank for now
        mex += v;
        oex += v > 0;
      }
    mbase += mt;
    obase += ot;
  }
  if (tid == 0) {
    bs[WH] = mbase;
    F.n_dnsp = obase;
  }
}

__global__ void __launch_bounds__(DP_THREADS) k_dp_scatter(DepthDev D) {
  __shared__ int wcnt[DP_CHUNK / 64];
  const int s = blockIdx.x / D.nchunk, c = blockIdx.x % D.nchunk;
  const DepthFrame& F = D.fr[s];
  if (!F.active || c * DP_CHUNK >= F.n) return;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int WH = D.W * D.H;
  // front rank within the chunk: element order r * DP_THREADS + tid, waves in order
  float4 o[DP_CHUNK / DP_THREADS];
  bool fr[DP_CHUNK / DP_THREADS];
  uint32_t pre[DP_CHUNK / DP_THREADS];
#pragma unroll
  for (int r = 0; r < DP_CHUNK / DP_THREADS; ++r) {
    const int i = c * DP_CHUNK + r * DP_THREADS + tid;
    fr[r] = false;
    if (i < F.n) {
      o[r] = D.tmp[(size_t)s * D.cap + i];
      fr[r] = __float_as_int(o[r].w) != -2;
    }
    const uint64_t bal = __ballot(fr[r]);
    pre[r] = __popcll(bal & lanemask_lt());
    if (lane == 0) wcnt[r * (DP_THREADS / 64) + wid] = __popcll(bal);
  }
  __syncthreads();
  const int off0 = D.chunk_cnt[(size_t)s * D.nchunk + c];
#pragma unroll
  for (int r = 0; r < DP_CHUNK / DP_THREADS; ++r) {
    if (!fr[r]) continue;
    int off = off0;
    for (int k = 0; k < r * (DP_THREADS / 64) + wid; ++k) off += wcnt[k];
    const int rank = off + (int)pre[r];
    D.p2d[(size_t)s * D.cap + rank] = make_float4(o[r].x, o[r].y, o[r].z, 0.f);
    const int b = __float_as_int(o[r].w);
    if (b >= 0) {
      const int slot = atomicAdd(&D.bfill[(size_t)s * WH + b], 1);
      D.members[(size_t)s * D.cap + D.bstart[(size_t)s * (WH + 1) + b] + slot] = rank;
    }
  }
}

__global__ void __launch_bounds__(DP_THREADS) k_dp_bucket(DepthDev D, int blocks_per_stream) {
  const int s = blockIdx.x / blocks_per_stream, g = blockIdx.x % blocks_per_stream;
  const DepthFrame& F = D.fr[s];
  if (!F.active) return;
  const int WH = D.W * D.H;
  const int b = g * DP_THREADS + threadIdx.x;
  if (b >= WH) return;
  const size_t sb = (size_t)s * WH + b;
  const int m = D.bcnt[sb];
  if (m == 0) return;
  const int* mem = D.members + (size_t)s * D.cap + D.bstart[(size_t)s * (WH + 1) + b];
  const float4* p2d = D.p2d + (size_t)s * D.cap;
  // members in input order: repeatedly the smallest rank above the previous one
  int prev = -1;
  float x = 0.f, y = 0.f, d = 0.f;
  for (int t = 0; t < m; ++t) {
    int next = 0x7FFFFFFF;
    for (int k = 0; k < m; ++k) {
      const int v = mem[k];
      if (v > prev && v < next) next = v;
    }
    prev = next;
    const float4 p = p2d[next];
    if (t == 0) {
      x = p.x;
      y = p.y;
      d = p.z;
    } else {  // :291-296
      const float cnt = (float)t;
      x += (p.x - x) / cnt;
      y += (p.y - y) / cnt;
      d += (p.z - d) / cnt;
    }
  }
  D.bx[sb] = x;
  D.by[sb] = y;
  D.bd[sb] = d;
  const int slot = F.n_dnsp - 1 - D.bslot[sb];
  D.dnsp[(size_t)s * WH + slot] = make_float4(x, y, d, 0.f);
}

// queryDepth (point_cloud_util.cpp:381-487) of nq image points of stream s
__global__ void __launch_bounds__(DP_THREADS) k_dp_query(DepthDev D, const int* q_stream, const float2* xy, int nq,
                                                         int radius, float* depth) {
  const int q = blockIdx.x * DP_THREADS + threadIdx.x;
  if (q >= nq) return;
  const int s = q_stream[q];
  if (s < 0 || s >= D.B) {  // device-side ids are not validated on the host
    depth[q] = -1.0f;
    return;
  }
  const int WH = D.W * D.H;
  const int* bc = D.bcnt + (size_t)s * WH;
  const float *bx = D.bx + (size_t)s * WH, *by = D.by + (size_t)s * WH, *bd = D.bd + (size_t)s * WH;
  const float x = xy[q].x, y = xy[q].y;
  const int ix = static_cast<int>(x / D.grid), iy = static_cast<int>(y / D.grid);
  // the 3 nearest in gather order (a stable sort's first three), and the count
  float nd[3] = {INFINITY, INFINITY, INFINITY}, nz[3] = {0.f, 0.f, 0.f};
  int cnt = 0;
  for (int i = ix - radius; i <= ix + radius; ++i)
    for (int j = iy - radius; j <= iy + radius; ++j) {
      if (!(i >= 0 && i < D.W && j >= 0 && j < D.H)) continue;
      const int b = i * D.H + j;
      if (bc[b] <= 0) continue;
      ++cnt;
      // std::pow(float, int) promotes to double (:407)
      const double dx = (double)(x - bx[b]), dy = (double)(y - by[b]);
      const float dist = (float)sqrt(dx * dx + dy * dy);
      const float z = bd[b];
      if (dist < nd[2]) {
        if (dist < nd[1]) {
          nd[2] = nd[1];
          nz[2] = nz[1];
          if (dist < nd[0]) {
            nd[1] = nd[0];
            nz[1] = nz[0];
            nd[0] = dist;
            nz[0] = z;
          } else {
            nd[1] = dist;
            nz[1] = z;
          }
        } else {
          nd[2] = dist;
          nz[2] = z;
        }
      }
    }
  if (cnt < 10) {
    depth[q] = -1.0f;
    return;
  }
  depth[q] = (nz[0] * nd[1] * nd[2] + nz[1] * nd[0] * nd[2] + nz[2] * nd[0] * nd[1]) /
             (0.0001f + nd[1] * nd[2] + nd[0] * nd[2] + nd[0] * nd[1]);
}

}  // namespace loam

using namespace loam;

struct loam_depth {
  int dev = 0;
  int B = 0;
  loam_depth_params P{};
  DepthDev D{};
  std::vector<DepthFrame> hf;
  std::vector<void*> allocs;
  float4* stage = nullptr;  // [B][cap] host-input staging
  int* d_qs = nullptr;      // query stream ids / points / results (grown on demand)
  float2* d_xy = nullptr;
  float* d_depth = nullptr;
  int q_cap = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  float ms = 0.f;
};

namespace {

template <typename T>
int32_t dp_alloc(loam_depth* h, T** p, size_t n) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  LOAM_HIP(hipMalloc(&q, bytes));
  LOAM_HIP(hipMemsetAsync(q, 0, bytes, h->st));
  h->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return LOAM_OK;
}

void dp_free(loam_depth* h) {
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  if (h->d_qs) (void)hipFree(h->d_qs);
  if (h->d_xy) (void)hipFree(h->d_xy);
  if (h->d_depth) (void)hipFree(h->d_depth);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->st) (void)hipStreamDestroy(h->st);
}

int32_t dp_check(loam_depth* h, int32_t s) {
  if (!h || s < 0 || s >= h->B) {
    set_error("loam_depth: bad handle or stream");
    return LOAM_ERR_ARG;
  }
  return LOAM_OK;
}

int32_t dp_query_cap(loam_depth* h, int n) {
  if (n <= h->q_cap) return LOAM_OK;
  if (h->d_qs) (void)hipFree(h->d_qs);
  if (h->d_xy) (void)hipFree(h->d_xy);
  if (h->d_depth) (void)hipFree(h->d_depth);
  h->d_qs = nullptr;
  h->d_xy = nullptr;
  h->d_depth = nullptr;
  h->q_cap = 0;
  LOAM_HIP(hipMalloc(&h->d_qs, sizeof(int) * n));
  LOAM_HIP(hipMalloc(&h->d_xy, sizeof(float2) * n));
  LOAM_HIP(hipMalloc(&h->d_depth, sizeof(float) * n));
  h->q_cap = n;
  return LOAM_OK;
}

}  // namespace

extern "C" {

void loam_depth_params_default(loam_depth_params* p) {
  if (!p) return;
  *p = loam_depth_params{};
  // PointCloudUtil() (point_cloud_util.h:28-35): matrices zero until the calibration is read;
  // KITTI image size (:49-50), downsample_grid_size 5 (visual_odometry.cpp)
  p->grid = 5;
  p->img_width = 1242;
  p->img_height = 375;
  p->max_points = 262144;
}

int32_t loam_depth_create(const loam_depth_params* p, int32_t device, int32_t n_streams, loam_depth** out) {
  if (!out || !p || n_streams <= 0 || p->grid <= 0 || p->img_width <= 0 || p->img_height <= 0 ||
      p->max_points <= 0) {
    set_error("loam_depth_create: bad arguments");
    return LOAM_ERR_ARG;
  }
  *out = nullptr;
  TRY(ensure_device(device));
  LOAM_HIP(hipSetDevice(device));
  auto* h = new loam_depth;
  h->P = *p;
  h->dev = device;
  h->B = n_streams;
  auto fail = [&](int32_t r) {
    dp_free(h);
    delete h;
    return r;
  };
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) return fail(LOAM_ERR_HIP);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(LOAM_ERR_HIP);
  DepthDev& D = h->D;
  D.B = n_streams;
  D.nchunk = (p->max_points + DP_CHUNK - 1) / DP_CHUNK;
  D.cap = D.nchunk * DP_CHUNK;
  // point_cloud_util.cpp:260-262: std::ceil(float(IMG) / float(grid))
  D.W = (int)std::ceil(static_cast<float>(p->img_width) / static_cast<float>(p->grid));
  D.H = (int)std::ceil(static_cast<float>(p->img_height) / static_cast<float>(p->grid));
  D.grid = (float)p->grid;
  for (int k = 0; k < 16; ++k) {
    D.A[k] = p->cam_T_velo[k];
    D.Bm[k] = p->rect0_T_cam[k];
  }
  for (int k = 0; k < 12; ++k) D.C[k] = p->P_rect0[k];
  const size_t B = n_streams, cap = D.cap, WH = (size_t)D.W * D.H;
  int32_t rc = LOAM_OK;
#define DA(ptr, n) \
  if ((rc = dp_alloc(h, &(ptr), (n))) != LOAM_OK) return fail(rc)
  DA(D.fr, B);
  DA(h->stage, B * cap);
  DA(D.tmp, B * cap);
  DA(D.chunk_cnt, B * D.nchunk);
  DA(D.p2d, B * cap);
  DA(D.bcnt, B * WH);
  DA(D.bstart, B * (WH + 1));
  DA(D.bfill, B * WH);
  DA(D.bslot, B * WH);
  DA(D.members, B * cap);
  DA(D.bx, B * WH);
  DA(D.by, B * WH);
  DA(D.bd, B * WH);
  DA(D.dnsp, B * WH);
#undef DA
  h->hf.assign(B, DepthFrame{});
  if (hipStreamSynchronize(h->st) != hipSuccess) return fail(LOAM_ERR_HIP);
  *out = h;
  return LOAM_OK;
}

int32_t loam_depth_destroy(loam_depth* h) {
  if (!h) return LOAM_ERR_ARG;
  (void)hipSetDevice(h->dev);
  dp_free(h);
  delete h;
  return LOAM_OK;
}

static int32_t dp_input(loam_depth* h, int32_t s, const float* xyz, int32_t n, int32_t stride, bool device) {
  TRY(dp_check(h, s));
  if (n < 0 || (n > 0 && !xyz) || stride < 3) {
    set_error("loam_depth_input: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (n > h->D.cap) {
    set_error("loam_depth_input: more points than max_points");
    return LOAM_ERR_CAPACITY;
  }
  LOAM_HIP(hipSetDevice(h->dev));
  DepthFrame& F = h->hf[s];
  F.n = n;
  F.active = 1;
  if (device) {
    F.xyz = xyz;
    F.stride = stride;
  } else {  // staged as 4 floats per point (visual_odometry.cpp:201-208 copies too)
    float4* dst = h->stage + (size_t)s * h->D.cap;
    if (n) LOAM_HIP(hipMemcpy2DAsync(dst, sizeof(float4), xyz, sizeof(float) * stride, sizeof(float) * 3, n,
                                     hipMemcpyHostToDevice, h->st));
    F.xyz = reinterpret_cast<const float*>(dst);
    F.stride = 4;
    LOAM_HIP(hipStreamSynchronize(h->st));  // the caller's buffer is free after return
  }
  return LOAM_OK;
}

int32_t loam_depth_input(loam_depth* h, int32_t s, const float* xyz, int32_t n, int32_t stride) {
  return dp_input(h, s, xyz, n, stride, false);
}

int32_t loam_depth_input_device(loam_depth* h, int32_t s, const float* d_xyz, int32_t n, int32_t stride) {
  return dp_input(h, s, d_xyz, n, stride, true);
}

int32_t loam_depth_process(loam_depth* h) {
  if (!h) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  DepthDev& D = h->D;
  const int B = h->B;
  bool any = false;
  for (auto& F : h->hf) {
    F.n_front = F.n_dnsp = 0;
    F.err = 0;
    any |= F.active != 0;
  }
  if (!any) return LOAM_OK;
  hipStream_t st = h->st;
  const size_t WH = (size_t)D.W * D.H;
  LOAM_HIP(hipEventRecord(h->ev[0], st));
  LOAM_HIP(hipMemcpyAsync(D.fr, h->hf.data(), sizeof(DepthFrame) * B, hipMemcpyHostToDevice, st));
  LOAM_HIP(hipMemsetAsync(D.bcnt, 0, sizeof(int) * B * WH, st));
  LOAM_HIP(hipMemsetAsync(D.bfill, 0, sizeof(int) * B * WH, st));
  k_dp_project<<<B * D.nchunk, DP_THREADS, 0, st>>>(D);
  k_dp_scan<<<B, DP_SCAN_THREADS, 0, st>>>(D);
  k_dp_scatter<<<B * D.nchunk, DP_THREADS, 0, st>>>(D);
  const int bps = (int)((WH + DP_THREADS - 1) / DP_THREADS);
  k_dp_bucket<<<B * bps, DP_THREADS, 0, st>>>(D, bps);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipEventRecord(h->ev[1], st));
  LOAM_HIP(hipMemcpyAsync(h->hf.data(), D.fr, sizeof(DepthFrame) * B, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipStreamSynchronize(st));
  LOAM_HIP(hipEventElapsedTime(&h->ms, h->ev[0], h->ev[1]));
  for (auto& F : h->hf) F.active = 0;
  return LOAM_OK;
}

int32_t loam_depth_counts(loam_depth* h, int32_t s, int32_t* n_front, int32_t* n_dnsp) {
  TRY(dp_check(h, s));
  if (n_front) *n_front = h->hf[s].n_front;
  if (n_dnsp) *n_dnsp = h->hf[s].n_dnsp;
  return LOAM_OK;
}

int32_t loam_depth_copy(loam_depth* h, int32_t s, int32_t which, float* out, int32_t cap) {
  TRY(dp_check(h, s));
  if (which < 0 || which > 1) return LOAM_ERR_ARG;
  const int n = which == 0 ? h->hf[s].n_front : h->hf[s].n_dnsp;
  if (n > cap || (n > 0 && !out)) return n;  // the count only
  if (n) {
    LOAM_HIP(hipSetDevice(h->dev));
    const float4* src = which == 0 ? h->D.p2d + (size_t)s * h->D.cap : h->D.dnsp + (size_t)s * h->D.W * h->D.H;
    LOAM_HIP(hipMemcpy2D(out, sizeof(float) * 3, src, sizeof(float4), sizeof(float) * 3, n, hipMemcpyDeviceToHost));
  }
  return n;
}

int32_t loam_depth_buckets(loam_depth* h, int32_t s, float* bx, float* by, float* bd, int32_t* bc) {
  TRY(dp_check(h, s));
  if (!bx || !by || !bd || !bc) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  const size_t WH = (size_t)h->D.W * h->D.H, o = (size_t)s * WH;
  LOAM_HIP(hipMemcpy(bx, h->D.bx + o, sizeof(float) * WH, hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(by, h->D.by + o, sizeof(float) * WH, hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(bd, h->D.bd + o, sizeof(float) * WH, hipMemcpyDeviceToHost));
  LOAM_HIP(hipMemcpy(bc, h->D.bcnt + o, sizeof(int) * WH, hipMemcpyDeviceToHost));
  return LOAM_OK;
}

int32_t loam_depth_query(loam_depth* h, int32_t n, const int32_t* streams, const float* xy, int32_t radius,
                         float* depth) {
  if (!h || n < 0 || (n > 0 && (!streams || !xy || !depth)) || radius < 0) {
    set_error("loam_depth_query: bad arguments");
    return LOAM_ERR_ARG;
  }
  for (int i = 0; i < n; ++i)
    if (streams[i] < 0 || streams[i] >= h->B) {
      set_error("loam_depth_query: stream out of range");
      return LOAM_ERR_ARG;
    }
  if (n == 0) return LOAM_OK;
  LOAM_HIP(hipSetDevice(h->dev));
  TRY(dp_query_cap(h, n));
  hipStream_t st = h->st;
  LOAM_HIP(hipMemcpyAsync(h->d_qs, streams, sizeof(int) * n, hipMemcpyHostToDevice, st));
  LOAM_HIP(hipMemcpyAsync(h->d_xy, xy, sizeof(float2) * n, hipMemcpyHostToDevice, st));
  k_dp_query<<<(n + DP_THREADS - 1) / DP_THREADS, DP_THREADS, 0, st>>>(h->D, h->d_qs, h->d_xy, n, radius, h->d_depth);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipMemcpyAsync(depth, h->d_depth, sizeof(float) * n, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipStreamSynchronize(st));
  return LOAM_OK;
}

int32_t loam_depth_query_device(loam_depth* h, int32_t n, const int32_t* d_streams, const float* d_xy,
                                int32_t radius, float* d_depth) {
  if (!h || n < 0 || (n > 0 && (!d_streams || !d_xy || !d_depth)) || radius < 0) {
    set_error("loam_depth_query_device: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (n == 0) return LOAM_OK;
  LOAM_HIP(hipSetDevice(h->dev));
  k_dp_query<<<(n + DP_THREADS - 1) / DP_THREADS, DP_THREADS, 0, h->st>>>(
      h->D, d_streams, reinterpret_cast<const float2*>(d_xy), n, radius, d_depth);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipStreamSynchronize(h->st));
  return LOAM_OK;
}

double loam_depth_ms(loam_depth* h) { return h ? (double)h->ms : -1.0; }

}  // extern "C"
