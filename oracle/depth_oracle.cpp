// depth_oracle.cpp — CPU restatement of the visual-odometry depth association
// (TEST INFRASTRUCTURE ONLY, see loam_oracle.h).
//
// Follows liuzm-slam/VLOAM-NOTED src/visual_odometry/src/point_cloud_util.cpp:
//   projectPointCloud     :183-219  X~ (n x 4, [x y z 1]) * cam_T_velo^T * rect0_T_cam^T *
//                                   P_rect0^T -> (u', v', depth); keep depth > 0.1; u = u' * (1/d)
//   downsamplePointCloud  :256-324  5 px buckets (249 x 75 for 1242 x 375), first point then
//                                   incremental averaging b += (p - b) / count in input order;
//                                   point_cloud_2d_dnsp filled from the end in (x, y) bucket order
//   queryDepth            :381-487  the occupied buckets of a 5 x 5 block around (x, y); < 10
//                                   of them -> -1; else the 3 nearest in the image plane
//                                   (distance in double: std::pow(float, int) promotes) and the
//                                   inverse-distance weighted depth in float
// Called from visual_odometry.cpp:195-214 (processPointCloud) and :371-372 (per match).
//
// Float order: Eigen's 4-term dot products of the matrix chain are evaluated here
// sequentially, k = 0..3, without FMA (Eigen's packet path for the row blocks; its scalar tail
// and -mfma builds may round differently in the last bit: "parity unpinned" against Eigen's
// internals, bit-exact against the HIP kernels, which follow this file).  The reference sorts
// the neighbours with std::sort (unstable); here ties keep the gather order.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "loam_oracle.h"

namespace {

struct DepthUtil {
  float A[16], B[16], C[12];  // cam_T_velo, rect0_T_cam (4x4), P_rect0 (3x4), row-major
  int grid = 5, img_w = 1242, img_h = 375;
  int new_w = 0, new_h = 0;
  std::vector<float> p2d;   // point_cloud_2d, n x 3
  std::vector<float> dnsp;  // point_cloud_2d_dnsp, m x 3
  std::vector<float> bx, by, bd;  // bucket_x / _y / _depth, [i * new_h + j]
  std::vector<int> bc;            // bucket_count
  double ms = 0.0;
};

// r[j] = sum_k v[k] * M[j][k] (the row-vector times M^T), k sequential
inline void mul_t(const float* v, const float* M, int rows, float* r) {
  for (int j = 0; j < rows; ++j) {
    float acc = v[0] * M[j * 4 + 0];
    acc = acc + v[1] * M[j * 4 + 1];
    acc = acc + v[2] * M[j * 4 + 2];
    acc = acc + v[3] * M[j * 4 + 3];
    r[j] = acc;
  }
}

void project(DepthUtil& U, const float* xyz, int n, int stride) {
  U.p2d.clear();
  for (int i = 0; i < n; ++i) {
    const float v0[4] = {xyz[(size_t)i * stride], xyz[(size_t)i * stride + 1], xyz[(size_t)i * stride + 2], 1.0f};
    float v1[4], v2[4], v3[3];
    mul_t(v0, U.A, 4, v1);
    mul_t(v1, U.B, 4, v2);
    mul_t(v2, U.C, 3, v3);
    if (!(v3[2] > 0.1f)) continue;  // :197-198
    const float inv = 1.0f / v3[2];  // Eigen::inverse, :214-216
    U.p2d.push_back(v3[0] * inv);
    U.p2d.push_back(v3[1] * inv);
    U.p2d.push_back(v3[2]);
  }
}

void downsample(DepthUtil& U) {
  const int W = U.new_w, H = U.new_h;
  U.bx.assign((size_t)W * H, 0.f);
  U.by.assign((size_t)W * H, 0.f);
  U.bd.assign((size_t)W * H, 0.f);
  U.bc.assign((size_t)W * H, 0);
  const float g = (float)U.grid;
  int global = 0;
  const int n = (int)(U.p2d.size() / 3);
  for (int i = 0; i < n; ++i) {
    const float x = U.p2d[3 * i], y = U.p2d[3 * i + 1], d = U.p2d[3 * i + 2];
    const int ix = static_cast<int>(x / g), iy = static_cast<int>(y / g);
    if (!(ix >= 0 && ix < W && iy >= 0 && iy < H)) continue;
    const size_t b = (size_t)ix * H + iy;
    if (U.bc[b] == 0) {
      U.bx[b] = x;
      U.by[b] = y;
      U.bd[b] = d;
      ++global;
    } else {
      const float c = (float)U.bc[b];
      U.bx[b] += (x - U.bx[b]) / c;
      U.by[b] += (y - U.by[b]) / c;
      U.bd[b] += (d - U.bd[b]) / c;
    }
    ++U.bc[b];
  }
  U.dnsp.assign((size_t)global * 3, 0.f);
  for (int i = 0; i < W; ++i)
    for (int j = 0; j < H; ++j) {
      const size_t b = (size_t)i * H + j;
      if (U.bc[b] > 0) {
        --global;
        U.dnsp[3 * (size_t)global] = U.bx[b];
        U.dnsp[3 * (size_t)global + 1] = U.by[b];
        U.dnsp[3 * (size_t)global + 2] = U.bd[b];
      }
    }
}

float query(const DepthUtil& U, float x, float y, int radius) {
  const float g = (float)U.grid;
  const int ix = static_cast<int>(x / g), iy = static_cast<int>(y / g);
  struct Nb {
    float x, y, d, dist;
  };
  std::vector<Nb> nb;
  for (int i = ix - radius; i <= ix + radius; ++i)
    for (int j = iy - radius; j <= iy + radius; ++j) {
      if (!(i >= 0 && i < U.new_w && j >= 0 && j < U.new_h)) continue;
      const size_t b = (size_t)i * U.new_h + j;
      if (U.bc[b] <= 0) continue;
      Nb e;
      e.x = U.bx[b];
      e.y = U.by[b];
      e.d = U.bd[b];
      const double dx = (double)(x - e.x), dy = (double)(y - e.y);
      e.dist = (float)std::sqrt(dx * dx + dy * dy);
      nb.push_back(e);
    }
  if (nb.size() < 10) return -1.0f;
  std::stable_sort(nb.begin(), nb.end(), [](const Nb& a, const Nb& b) { return a.dist < b.dist; });
  const Nb &n0 = nb[0], &n1 = nb[1], &n2 = nb[2];
  return (n0.d * n1.dist * n2.dist + n1.d * n0.dist * n2.dist + n2.d * n0.dist * n1.dist) /
         (0.0001f + n1.dist * n2.dist + n0.dist * n2.dist + n0.dist * n1.dist);
}

}  // namespace

extern "C" {

void* oracle_depth_create(const float* cam_T_velo, const float* rect0_T_cam, const float* P_rect0, int32_t grid,
                          int32_t img_w, int32_t img_h) {
  auto* U = new DepthUtil;
  std::memcpy(U->A, cam_T_velo, sizeof(U->A));
  std::memcpy(U->B, rect0_T_cam, sizeof(U->B));
  std::memcpy(U->C, P_rect0, sizeof(U->C));
  U->grid = grid;
  U->img_w = img_w;
  U->img_h = img_h;
  // :260-262: std::ceil(float(IMG) / float(grid))
  U->new_w = (int)std::ceil(static_cast<float>(img_w) / static_cast<float>(grid));
  U->new_h = (int)std::ceil(static_cast<float>(img_h) / static_cast<float>(grid));
  return U;
}

void oracle_depth_destroy(void* h) { delete static_cast<DepthUtil*>(h); }

int32_t oracle_depth_process(void* h, const float* xyz, int32_t n, int32_t stride) {
  auto* U = static_cast<DepthUtil*>(h);
  const auto t0 = std::chrono::steady_clock::now();
  project(*U, xyz, n, stride);
  downsample(*U);
  U->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return (int32_t)(U->dnsp.size() / 3);
}

int32_t oracle_depth_count(void* h, int32_t which) {
  auto* U = static_cast<DepthUtil*>(h);
  return (int32_t)((which == 0 ? U->p2d.size() : U->dnsp.size()) / 3);
}

void oracle_depth_copy(void* h, int32_t which, float* out) {
  auto* U = static_cast<DepthUtil*>(h);
  const auto& v = which == 0 ? U->p2d : U->dnsp;
  std::memcpy(out, v.data(), sizeof(float) * v.size());
}

void oracle_depth_buckets(void* h, float* bx, float* by, float* bd, int32_t* bc) {
  auto* U = static_cast<DepthUtil*>(h);
  std::memcpy(bx, U->bx.data(), sizeof(float) * U->bx.size());
  std::memcpy(by, U->by.data(), sizeof(float) * U->by.size());
  std::memcpy(bd, U->bd.data(), sizeof(float) * U->bd.size());
  std::memcpy(bc, U->bc.data(), sizeof(int32_t) * U->bc.size());
}

double oracle_depth_query(void* h, const float* xy, int32_t n, int32_t radius, float* depth) {
  auto* U = static_cast<DepthUtil*>(h);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) depth[i] = query(*U, xy[2 * i], xy[2 * i + 1], radius);
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

double oracle_depth_ms(void* h) { return static_cast<DepthUtil*>(h)->ms; }

}  // extern "C"
