// loam_oracle.cpp — CPU oracle for the LOAM scan-matching hot path.
//
// TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
// PARITY UNPINNED: the reference (liuzm-slam/VLOAM-NOTED) ships no tests / golden
// vectors and cannot be built here (ROS1/PCL/Ceres/Eigen absent), so this
// restatement follows the reference source line by line and is cross-checked against
// independent implementations (scipy cKDTree, numpy eigh/lstsq, finite differences).
//
// Paths below are relative to /root/reference/src/lidar_odometry_mapping/.
// Build: oracle/Makefile  (g++ -O3 -ffp-contract=off; single-threaded, like the reference).
#include "loam_oracle.h"

#include <algorithm>
#include <array>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <numeric>
#include <vector>

namespace oracle {

struct Pt {
  float x, y, z, intensity;
};
using Cloud = std::vector<Pt>;

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------------------------------
// Eigen 3.3 quaternion arithmetic (generic, non-SIMD path), xyzw storage like para_q.
// ---------------------------------------------------------------------------------------
struct Quat {
  double x, y, z, w;
};
struct V3 {
  double x, y, z;
};
static inline V3 cross(const V3& a, const V3& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// Eigen QuaternionBase::_transformVector: uv = vec x v; uv += uv; v + w*uv + vec x uv
static inline V3 qrot(const Quat& q, const V3& v) {
  V3 qv{q.x, q.y, q.z};
  V3 uv = cross(qv, v);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  V3 c = cross(qv, uv);
  return {(v.x + q.w * uv.x) + c.x, (v.y + q.w * uv.y) + c.y, (v.z + q.w * uv.z) + c.z};
}
// Eigen quat_product (generic)
static inline Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
// Eigen QuaternionBase::inverse: conjugate / squaredNorm
static inline Quat qinv(const Quat& q) {
  double n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  if (n2 > 0) return {-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
  return {0, 0, 0, 0};
}

// ---------------------------------------------------------------------------------------
// PCL VoxelGrid<PointXYZI>::applyFilter (pcl/filters/impl/voxel_grid.hpp, PCL 1.10):
// bbox → leaf ijk = floor(p*inv) - min_b → idx = i + j*dx + k*dx*dy → sort → centroid of
// x,y,z,intensity (CentroidPoint, float sums / float(n)).  The sort is PCL's: std::sort of
// cloud_point_index_idx {idx, cloud_point_index} with operator< comparing idx only, so the
// order of a voxel's points (its float summation order) is libstdc++'s introsort permutation
// (GCC 4.9-13 bits/stl_algo.h; this file is built with GCC 11, the same algorithm as the
// GCC 7 / 9 of the reference's Ubuntu 18.04 / 20.04 ROS builds).
// g_voxel_order = 1 sums a voxel's points in input order instead (std::stable_sort): the
// order of the mapper's VoxelGrid kernels (voxel.h), for their bit-exact tests.
// ---------------------------------------------------------------------------------------
static int g_voxel_order = 0;  // 0: PCL (std::sort), 1: input order

struct CloudPointIndexIdx {  // pcl::VoxelGrid's cloud_point_index_idx
  uint32_t idx;
  uint32_t cloud_point_index;
  bool operator<(const CloudPointIndexIdx& p) const { return idx < p.idx; }
};

Cloud voxel_grid(const Cloud& in, float leaf) {
  Cloud out;
  if (in.empty()) return out;
  const float inv = 1.0f / leaf;
  float mnx = FLT_MAX, mny = FLT_MAX, mnz = FLT_MAX;
  float mxx = -FLT_MAX, mxy = -FLT_MAX, mxz = -FLT_MAX;
  for (const Pt& p : in) {
    mnx = std::min(mnx, p.x); mny = std::min(mny, p.y); mnz = std::min(mnz, p.z);
    mxx = std::max(mxx, p.x); mxy = std::max(mxy, p.y); mxz = std::max(mxz, p.z);
  }
  int64_t dx = static_cast<int64_t>((mxx - mnx) * inv) + 1;
  int64_t dy = static_cast<int64_t>((mxy - mny) * inv) + 1;
  int64_t dz = static_cast<int64_t>((mxz - mnz) * inv) + 1;
  if (dx * dy * dz > static_cast<int64_t>(std::numeric_limits<int32_t>::max())) return in;
  const int minbx = static_cast<int>(std::floor(mnx * inv));
  const int maxbx = static_cast<int>(std::floor(mxx * inv));
  const int minby = static_cast<int>(std::floor(mny * inv));
  const int maxby = static_cast<int>(std::floor(mxy * inv));
  const int minbz = static_cast<int>(std::floor(mnz * inv));
  const int divx = maxbx - minbx + 1;
  const int divy = maxby - minby + 1;
  const int mul1 = divx, mul2 = divx * divy;
  std::vector<CloudPointIndexIdx> iv(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    const Pt& p = in[i];
    int i0 = static_cast<int>(std::floor(p.x * inv) - static_cast<float>(minbx));
    int i1 = static_cast<int>(std::floor(p.y * inv) - static_cast<float>(minby));
    int i2 = static_cast<int>(std::floor(p.z * inv) - static_cast<float>(minbz));
    int idx = i0 + i1 * mul1 + i2 * mul2;
    iv[i] = {static_cast<uint32_t>(idx), static_cast<uint32_t>(i)};
  }
  if (g_voxel_order == 0) std::sort(iv.begin(), iv.end(), std::less<CloudPointIndexIdx>());
  else std::stable_sort(iv.begin(), iv.end());
  size_t s = 0;
  while (s < iv.size()) {
    size_t e = s + 1;
    while (e < iv.size() && iv[e].idx == iv[s].idx) ++e;
    float sx = 0, sy = 0, sz = 0, si = 0;
    for (size_t k = s; k < e; ++k) {
      const Pt& p = in[iv[k].cloud_point_index];
      sx += p.x; sy += p.y; sz += p.z; si += p.intensity;
    }
    const float n = static_cast<float>(e - s);
    out.push_back({sx / n, sy / n, sz / n, si / n});
    s = e;
  }
  return out;
}

// ---------------------------------------------------------------------------------------
// Exact kNN with FLANN KDTreeSingleIndex semantics (eps = 0, sorted, L2_Simple<float>:
// d = ((dx*dx) + dy*dy) + dz*dz in float, xyz only — PCL DefaultPointRepresentation
// <PointXYZI>).  Ties are broken by index (FLANN's tie order is traversal-dependent).
// ---------------------------------------------------------------------------------------
static inline float fdist(float qx, float qy, float qz, const Pt& p) {
  float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  float r = 0.0f;
  r += dx * dx;
  r += dy * dy;
  r += dz * dz;
  return r;
}

class KdTree {
 public:
  void build(const Cloud* c) {
    cloud_ = c;
    nodes_.clear();
    perm_.resize(c->size());
    std::iota(perm_.begin(), perm_.end(), 0);
    if (!c->empty()) build_rec(0, static_cast<int>(c->size()));
  }
  // k nearest, sorted ascending by (d2, idx); returns count found (<= k)
  int knn(float qx, float qy, float qz, int k, int* idx, float* d2) const {
    if (!cloud_ || cloud_->empty()) return 0;
    cnt_ = 0;
    k_ = k;
    bi_ = idx;
    bd_ = d2;
    search(0, qx, qy, qz);
    return cnt_;
  }

 private:
  struct Node {
    int begin, end;
    int left, right;  // -1: leaf
    int dim;
    float split;
  };
  static constexpr int kLeaf = 10;
  int build_rec(int b, int e) {
    int id = static_cast<int>(nodes_.size());
    nodes_.push_back({b, e, -1, -1, 0, 0.f});
    if (e - b <= kLeaf) return id;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = b; i < e; ++i) {
      const Pt& p = (*cloud_)[perm_[i]];
      const float c[3] = {p.x, p.y, p.z};
      for (int d = 0; d < 3; ++d) { mn[d] = std::min(mn[d], c[d]); mx[d] = std::max(mx[d], c[d]); }
    }
    int dim = 0;
    for (int d = 1; d < 3; ++d)
      if (mx[d] - mn[d] > mx[dim] - mn[dim]) dim = d;
    if (mx[dim] - mn[dim] <= 0.f) return id;  // all identical: leaf
    int m = (b + e) / 2;
    auto coord = [&](int i) {
      const Pt& p = (*cloud_)[i];
      return dim == 0 ? p.x : (dim == 1 ? p.y : p.z);
    };
    std::nth_element(perm_.begin() + b, perm_.begin() + m, perm_.begin() + e,
                     [&](int a, int c) { return coord(a) < coord(c); });
    float split = coord(perm_[m]);
    nodes_[id].dim = dim;
    nodes_[id].split = split;
    int l = build_rec(b, m);
    int r = build_rec(m, e);
    nodes_[id].left = l;
    nodes_[id].right = r;
    return id;
  }
  inline bool better(float d, int i, float d2, int i2) const { return d < d2 || (d == d2 && i < i2); }
  void offer(float d, int i) const {
    if (cnt_ == k_ && !better(d, i, bd_[cnt_ - 1], bi_[cnt_ - 1])) return;
    int pos = (cnt_ < k_) ? cnt_++ : k_ - 1;
    while (pos > 0 && better(d, i, bd_[pos - 1], bi_[pos - 1])) {
      bd_[pos] = bd_[pos - 1];
      bi_[pos] = bi_[pos - 1];
      --pos;
    }
    bd_[pos] = d;
    bi_[pos] = i;
  }
  void search(int nid, float qx, float qy, float qz) const {
    const Node& n = nodes_[nid];
    if (n.left < 0) {
      for (int i = n.begin; i < n.end; ++i) {
        int pi = perm_[i];
        offer(fdist(qx, qy, qz, (*cloud_)[pi]), pi);
      }
      return;
    }
    float q = n.dim == 0 ? qx : (n.dim == 1 ? qy : qz);
    float diff = q - n.split;
    int nearc = diff < 0 ? n.left : n.right;
    int farc = diff < 0 ? n.right : n.left;
    search(nearc, qx, qy, qz);
    if (cnt_ < k_ || diff * diff <= bd_[cnt_ - 1]) search(farc, qx, qy, qz);
  }
  const Cloud* cloud_ = nullptr;
  std::vector<Node> nodes_;
  std::vector<int> perm_;
  mutable int cnt_ = 0, k_ = 0;
  mutable int* bi_ = nullptr;
  mutable float* bd_ = nullptr;
};

// ---------------------------------------------------------------------------------------
// 3x3 symmetric eigen-decomposition (cyclic Jacobi, ascending eigenvalues) — stands in for
// Eigen::SelfAdjointEigenSolver<Matrix3d> (laser_mapping.cpp:583).  The HIP kernel runs the
// same sequence of operations, so oracle and device agree bit-for-bit.
// ---------------------------------------------------------------------------------------
void eig3(const double Ain[3][3], double evals[3], double evecs[3][3]) {
  double a[3][3], v[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      a[i][j] = Ain[i][j];
      v[i][j] = (i == j) ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = std::fabs(a[0][1]) + std::fabs(a[0][2]) + std::fabs(a[1][2]);
    if (off == 0.0) break;
    for (int p = 0; p < 2; ++p) {
      for (int q = p + 1; q < 3; ++q) {
        double apq = a[p][q];
        if (apq == 0.0) continue;
        double app = a[p][p], aqq = a[q][q];
        double theta = (aqq - app) / (2.0 * apq);
        double t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
        double c = 1.0 / std::sqrt(t * t + 1.0);
        double s = t * c;
        for (int k = 0; k < 3; ++k) {
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        a[p][q] = 0.0;
        a[q][p] = 0.0;
        for (int k = 0; k < 3; ++k) {
          double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
    }
  }
  int ord[3] = {0, 1, 2};
  // ascending, stable on ties
  for (int i = 1; i < 3; ++i) {
    int j = i;
    while (j > 0 && a[ord[j]][ord[j]] < a[ord[j - 1]][ord[j - 1]]) {
      std::swap(ord[j], ord[j - 1]);
      --j;
    }
  }
  for (int i = 0; i < 3; ++i) {
    evals[i] = a[ord[i]][ord[i]];
    for (int k = 0; k < 3; ++k) evecs[k][i] = v[k][ord[i]];
  }
}

// ---------------------------------------------------------------------------------------
// 5x3 least squares A n = -1 by column-pivoted Householder QR — stands in for
// Eigen::ColPivHouseholderQR<Matrix<double,5,3>>::solve (laser_mapping.cpp:655).
// ---------------------------------------------------------------------------------------
void lsq53(const double Ain[5][3], double x[3]) {
  double A[5][3];
  double b[5];
  for (int i = 0; i < 5; ++i) {
    b[i] = -1.0;
    for (int j = 0; j < 3; ++j) A[i][j] = Ain[i][j];
  }
  int perm[3] = {0, 1, 2};
  double diag[3] = {0, 0, 0};
  for (int k = 0; k < 3; ++k) {
    // pivot: largest remaining column norm (first on ties)
    int best = k;
    double bestn = -1.0;
    for (int j = k; j < 3; ++j) {
      double s = 0.0;
      for (int i = k; i < 5; ++i) s += A[i][j] * A[i][j];
      if (s > bestn) {
        bestn = s;
        best = j;
      }
    }
    if (best != k) {
      for (int i = 0; i < 5; ++i) std::swap(A[i][k], A[i][best]);
      std::swap(perm[k], perm[best]);
    }
    // Householder on A[k:5, k]  (Eigen makeHouseholder convention)
    double c0 = A[k][k];
    double tail = 0.0;
    for (int i = k + 1; i < 5; ++i) tail += A[i][k] * A[i][k];
    double tau, beta;
    double ess[5] = {0, 0, 0, 0, 0};
    if (tail <= DBL_MIN) {
      tau = 0.0;
      beta = c0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      for (int i = k + 1; i < 5; ++i) ess[i] = A[i][k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    diag[k] = beta;
    A[k][k] = beta;
    for (int i = k + 1; i < 5; ++i) A[i][k] = 0.0;
    // apply H = I - tau v v^T, v = [1; ess] to remaining columns and b
    for (int j = k + 1; j < 3; ++j) {
      double s = A[k][j];
      for (int i = k + 1; i < 5; ++i) s += ess[i] * A[i][j];
      s *= tau;
      A[k][j] -= s;
      for (int i = k + 1; i < 5; ++i) A[i][j] -= s * ess[i];
    }
    {
      double s = b[k];
      for (int i = k + 1; i < 5; ++i) s += ess[i] * b[i];
      s *= tau;
      b[k] -= s;
      for (int i = k + 1; i < 5; ++i) b[i] -= s * ess[i];
    }
  }
  double z[3] = {0, 0, 0};
  for (int k = 2; k >= 0; --k) {
    if (diag[k] == 0.0) {
      z[k] = 0.0;
      continue;
    }
    double s = b[k];
    for (int j = k + 1; j < 3; ++j) s -= A[k][j] * z[j];
    z[k] = s / A[k][k];
  }
  for (int k = 0; k < 3; ++k) x[perm[k]] = z[k];
}

// edge correspondence (laser_mapping.cpp:557-603): nbr already gated by sqDis[4] < 1
bool edge_from_nbrs(const Pt* nb, V3& pa, V3& pb) {
  double cx = 0, cy = 0, cz = 0;
  for (int j = 0; j < 5; ++j) {
    cx = cx + (double)nb[j].x;
    cy = cy + (double)nb[j].y;
    cz = cz + (double)nb[j].z;
  }
  cx = cx / 5.0; cy = cy / 5.0; cz = cz / 5.0;
  double C[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int j = 0; j < 5; ++j) {
    double d[3] = {(double)nb[j].x - cx, (double)nb[j].y - cy, (double)nb[j].z - cz};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) C[r][c] = C[r][c] + d[r] * d[c];
  }
  double ev[3], evec[3][3];
  eig3(C, ev, evec);
  if (ev[2] > 3 * ev[1]) {
    double ux = evec[0][2], uy = evec[1][2], uz = evec[2][2];
    pa = {0.1 * ux + cx, 0.1 * uy + cy, 0.1 * uz + cz};
    pb = {-0.1 * ux + cx, -0.1 * uy + cy, -0.1 * uz + cz};
    return true;
  }
  return false;
}

// plane correspondence (laser_mapping.cpp:642-680)
bool plane_from_nbrs(const Pt* nb, V3& n, double& d) {
  double A[5][3];
  for (int j = 0; j < 5; ++j) {
    A[j][0] = nb[j].x;
    A[j][1] = nb[j].y;
    A[j][2] = nb[j].z;
  }
  double x[3];
  lsq53(A, x);
  double nn = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  double negdot = 1 / nn;
  n = {x[0] / nn, x[1] / nn, x[2] / nn};
  d = negdot;
  for (int j = 0; j < 5; ++j) {
    if (std::fabs(n.x * nb[j].x + n.y * nb[j].y + n.z * nb[j].z + negdot) > 0.2) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------
// Residual blocks (lidarFactor.hpp).  Analytic Jacobians in the 6-dof local space of
// Ceres' EigenQuaternionParameterization (Plus(x, δ) = [cos|δ|, sinc|δ| δ] ⊗ x):
//   ∂p'/∂δθ = -2 [R p]_x,  ∂p'/∂t = I;  s = 1 (DISTORTION = false, laser_odometry.h:90).
// ---------------------------------------------------------------------------------------
struct Factor {
  int type;  // 1 edge (3 rows), 2 plane via (j, n) (odometry), 3 plane-norm (n, d) (mapping)
  double p[3], a[3], b[3];
};

struct Eval {
  double cost;
  std::vector<double> f;  // corrected residuals (M)
  std::vector<double> J;  // corrected Jacobian M x 6 (row-major)
  double g[6];            // J^T f
};

static int factor_rows(const Factor& f) { return f.type == 1 ? 3 : 1; }

// Evaluate one residual block: r[3] (rows), dr/dp' (rows x 3), and Rp.
static inline int eval_block(const Factor& F, const Quat& q, const V3& t, double r[3],
                             double drdp[3][3], V3& Rp) {
  V3 p{F.p[0], F.p[1], F.p[2]};
  Rp = qrot(q, p);
  V3 lp{Rp.x + t.x, Rp.y + t.y, Rp.z + t.z};
  if (F.type == 1) {
    V3 a{F.a[0], F.a[1], F.a[2]}, b{F.b[0], F.b[1], F.b[2]};
    V3 u{lp.x - a.x, lp.y - a.y, lp.z - a.z};
    V3 w{lp.x - b.x, lp.y - b.y, lp.z - b.z};
    V3 nu = cross(u, w);
    V3 de{a.x - b.x, a.y - b.y, a.z - b.z};
    double dn = std::sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
    r[0] = nu.x / dn;
    r[1] = nu.y / dn;
    r[2] = nu.z / dn;
    // d(u x w)/dlp = [b - a]_x
    V3 ba{b.x - a.x, b.y - a.y, b.z - a.z};
    drdp[0][0] = 0;           drdp[0][1] = -ba.z / dn;  drdp[0][2] = ba.y / dn;
    drdp[1][0] = ba.z / dn;   drdp[1][1] = 0;           drdp[1][2] = -ba.x / dn;
    drdp[2][0] = -ba.y / dn;  drdp[2][1] = ba.x / dn;   drdp[2][2] = 0;
    return 3;
  } else if (F.type == 2) {
    // (lp - j) . n
    double d0 = lp.x - F.a[0], d1 = lp.y - F.a[1], d2 = lp.z - F.a[2];
    r[0] = (d0 * F.b[0] + d1 * F.b[1]) + d2 * F.b[2];
    drdp[0][0] = F.b[0]; drdp[0][1] = F.b[1]; drdp[0][2] = F.b[2];
    return 1;
  } else {
    // n . lp + d
    r[0] = ((F.a[0] * lp.x + F.a[1] * lp.y) + F.a[2] * lp.z) + F.b[0];
    drdp[0][0] = F.a[0]; drdp[0][1] = F.a[1]; drdp[0][2] = F.a[2];
    return 1;
  }
}

// ---------------------------------------------------------------------------------------
// Visual-odometry residual blocks (src/visual_odometry/include/visual_odometry/
// ceres_cost_function.h), parameters angles_0to1 (angle-axis) and t_0to1, evaluated the way
// Ceres' AutoDiffCostFunction<.., 3, 3> does: forward-mode Jets through the functor, with
// ceres::AngleAxisRotatePoint / CrossProduct / DotProduct (ceres/rotation.h) and the Jet
// rules of ceres/jet.h.
//   type 4 CostFunctor32 (:58-102): p = X0, a[0..1] = (x1_bar, y1_bar), 2 rows
//   type 5 CostFunctor22 (:151-189): a[0..1] = (x0_bar, y0_bar), b[0..1] = (x1_bar, y1_bar), 1 row
// ---------------------------------------------------------------------------------------
struct Jet {
  double a;
  double v[6];
};
static inline Jet jconst(double c) {
  Jet j{c, {0, 0, 0, 0, 0, 0}};
  return j;
}
static inline Jet operator+(const Jet& f, const Jet& g) {
  Jet r{f.a + g.a, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = f.v[k] + g.v[k];
  return r;
}
static inline Jet operator-(const Jet& f, const Jet& g) {
  Jet r{f.a - g.a, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = f.v[k] - g.v[k];
  return r;
}
static inline Jet operator-(const Jet& f) {
  Jet r{-f.a, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = -f.v[k];
  return r;
}
static inline Jet operator*(const Jet& f, const Jet& g) {  // jet.h: (f.a g.a, f.a g.v + f.v g.a)
  Jet r{f.a * g.a, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = f.a * g.v[k] + f.v[k] * g.a;
  return r;
}
static inline Jet operator/(const Jet& f, const Jet& g) {  // jet.h: a = f.a / g.a, v = (f.v - a g.v) / g.a
  const double gi = 1.0 / g.a, fa = f.a * gi;
  Jet r{fa, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = (f.v[k] - fa * g.v[k]) * gi;
  return r;
}
static inline Jet jsqrt(const Jet& f) {
  const double t = std::sqrt(f.a), ti = 1.0 / (2.0 * t);
  Jet r{t, {}};
  for (int k = 0; k < 6; ++k) r.v[k] = f.v[k] * ti;
  return r;
}
static inline Jet jcos(const Jet& f) {
  const double sn = -std::sin(f.a);
  Jet r{std::cos(f.a), {}};
  for (int k = 0; k < 6; ++k) r.v[k] = sn * f.v[k];
  return r;
}
static inline Jet jsin(const Jet& f) {
  const double cs = std::cos(f.a);
  Jet r{std::sin(f.a), {}};
  for (int k = 0; k < 6; ++k) r.v[k] = cs * f.v[k];
  return r;
}

// ceres::AngleAxisRotatePoint (rotation.h)
static void aa_rotate(const Jet aa[3], const Jet pt[3], Jet out[3]) {
  const Jet theta2 = (aa[0] * aa[0] + aa[1] * aa[1]) + aa[2] * aa[2];
  if (theta2.a > std::numeric_limits<double>::epsilon()) {
    const Jet theta = jsqrt(theta2);
    const Jet costheta = jcos(theta), sintheta = jsin(theta);
    const Jet theta_inverse = jconst(1.0) / theta;
    const Jet w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
    const Jet wc[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
    const Jet tmp = ((w[0] * pt[0] + w[1] * pt[1]) + w[2] * pt[2]) * (jconst(1.0) - costheta);
    for (int i = 0; i < 3; ++i) out[i] = (pt[i] * costheta + wc[i] * sintheta) + w[i] * tmp;
  } else {
    const Jet wc[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
    for (int i = 0; i < 3; ++i) out[i] = pt[i] + wc[i];
  }
}

// residual rows r[m] and Jacobian rows J[m][6] of a VO block at x = (angles, t)
static int eval_vo_block(const Factor& F, const double* x, double r[3], double J[3][6]) {
  Jet aa[3], t[3];
  for (int i = 0; i < 3; ++i) {
    aa[i] = jconst(x[i]);
    aa[i].v[i] = 1.0;
    t[i] = jconst(x[3 + i]);
    t[i].v[3 + i] = 1.0;
  }
  Jet res[2];
  int m;
  if (F.type == 4) {  // CostFunctor32::operator()
    const Jet X0[3] = {jconst(F.p[0]), jconst(F.p[1]), jconst(F.p[2])};
    Jet R[3];
    aa_rotate(aa, X0, R);
    for (int i = 0; i < 3; ++i) R[i] = R[i] + t[i];
    res[0] = R[0] - R[2] * jconst(F.a[0]);
    res[1] = R[1] - R[2] * jconst(F.a[1]);
    m = 2;
  } else {  // CostFunctor22::operator()
    const Jet X0[3] = {jconst(F.a[0]), jconst(F.a[1]), jconst(1.0)};
    const Jet X1[3] = {jconst(F.b[0]), jconst(F.b[1]), jconst(1.0)};
    Jet q[3];
    aa_rotate(aa, X0, q);
    const Jet c[3] = {t[1] * q[2] - t[2] * q[1], t[2] * q[0] - t[0] * q[2], t[0] * q[1] - t[1] * q[0]};
    res[0] = (X1[0] * c[0] + X1[1] * c[1]) + X1[2] * c[2];
    m = 1;
  }
  for (int i = 0; i < m; ++i) {
    r[i] = res[i].a;
    for (int k = 0; k < 6; ++k) J[i][k] = res[i].v[k];
  }
  return m;
}

// HuberLoss(a=0.1): rho(s) and Corrector scale sqrt(rho') (ceres/loss_function.cc,
// ceres/corrector.cc; rho'' <= 0 branch => r, J scaled by sqrt(rho'))
static inline void huber(double s, double& rho0, double& rho1) {
  const double a = 0.1, b = 0.01;
  if (s > b) {
    const double r = std::sqrt(s);
    rho0 = 2.0 * a * r - b;
    rho1 = std::max(std::numeric_limits<double>::min(), a / r);
  } else {
    rho0 = s;
    rho1 = 1.0;
  }
}

static double evaluate(const std::vector<Factor>& fs, const double* x, Eval* ev) {
  Quat q{x[0], x[1], x[2], x[3]};
  V3 t{x[4], x[5], x[6]};
  double cost = 0.0;
  if (ev) {
    ev->f.clear();
    ev->J.clear();
    for (double& g : ev->g) g = 0.0;
  }
  for (const Factor& F : fs) {
    double r[3], drdp[3][3];
    V3 Rp;
    if (F.type >= 4) {  // VO block: full Jacobian rows from the Jets
      double Jv[3][6];
      const int mv = eval_vo_block(F, x, r, Jv);
      double sq = 0.0;
      for (int i = 0; i < mv; ++i) sq += r[i] * r[i];
      double rho0, rho1;
      huber(sq, rho0, rho1);
      cost += 0.5 * rho0;
      if (!ev) continue;
      const double sc = std::sqrt(rho1);
      for (int i = 0; i < mv; ++i) {
        const double ri = r[i] * sc;
        for (int c = 0; c < 6; ++c) {
          const double v = Jv[i][c] * sc;
          ev->J.push_back(v);
          ev->g[c] += v * ri;
        }
        ev->f.push_back(ri);
      }
      continue;
    }
    int m = eval_block(F, q, t, r, drdp, Rp);
    double sq = 0.0;
    for (int i = 0; i < m; ++i) sq += r[i] * r[i];
    double rho0, rho1;
    huber(sq, rho0, rho1);
    cost += 0.5 * rho0;
    if (!ev) continue;
    double sc = std::sqrt(rho1);
    // -2 [Rp]_x
    double M[3][3] = {{0, 2 * Rp.z, -2 * Rp.y}, {-2 * Rp.z, 0, 2 * Rp.x}, {2 * Rp.y, -2 * Rp.x, 0}};
    for (int i = 0; i < m; ++i) {
      double row[6];
      for (int c = 0; c < 3; ++c) {
        row[c] = (drdp[i][0] * M[0][c] + drdp[i][1] * M[1][c]) + drdp[i][2] * M[2][c];
        row[3 + c] = drdp[i][c];
      }
      double ri = r[i] * sc;
      for (int c = 0; c < 6; ++c) {
        row[c] *= sc;
        ev->J.push_back(row[c]);
        ev->g[c] += row[c] * ri;
      }
      ev->f.push_back(ri);
    }
  }
  if (ev) ev->cost = cost;
  return cost;
}

// EigenQuaternionParameterization::Plus + Euclidean t; euclid: plain x + d on 6 parameters
// (the VO problem's angle-axis + t blocks have no parameterization), x[6] = 0 kept
static bool g_plus_euclid = false;
static void plus(const double* x, const double* d, double* out) {
  if (g_plus_euclid) {
    for (int i = 0; i < 6; ++i) out[i] = x[i] + d[i];
    out[6] = x[6];
    return;
  }
  double nd = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    double s = std::sin(nd) / nd;
    Quat dq{s * d[0], s * d[1], s * d[2], std::cos(nd)};
    Quat r = qmul(dq, Quat{x[0], x[1], x[2], x[3]});
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
  } else {
    out[0] = x[0]; out[1] = x[1]; out[2] = x[2]; out[3] = x[3];
  }
  out[4] = x[4] + d[3];
  out[5] = x[5] + d[4];
  out[6] = x[6] + d[5];
}

// DenseQRSolver (ceres/dense_qr_solver.cc, EIGEN backend): y = householderQr([A; D]) \ [b; 0]
static bool dense_qr_solve(const std::vector<double>& Ain, int m, const double* D,
                           const std::vector<double>& bin, double* y) {
  const int n = 6;
  const int rows = m + n;
  std::vector<double> A(static_cast<size_t>(rows) * n, 0.0), b(rows, 0.0);
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j < n; ++j) A[i * n + j] = Ain[i * n + j];
    b[i] = bin[i];
  }
  for (int j = 0; j < n; ++j) A[(m + j) * n + j] = D[j];
  std::vector<double> ess(rows);
  for (int k = 0; k < n; ++k) {
    double c0 = A[k * n + k];
    double tail = 0.0;
    for (int i = k + 1; i < rows; ++i) tail += A[i * n + k] * A[i * n + k];
    double tau, beta;
    if (tail <= DBL_MIN) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1; i < rows; ++i) ess[i] = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      double den = c0 - beta;
      for (int i = k + 1; i < rows; ++i) ess[i] = A[i * n + k] / den;
      tau = (beta - c0) / beta;
    }
    A[k * n + k] = beta;
    for (int j = k + 1; j < n; ++j) {
      double s = A[k * n + j];
      for (int i = k + 1; i < rows; ++i) s += ess[i] * A[i * n + j];
      s *= tau;
      A[k * n + j] -= s;
      for (int i = k + 1; i < rows; ++i) A[i * n + j] -= s * ess[i];
    }
    double s = b[k];
    for (int i = k + 1; i < rows; ++i) s += ess[i] * b[i];
    s *= tau;
    b[k] -= s;
    for (int i = k + 1; i < rows; ++i) b[i] -= s * ess[i];
  }
  for (int k = n - 1; k >= 0; --k) {
    double s = b[k];
    for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * y[j];
    y[k] = s / A[k * n + k];
  }
  for (int k = 0; k < n; ++k)
    if (!std::isfinite(y[k])) return false;
  return true;
}

// ---------------------------------------------------------------------------------------
// Ceres 2.0 TrustRegionMinimizer + LevenbergMarquardtStrategy as configured by the
// reference (laser_odometry.cpp:500-509, laser_mapping.cpp:709-717): defaults except
// linear_solver_type = DENSE_QR, max_num_iterations = 4.
// ---------------------------------------------------------------------------------------
int lm_solve(const std::vector<Factor>& fs, double* x, int max_iter, oracle_lm_stats* st) {
  oracle_lm_stats s{};
  if (fs.empty()) {
    s.termination = 4;
    if (st) *st = s;
    return 0;
  }
  const double function_tolerance = 1e-6, gradient_tolerance = 1e-10,
               parameter_tolerance = 1e-8, min_relative_decrease = 1e-3,
               min_trust_region_radius = 1e-32, max_trust_region_radius = 1e16,
               min_lm_diagonal = 1e-6, max_lm_diagonal = 1e32;
  const int max_consecutive_invalid = 5;
  double radius = 1e4, decrease_factor = 2.0;
  bool reuse_diagonal = false;
  double diagonal[6];

  std::vector<double> xv(x, x + 7);
  Eval ev;
  evaluate(fs, xv.data(), &ev);
  const int M = static_cast<int>(ev.f.size());
  double x_cost = ev.cost;
  s.initial_cost = x_cost;
  double scaling[6];
  // Jacobi scaling fixed at iteration 0
  for (int c = 0; c < 6; ++c) {
    double sq = 0.0;
    for (int i = 0; i < M; ++i) sq += ev.J[i * 6 + c] * ev.J[i * 6 + c];
    scaling[c] = 1.0 / (1.0 + std::sqrt(sq));
  }
  auto scale_jac = [&](Eval& e) {
    for (int i = 0; i < M; ++i)
      for (int c = 0; c < 6; ++c) e.J[i * 6 + c] *= scaling[c];
  };
  auto grad_max_norm = [&](const std::vector<double>& xx, const double* g) {
    double ng[6];
    for (int c = 0; c < 6; ++c) ng[c] = -g[c];
    double pg[7];
    plus(xx.data(), ng, pg);
    double mx = 0.0;
    for (int i = 0; i < 7; ++i) mx = std::max(mx, std::fabs(xx[i] - pg[i]));
    return mx;
  };
  scale_jac(ev);
  double gmax = grad_max_norm(xv, ev.g);
  double x_norm = 0.0;
  for (int i = 0; i < 7; ++i) x_norm += xv[i] * xv[i];
  x_norm = std::sqrt(x_norm);
  double minimum_cost = std::numeric_limits<double>::max();
  std::vector<double> best = xv;
  int iteration = 0;
  bool step_successful = true;
  int consecutive_invalid = 0;
  int term = 0;
  double cand_cost = x_cost;
  std::vector<double> cand(7);
  double model_cost_change = 0.0;

  while (true) {
    // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (step_successful) {
      if (x_cost < minimum_cost) {
        minimum_cost = x_cost;
        best = xv;
      }
    }
    if (iteration >= max_iter) { term = 0; break; }
    if (step_successful && gmax <= gradient_tolerance) { term = 3; break; }
    if (radius <= min_trust_region_radius) { term = 5; break; }

    ++iteration;
    step_successful = false;
    // ComputeTrustRegionStep
    if (!reuse_diagonal) {
      for (int c = 0; c < 6; ++c) {
        double sq = 0.0;
        for (int i = 0; i < M; ++i) sq += ev.J[i * 6 + c] * ev.J[i * 6 + c];
        diagonal[c] = std::min(std::max(sq, min_lm_diagonal), max_lm_diagonal);
      }
    }
    double D[6];
    for (int c = 0; c < 6; ++c) D[c] = std::sqrt(diagonal[c] / radius);
    double y[6];
    bool solved = dense_qr_solve(ev.J, M, D, ev.f, y);
    reuse_diagonal = true;
    bool step_valid = false;
    double delta[6];
    if (solved) {
      double step[6];
      for (int c = 0; c < 6; ++c) step[c] = -y[c];
      // model_cost_change = -(J step)'(f + J step / 2)
      double mcc = 0.0;
      for (int i = 0; i < M; ++i) {
        double js = 0.0;
        for (int c = 0; c < 6; ++c) js += ev.J[i * 6 + c] * step[c];
        mcc += js * (ev.f[i] + js / 2.0);
      }
      model_cost_change = -mcc;
      step_valid = model_cost_change > 0.0;
      if (step_valid) {
        for (int c = 0; c < 6; ++c) delta[c] = step[c] * scaling[c];
        consecutive_invalid = 0;
      }
    }
    if (!step_valid) {
      // HandleInvalidStep
      s.invalid++;
      if (++consecutive_invalid >= max_consecutive_invalid) { term = 5; break; }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = true;
      continue;
    }
    // ComputeCandidatePointAndEvaluateCost
    plus(xv.data(), delta, cand.data());
    cand_cost = evaluate(fs, cand.data(), nullptr);
    // ParameterToleranceReached
    double step_norm = 0.0;
    for (int i = 0; i < 7; ++i) step_norm += (xv[i] - cand[i]) * (xv[i] - cand[i]);
    step_norm = std::sqrt(step_norm);
    if (step_norm <= parameter_tolerance * (x_norm + parameter_tolerance)) { term = 2; break; }
    // FunctionToleranceReached
    double cost_change = x_cost - cand_cost;
    if (std::fabs(cost_change) <= function_tolerance * x_cost) { term = 1; break; }
    // IsStepSuccessful (monotonic: StepQuality = relative decrease)
    double rel = (x_cost - cand_cost) / model_cost_change;
    if (rel > min_relative_decrease) {
      // HandleSuccessfulStep
      xv = cand;
      x_norm = 0.0;
      for (int i = 0; i < 7; ++i) x_norm += xv[i] * xv[i];
      x_norm = std::sqrt(x_norm);
      evaluate(fs, xv.data(), &ev);
      x_cost = ev.cost;
      scale_jac(ev);
      gmax = grad_max_norm(xv, ev.g);
      step_successful = true;
      s.successful++;
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3));
      radius = std::min(max_trust_region_radius, radius);
      decrease_factor = 2.0;
      reuse_diagonal = false;
    } else {
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = true;
    }
  }
  s.iterations = iteration;
  s.termination = term;
  s.final_cost = minimum_cost;
  for (int i = 0; i < 7; ++i) x[i] = best[i];
  if (st) *st = s;
  return 0;
}

// ---------------------------------------------------------------------------------------
// ScanRegistration::input (scan_registration.cpp:144-513), N_SCANS = 64 (KITTI launch)
// ---------------------------------------------------------------------------------------
struct ScanRegistration {
  int N_SCANS = 64;
  double MINIMUM_RANGE = 5.0;
  const double scanPeriod = 0.1;
  Cloud laserCloud, sharp, lessSharp, flat, lessFlat;
  std::vector<float> curvature;
  std::vector<int> sortInd, picked, label;
  double ms = 0;

  void input(const float* xyz, int n, int stride) {
    double t0 = now_ms();
    laserCloud.clear(); sharp.clear(); lessSharp.clear(); flat.clear(); lessFlat.clear();
    std::vector<Cloud> scans(N_SCANS);
    // removeNaNFromPointCloud + removeClosedPointCloud (:168-176, :107-141)
    std::vector<Pt> in;
    in.reserve(n);
    const float thres = static_cast<float>(MINIMUM_RANGE);
    for (int i = 0; i < n; ++i) {
      float x = xyz[(size_t)i * stride], y = xyz[(size_t)i * stride + 1], z = xyz[(size_t)i * stride + 2];
      if (!std::isfinite(x) || !std::isfinite(y) || !std::isfinite(z)) continue;
      if (x * x + y * y + z * z < thres * thres) continue;
      in.push_back({x, y, z, 0.f});
    }
    int cloudSize = static_cast<int>(in.size());
    std::vector<int> scanStartInd(N_SCANS, 0), scanEndInd(N_SCANS, 0);
    if (cloudSize == 0) {
      ms = now_ms() - t0;
      return;
    }
    float startOri = -std::atan2(in[0].y, in[0].x);
    float endOri = -std::atan2(in[cloudSize - 1].y, in[cloudSize - 1].x) + 2 * M_PI;
    if (endOri - startOri > 3 * M_PI) endOri -= 2 * M_PI;
    else if (endOri - startOri < M_PI) endOri += 2 * M_PI;
    bool halfPassed = false;
    int count = cloudSize;
    for (int i = 0; i < cloudSize; ++i) {
      Pt point{in[i].x, in[i].y, in[i].z, 0.f};
      float angle = std::atan(point.z / std::sqrt(point.x * point.x + point.y * point.y)) * 180 / M_PI;
      int scanID = 0;
      if (N_SCANS == 16) {
        scanID = int((angle + 15) / 2 + 0.5);
        if (scanID > (N_SCANS - 1) || scanID < 0) { count--; continue; }
      } else if (N_SCANS == 32) {
        scanID = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
        if (scanID > (N_SCANS - 1) || scanID < 0) { count--; continue; }
      } else {
        if (angle >= -8.83) scanID = int((2 - angle) * 3.0 + 0.5);
        else scanID = N_SCANS / 2 + int((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || scanID > 50 || scanID < 0) { count--; continue; }
      }
      float ori = -std::atan2(point.y, point.x);
      if (!halfPassed) {
        if (ori < startOri - M_PI / 2) ori += 2 * M_PI;
        else if (ori > startOri + M_PI * 3 / 2) ori -= 2 * M_PI;
        if (ori - startOri > M_PI) halfPassed = true;
      } else {
        ori += 2 * M_PI;
        if (ori < endOri - M_PI * 3 / 2) ori += 2 * M_PI;
        else if (ori > endOri + M_PI / 2) ori -= 2 * M_PI;
      }
      float relTime = (ori - startOri) / (endOri - startOri);
      point.intensity = scanID + scanPeriod * relTime;
      scans[scanID].push_back(point);
    }
    cloudSize = count;
    for (int i = 0; i < N_SCANS; ++i) {
      scanStartInd[i] = static_cast<int>(laserCloud.size()) + 5;
      laserCloud.insert(laserCloud.end(), scans[i].begin(), scans[i].end());
      scanEndInd[i] = static_cast<int>(laserCloud.size()) - 6;
    }
    curvature.assign(cloudSize, 0.f);
    sortInd.assign(cloudSize, 0);
    picked.assign(cloudSize, 0);
    label.assign(cloudSize, 0);
    const Cloud& L = laserCloud;
    for (int i = 5; i < cloudSize - 5; i++) {
      float diffX = L[i - 5].x + L[i - 4].x + L[i - 3].x + L[i - 2].x + L[i - 1].x - 10 * L[i].x +
                    L[i + 1].x + L[i + 2].x + L[i + 3].x + L[i + 4].x + L[i + 5].x;
      float diffY = L[i - 5].y + L[i - 4].y + L[i - 3].y + L[i - 2].y + L[i - 1].y - 10 * L[i].y +
                    L[i + 1].y + L[i + 2].y + L[i + 3].y + L[i + 4].y + L[i + 5].y;
      float diffZ = L[i - 5].z + L[i - 4].z + L[i - 3].z + L[i - 2].z + L[i - 1].z - 10 * L[i].z +
                    L[i + 1].z + L[i + 2].z + L[i + 3].z + L[i + 4].z + L[i + 5].z;
      curvature[i] = diffX * diffX + diffY * diffY + diffZ * diffZ;
      sortInd[i] = i;
      picked[i] = 0;
      label[i] = 0;
    }
    auto suppress = [&](int ind) {
      for (int l = 1; l <= 5; l++) {
        float dX = L[ind + l].x - L[ind + l - 1].x;
        float dY = L[ind + l].y - L[ind + l - 1].y;
        float dZ = L[ind + l].z - L[ind + l - 1].z;
        if (dX * dX + dY * dY + dZ * dZ > 0.05) break;
        picked[ind + l] = 1;
      }
      for (int l = -1; l >= -5; l--) {
        float dX = L[ind + l].x - L[ind + l + 1].x;
        float dY = L[ind + l].y - L[ind + l + 1].y;
        float dZ = L[ind + l].z - L[ind + l + 1].z;
        if (dX * dX + dY * dY + dZ * dZ > 0.05) break;
        picked[ind + l] = 1;
      }
    };
    for (int i = 0; i < N_SCANS; i++) {
      if (scanEndInd[i] - scanStartInd[i] < 6) continue;
      Cloud lessFlatScan;
      for (int j = 0; j < 6; j++) {
        int sp = scanStartInd[i] + (scanEndInd[i] - scanStartInd[i]) * j / 6;
        int ep = scanStartInd[i] + (scanEndInd[i] - scanStartInd[i]) * (j + 1) / 6 - 1;
        std::sort(sortInd.begin() + sp, sortInd.begin() + ep + 1,
                  [&](const int& a, const int& b) { return curvature[a] < curvature[b]; });
        int largestPickedNum = 0;
        for (int k = ep; k >= sp; k--) {
          int ind = sortInd[k];
          if (picked[ind] == 0 && curvature[ind] > 0.1) {
            largestPickedNum++;
            if (largestPickedNum <= 2) {
              label[ind] = 2;
              sharp.push_back(L[ind]);
              lessSharp.push_back(L[ind]);
            } else if (largestPickedNum <= 20) {
              label[ind] = 1;
              lessSharp.push_back(L[ind]);
            } else {
              break;
            }
            picked[ind] = 1;
            suppress(ind);
          }
        }
        int smallestPickedNum = 0;
        for (int k = sp; k <= ep; k++) {
          int ind = sortInd[k];
          if (picked[ind] == 0 && curvature[ind] < 0.1) {
            label[ind] = -1;
            flat.push_back(L[ind]);
            smallestPickedNum++;
            if (smallestPickedNum >= 4) break;
            picked[ind] = 1;
            suppress(ind);
          }
        }
        for (int k = sp; k <= ep; k++)
          if (label[k] <= 0) lessFlatScan.push_back(L[k]);
      }
      Cloud ds = voxel_grid(lessFlatScan, 0.2f);
      lessFlat.insert(lessFlat.end(), ds.begin(), ds.end());
    }
    ms = now_ms() - t0;
  }
};

// ---------------------------------------------------------------------------------------
// LaserOdometry::solveLO (laser_odometry.cpp:199-584).  detach_VO_LO = true unless a VO prior
// is set for the frame: then (!detach_VO_LO, :237-250) every outer round starts from it
// (para_q / para_t overwritten with velo_last_VOT_velo_curr before the round's problem).
// ---------------------------------------------------------------------------------------
struct LaserOdometry {
  bool has_prior = false;
  double prior_q[4] = {0, 0, 0, 1}, prior_t[3] = {0, 0, 0};
  const double DISTANCE_SQ_THRESHOLD = 25;
  const double NEARBY_SCAN = 2.5;
  int mapping_skip_frame = 1;
  bool systemInited = false;
  Cloud fullRes, sharp, lessSharp, flat, lessFlat;
  Cloud cornerLast, surfLast;
  KdTree kdCorner, kdSurf;
  Quat q_w{0, 0, 0, 1};
  V3 t_w{0, 0, 0};
  double para_q[4] = {0, 0, 0, 1};
  double para_t[3] = {0, 0, 0};
  int frameCount = 0;
  int corr[4] = {0, 0, 0, 0};
  oracle_lm_stats lm[2] = {};
  double ms = 0;

  void solve() {
    double t0 = now_ms();
    if (!systemInited) {
      systemInited = true;
    } else {
      for (int opti = 0; opti < 2; ++opti) {
        if (has_prior) {  // laser_odometry.cpp:237-250
          for (int i = 0; i < 4; ++i) para_q[i] = prior_q[i];
          for (int i = 0; i < 3; ++i) para_t[i] = prior_t[i];
        }
        std::vector<Factor> fs;
        int corner_c = 0, plane_c = 0;
        Quat q{para_q[0], para_q[1], para_q[2], para_q[3]};
        V3 t{para_t[0], para_t[1], para_t[2]};
        // TransformToStart with s = 1 (slerp(1, q) == q)
        auto toStart = [&](const Pt& p) {
          V3 r = qrot(q, V3{p.x, p.y, p.z});
          return Pt{static_cast<float>(r.x + t.x), static_cast<float>(r.y + t.y),
                    static_cast<float>(r.z + t.z), p.intensity};
        };
        int idx1;
        float d1;
        for (const Pt& cp : sharp) {
          Pt sel = toStart(cp);
          int closest = -1, ind2 = -1;
          if (kdCorner.knn(sel.x, sel.y, sel.z, 1, &idx1, &d1) == 1 && d1 < DISTANCE_SQ_THRESHOLD) {
            closest = idx1;
            int cid = int(cornerLast[closest].intensity);
            double minD2 = DISTANCE_SQ_THRESHOLD;
            for (int j = closest + 1; j < (int)cornerLast.size(); ++j) {
              if (int(cornerLast[j].intensity) <= cid) continue;
              if (int(cornerLast[j].intensity) > (cid + NEARBY_SCAN)) break;
              double d = (cornerLast[j].x - sel.x) * (cornerLast[j].x - sel.x) +
                         (cornerLast[j].y - sel.y) * (cornerLast[j].y - sel.y) +
                         (cornerLast[j].z - sel.z) * (cornerLast[j].z - sel.z);
              if (d < minD2) { minD2 = d; ind2 = j; }
            }
            for (int j = closest - 1; j >= 0; --j) {
              if (int(cornerLast[j].intensity) >= cid) continue;
              if (int(cornerLast[j].intensity) < (cid - NEARBY_SCAN)) break;
              double d = (cornerLast[j].x - sel.x) * (cornerLast[j].x - sel.x) +
                         (cornerLast[j].y - sel.y) * (cornerLast[j].y - sel.y) +
                         (cornerLast[j].z - sel.z) * (cornerLast[j].z - sel.z);
              if (d < minD2) { minD2 = d; ind2 = j; }
            }
          }
          if (ind2 >= 0) {
            Factor F{1, {cp.x, cp.y, cp.z},
                     {cornerLast[closest].x, cornerLast[closest].y, cornerLast[closest].z},
                     {cornerLast[ind2].x, cornerLast[ind2].y, cornerLast[ind2].z}};
            fs.push_back(F);
            corner_c++;
          }
        }
        for (const Pt& fp : flat) {
          Pt sel = toStart(fp);
          int closest = -1, ind2 = -1, ind3 = -1;
          if (kdSurf.knn(sel.x, sel.y, sel.z, 1, &idx1, &d1) == 1 && d1 < DISTANCE_SQ_THRESHOLD) {
            closest = idx1;
            int cid = int(surfLast[closest].intensity);
            double minD2 = DISTANCE_SQ_THRESHOLD, minD3 = DISTANCE_SQ_THRESHOLD;
            for (int j = closest + 1; j < (int)surfLast.size(); ++j) {
              if (int(surfLast[j].intensity) > (cid + NEARBY_SCAN)) break;
              double d = (surfLast[j].x - sel.x) * (surfLast[j].x - sel.x) +
                         (surfLast[j].y - sel.y) * (surfLast[j].y - sel.y) +
                         (surfLast[j].z - sel.z) * (surfLast[j].z - sel.z);
              if (int(surfLast[j].intensity) <= cid && d < minD2) { minD2 = d; ind2 = j; }
              else if (int(surfLast[j].intensity) > cid && d < minD3) { minD3 = d; ind3 = j; }
            }
            for (int j = closest - 1; j >= 0; --j) {
              if (int(surfLast[j].intensity) < (cid - NEARBY_SCAN)) break;
              double d = (surfLast[j].x - sel.x) * (surfLast[j].x - sel.x) +
                         (surfLast[j].y - sel.y) * (surfLast[j].y - sel.y) +
                         (surfLast[j].z - sel.z) * (surfLast[j].z - sel.z);
              if (int(surfLast[j].intensity) >= cid && d < minD2) { minD2 = d; ind2 = j; }
              else if (int(surfLast[j].intensity) < cid && d < minD3) { minD3 = d; ind3 = j; }
            }
            if (ind2 >= 0 && ind3 >= 0) {
              // LidarPlaneFactor ctor: ljm = (j - l) x (j - m), normalized (lidarFactor.hpp:73-74)
              V3 j{surfLast[closest].x, surfLast[closest].y, surfLast[closest].z};
              V3 l{surfLast[ind2].x, surfLast[ind2].y, surfLast[ind2].z};
              V3 m{surfLast[ind3].x, surfLast[ind3].y, surfLast[ind3].z};
              V3 n = cross(V3{j.x - l.x, j.y - l.y, j.z - l.z}, V3{j.x - m.x, j.y - m.y, j.z - m.z});
              double nn = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
              if (nn > 0) n = {n.x / nn, n.y / nn, n.z / nn};
              Factor F{2, {fp.x, fp.y, fp.z}, {j.x, j.y, j.z}, {n.x, n.y, n.z}};
              fs.push_back(F);
              plane_c++;
            }
          }
        }
        corr[opti * 2] = corner_c;
        corr[opti * 2 + 1] = plane_c;
        double x[7] = {para_q[0], para_q[1], para_q[2], para_q[3], para_t[0], para_t[1], para_t[2]};
        lm_solve(fs, x, 4, &lm[opti]);
        for (int i = 0; i < 4; ++i) para_q[i] = x[i];
        for (int i = 0; i < 3; ++i) para_t[i] = x[4 + i];
      }
      Quat qlc{para_q[0], para_q[1], para_q[2], para_q[3]};
      V3 tr = qrot(q_w, V3{para_t[0], para_t[1], para_t[2]});
      t_w = {t_w.x + tr.x, t_w.y + tr.y, t_w.z + tr.z};
      q_w = qmul(q_w, qlc);
    }
    std::swap(cornerLast, lessSharp);
    std::swap(surfLast, lessFlat);
    kdCorner.build(&cornerLast);
    kdSurf.build(&surfLast);
    frameCount++;
    ms = now_ms() - t0;
  }
};

// ---------------------------------------------------------------------------------------
// LaserMapping (laser_mapping.cpp:147-814) — 21 x 21 x 11 cube ring buffer of 50 m cubes
// ---------------------------------------------------------------------------------------
struct LaserMapping {
  static constexpr int W = 21, H = 21, D = 11, N = W * H * D;
  int cenW = 10, cenH = 10, cenD = 5;
  std::vector<Cloud> cornerArr = std::vector<Cloud>(N), surfArr = std::vector<Cloud>(N);
  float lineRes = 0.4f, planeRes = 0.8f;
  double parameters[7] = {0, 0, 0, 1, 0, 0, 0};
  Quat q_wmap_wodom{0, 0, 0, 1};
  V3 t_wmap_wodom{0, 0, 0};
  Quat q_wodom{0, 0, 0, 1};
  V3 t_wodom{0, 0, 0};
  Cloud cornerLast, surfLast, fullRes;
  bool skip = false;
  int frameCount = 0;
  oracle_map_stats st{};
  std::vector<Factor> factors[2];
  double roundPose[2][7];

  Quat qw() const { return {parameters[0], parameters[1], parameters[2], parameters[3]}; }
  V3 tw() const { return {parameters[4], parameters[5], parameters[6]}; }

  void input(const Cloud& c, const Cloud& s, const Cloud& f, const Quat& qo, const V3& to, bool sk) {
    skip = sk;
    if (!skip) {
      cornerLast = c;
      surfLast = s;
      fullRes = f;
    }
    q_wodom = qo;
    t_wodom = to;
    if (!skip) {
      Quat q = qmul(q_wmap_wodom, q_wodom);
      V3 r = qrot(q_wmap_wodom, t_wodom);
      parameters[0] = q.x; parameters[1] = q.y; parameters[2] = q.z; parameters[3] = q.w;
      parameters[4] = r.x + t_wmap_wodom.x;
      parameters[5] = r.y + t_wmap_wodom.y;
      parameters[6] = r.z + t_wmap_wodom.z;
    }
  }

  Pt toMap(const Pt& p) const {
    V3 r = qrot(qw(), V3{p.x, p.y, p.z});
    return {static_cast<float>(r.x + parameters[4]), static_cast<float>(r.y + parameters[5]),
            static_cast<float>(r.z + parameters[6]), p.intensity};
  }

  static int cubeOf(double v, int cen) {
    int c = int((v + 25.0) / 50.0) + cen;
    if (v + 25.0 < 0) c--;
    return c;
  }

  void shiftCubes(int axis, int dir) {
    // dir +1: content moves to higher index (centerCube < 3), the last slab wraps & clears
    const int dims[3] = {W, H, D};
    const int n = dims[axis];
    int o1 = (axis + 1) % 3, o2 = (axis + 2) % 3;
    for (int a = 0; a < dims[o1]; ++a)
      for (int b = 0; b < dims[o2]; ++b) {
        auto idx = [&](int v) {
          int c[3];
          c[axis] = v; c[o1] = a; c[o2] = b;
          return c[0] + W * c[1] + W * H * c[2];
        };
        if (dir > 0) {
          Cloud cc = std::move(cornerArr[idx(n - 1)]), ss = std::move(surfArr[idx(n - 1)]);
          for (int v = n - 1; v >= 1; --v) {
            cornerArr[idx(v)] = std::move(cornerArr[idx(v - 1)]);
            surfArr[idx(v)] = std::move(surfArr[idx(v - 1)]);
          }
          cc.clear(); ss.clear();
          cornerArr[idx(0)] = std::move(cc);
          surfArr[idx(0)] = std::move(ss);
        } else {
          Cloud cc = std::move(cornerArr[idx(0)]), ss = std::move(surfArr[idx(0)]);
          for (int v = 0; v < n - 1; ++v) {
            cornerArr[idx(v)] = std::move(cornerArr[idx(v + 1)]);
            surfArr[idx(v)] = std::move(surfArr[idx(v + 1)]);
          }
          cc.clear(); ss.clear();
          cornerArr[idx(n - 1)] = std::move(cc);
          surfArr[idx(n - 1)] = std::move(ss);
        }
      }
  }

  void solve() {
    double t_whole = now_ms();
    st = oracle_map_stats{};
    factors[0].clear();
    factors[1].clear();
    int cI = cubeOf(parameters[4], cenW), cJ = cubeOf(parameters[5], cenH), cK = cubeOf(parameters[6], cenD);
    while (cI < 3) { shiftCubes(0, +1); cI++; cenW++; }
    while (cI >= W - 3) { shiftCubes(0, -1); cI--; cenW--; }
    while (cJ < 3) { shiftCubes(1, +1); cJ++; cenH++; }
    while (cJ >= H - 3) { shiftCubes(1, -1); cJ--; cenH--; }
    while (cK < 3) { shiftCubes(2, +1); cK++; cenD++; }
    while (cK >= D - 3) { shiftCubes(2, -1); cK--; cenD--; }
    st.center[0] = cI; st.center[1] = cJ; st.center[2] = cK;
    int valid[125];
    int validNum = 0;
    for (int i = cI - 2; i <= cI + 2; i++)
      for (int j = cJ - 2; j <= cJ + 2; j++)
        for (int k = cK - 1; k <= cK + 1; k++)
          if (i >= 0 && i < W && j >= 0 && j < H && k >= 0 && k < D) valid[validNum++] = i + W * j + W * H * k;
    st.valid_num = validNum;
    Cloud cornerMap, surfMap;
    for (int i = 0; i < validNum; i++) {
      cornerMap.insert(cornerMap.end(), cornerArr[valid[i]].begin(), cornerArr[valid[i]].end());
      surfMap.insert(surfMap.end(), surfArr[valid[i]].begin(), surfArr[valid[i]].end());
    }
    Cloud cornerStack = voxel_grid(cornerLast, lineRes);
    Cloud surfStack = voxel_grid(surfLast, planeRes);
    st.corner_stack = static_cast<int>(cornerStack.size());
    st.surf_stack = static_cast<int>(surfStack.size());
    st.corner_map = static_cast<int>(cornerMap.size());
    st.surf_map = static_cast<int>(surfMap.size());
    if (cornerMap.size() > 10 && surfMap.size() > 50) {
      double t_opt = now_ms();
      st.optimized = 1;
      KdTree kdC, kdS;
      kdC.build(&cornerMap);
      kdS.build(&surfMap);
      int idx[5];
      float d2[5];
      for (int it = 0; it < 2; ++it) {
        for (int i = 0; i < 7; ++i) roundPose[it][i] = parameters[i];
        std::vector<Factor>& fs = factors[it];
        int corner_num = 0, surf_num = 0;
        for (const Pt& po : cornerStack) {
          Pt sel = toMap(po);
          if (kdC.knn(sel.x, sel.y, sel.z, 5, idx, d2) < 5) continue;
          if (d2[4] < 1.0) {
            Pt nb[5];
            for (int j = 0; j < 5; ++j) nb[j] = cornerMap[idx[j]];
            V3 a, b;
            if (edge_from_nbrs(nb, a, b)) {
              fs.push_back(Factor{1, {po.x, po.y, po.z}, {a.x, a.y, a.z}, {b.x, b.y, b.z}});
              corner_num++;
            }
          }
        }
        for (const Pt& po : surfStack) {
          Pt sel = toMap(po);
          if (kdS.knn(sel.x, sel.y, sel.z, 5, idx, d2) < 5) continue;
          if (d2[4] < 1.0) {
            Pt nb[5];
            for (int j = 0; j < 5; ++j) nb[j] = surfMap[idx[j]];
            V3 n;
            double d;
            if (plane_from_nbrs(nb, n, d)) {
              fs.push_back(Factor{3, {po.x, po.y, po.z}, {n.x, n.y, n.z}, {d, 0, 0}});
              surf_num++;
            }
          }
        }
        st.corner_num[it] = corner_num;
        st.surf_num[it] = surf_num;
        lm_solve(fs, parameters, 4, &st.lm[it]);
      }
      st.ms_opt = now_ms() - t_opt;
    }
    // transformUpdate (:147-151)
    q_wmap_wodom = qmul(qw(), qinv(q_wodom));
    V3 r = qrot(q_wmap_wodom, t_wodom);
    t_wmap_wodom = {parameters[4] - r.x, parameters[5] - r.y, parameters[6] - r.z};
    // insert (:741-788)
    for (const Pt& p : cornerStack) {
      Pt sel = toMap(p);
      int ci = cubeOf(sel.x, cenW), cj = cubeOf(sel.y, cenH), ck = cubeOf(sel.z, cenD);
      if (ci >= 0 && ci < W && cj >= 0 && cj < H && ck >= 0 && ck < D) cornerArr[ci + W * cj + W * H * ck].push_back(sel);
    }
    for (const Pt& p : surfStack) {
      Pt sel = toMap(p);
      int ci = cubeOf(sel.x, cenW), cj = cubeOf(sel.y, cenH), ck = cubeOf(sel.z, cenD);
      if (ci >= 0 && ci < W && cj >= 0 && cj < H && ck >= 0 && ck < D) surfArr[ci + W * cj + W * H * ck].push_back(sel);
    }
    // re-voxelize the submap cubes (:795-808)
    for (int i = 0; i < validNum; i++) {
      int ind = valid[i];
      cornerArr[ind] = voxel_grid(cornerArr[ind], lineRes);
      surfArr[ind] = voxel_grid(surfArr[ind], planeRes);
    }
    frameCount++;
    st.ms_total = now_ms() - t_whole;
  }
};

}  // namespace oracle

// =========================================================================================
// C API
// =========================================================================================
using namespace oracle;

static Cloud to_cloud(const float* p, int32_t n) {
  Cloud c(n > 0 ? n : 0);
  if (n > 0) std::memcpy(c.data(), p, sizeof(Pt) * n);
  return c;
}
static void from_cloud(const Cloud& c, float* out) {
  if (!c.empty()) std::memcpy(out, c.data(), sizeof(Pt) * c.size());
}
static std::vector<Factor> to_factors(const double* f, int32_t nf) {
  std::vector<Factor> fs(nf);
  for (int i = 0; i < nf; ++i) {
    const double* r = f + (size_t)i * 10;
    fs[i].type = static_cast<int>(r[0]);
    for (int k = 0; k < 3; ++k) {
      fs[i].p[k] = r[1 + k];
      fs[i].a[k] = r[4 + k];
      fs[i].b[k] = r[7 + k];
    }
  }
  return fs;
}

extern "C" {

int32_t oracle_voxel_grid(const float* in, int32_t n, float leaf, float* out) {
  Cloud c = voxel_grid(to_cloud(in, n), leaf);
  from_cloud(c, out);
  return static_cast<int32_t>(c.size());
}

int32_t oracle_set_voxel_order(int32_t order) {
  const int32_t old = g_voxel_order;
  g_voxel_order = order ? 1 : 0;
  return old;
}

int32_t oracle_std_sort_perm(const uint32_t* keys, int32_t n, int32_t* perm) {
  std::vector<CloudPointIndexIdx> v(n);
  for (int32_t i = 0; i < n; ++i) v[i] = {keys[i], static_cast<uint32_t>(i)};
  std::sort(v.begin(), v.end(), std::less<CloudPointIndexIdx>());
  for (int32_t i = 0; i < n; ++i) perm[i] = static_cast<int32_t>(v[i].cloud_point_index);
  return n;
}

int32_t oracle_knn(const float* pts, int32_t n, const float* q, int32_t nq, int32_t k,
                   int32_t* idx, float* d2) {
  Cloud c = to_cloud(pts, n);
  KdTree kd;
  kd.build(&c);
  std::vector<int> ii(k);
  std::vector<float> dd(k);
  for (int i = 0; i < nq; ++i) {
    int cnt = kd.knn(q[i * 4], q[i * 4 + 1], q[i * 4 + 2], k, ii.data(), dd.data());
    for (int j = 0; j < k; ++j) {
      idx[(size_t)i * k + j] = j < cnt ? ii[j] : -1;
      d2[(size_t)i * k + j] = j < cnt ? dd[j] : INFINITY;
    }
  }
  return 0;
}

int32_t oracle_edge_from_nbrs(const float* nbr, double* a, double* b) {
  Pt nb[5];
  std::memcpy(nb, nbr, sizeof(nb));
  V3 pa, pb;
  if (!edge_from_nbrs(nb, pa, pb)) return 0;
  a[0] = pa.x; a[1] = pa.y; a[2] = pa.z;
  b[0] = pb.x; b[1] = pb.y; b[2] = pb.z;
  return 1;
}

int32_t oracle_plane_from_nbrs(const float* nbr, double* n, double* d) {
  Pt nb[5];
  std::memcpy(nb, nbr, sizeof(nb));
  V3 nn;
  double dd;
  bool ok = plane_from_nbrs(nb, nn, dd);
  n[0] = nn.x; n[1] = nn.y; n[2] = nn.z;
  *d = dd;
  return ok ? 1 : 0;
}

int32_t oracle_lm_solve(const double* factors, int32_t nf, double* x, int32_t max_iter,
                        oracle_lm_stats* st) {
  return lm_solve(to_factors(factors, nf), x, max_iter, st);
}

int32_t oracle_vo_solve(const double* factors, int32_t nf, double* x6, int32_t max_iter, oracle_lm_stats* st) {
  double x[7] = {x6[0], x6[1], x6[2], x6[3], x6[4], x6[5], 0.0};
  g_plus_euclid = true;
  const int32_t rc = lm_solve(to_factors(factors, nf), x, max_iter, st);
  g_plus_euclid = false;
  for (int i = 0; i < 6; ++i) x6[i] = x[i];
  return rc;
}

int32_t oracle_vo_normal_eq(const double* factors, int32_t nf, const double* x6, double* cost, double* jtj,
                            double* jtr) {
  const double x[7] = {x6[0], x6[1], x6[2], x6[3], x6[4], x6[5], 0.0};
  Eval ev;
  evaluate(to_factors(factors, nf), x, &ev);
  const int M = static_cast<int>(ev.f.size());
  *cost = ev.cost;
  for (int a = 0; a < 6; ++a) {
    jtr[a] = ev.g[a];
    for (int b = 0; b < 6; ++b) {
      double v = 0.0;
      for (int i = 0; i < M; ++i) v += ev.J[i * 6 + a] * ev.J[i * 6 + b];
      jtj[a * 6 + b] = v;
    }
  }
  return M;
}

int32_t oracle_lm_normal_eq(const double* factors, int32_t nf, const double* x, double* cost,
                            double* jtj36, double* jtr6) {
  std::vector<Factor> fs = to_factors(factors, nf);
  Eval ev;
  evaluate(fs, x, &ev);
  *cost = ev.cost;
  const int M = static_cast<int>(ev.f.size());
  for (int a = 0; a < 6; ++a) {
    jtr6[a] = ev.g[a];
    for (int b = 0; b < 6; ++b) {
      double s = 0;
      for (int i = 0; i < M; ++i) s += ev.J[i * 6 + a] * ev.J[i * 6 + b];
      jtj36[a * 6 + b] = s;
    }
  }
  return M;
}

// ---- scan registration
struct oracle_scanreg {
  ScanRegistration s;
};
oracle_scanreg* oracle_scanreg_create(int32_t n_scans, double minimum_range) {
  auto* h = new oracle_scanreg;
  h->s.N_SCANS = n_scans;
  h->s.MINIMUM_RANGE = minimum_range;
  return h;
}
void oracle_scanreg_destroy(oracle_scanreg* h) { delete h; }
int32_t oracle_scanreg_input(oracle_scanreg* h, const float* xyz, int32_t n, int32_t stride) {
  h->s.input(xyz, n, stride);
  return 0;
}
static const Cloud& sr_cloud(oracle_scanreg* h, int which) {
  switch (which) {
    case 0: return h->s.laserCloud;
    case 1: return h->s.sharp;
    case 2: return h->s.lessSharp;
    case 3: return h->s.flat;
    default: return h->s.lessFlat;
  }
}
int32_t oracle_scanreg_count(oracle_scanreg* h, int32_t which) {
  return static_cast<int32_t>(sr_cloud(h, which).size());
}
int32_t oracle_scanreg_copy(oracle_scanreg* h, int32_t which, float* out) {
  from_cloud(sr_cloud(h, which), out);
  return static_cast<int32_t>(sr_cloud(h, which).size());
}
int32_t oracle_scanreg_curvature(oracle_scanreg* h, float* curv, int32_t* label) {
  int n = static_cast<int>(h->s.curvature.size());
  for (int i = 0; i < n; ++i) {
    curv[i] = h->s.curvature[i];
    label[i] = h->s.label[i];
  }
  return n;
}
double oracle_scanreg_ms(oracle_scanreg* h) { return h->s.ms; }

// ---- odometry
struct oracle_odom {
  LaserOdometry o;
};
oracle_odom* oracle_odom_create(int32_t mapping_skip_frame) {
  auto* h = new oracle_odom;
  h->o.mapping_skip_frame = mapping_skip_frame;
  return h;
}
void oracle_odom_destroy(oracle_odom* h) { delete h; }
int32_t oracle_odom_input(oracle_odom* h, const float* full, int32_t nfull, const float* sharp,
                          int32_t nsharp, const float* less_sharp, int32_t nless_sharp,
                          const float* flat, int32_t nflat, const float* less_flat,
                          int32_t nless_flat) {
  h->o.fullRes = to_cloud(full, nfull);
  h->o.sharp = to_cloud(sharp, nsharp);
  h->o.lessSharp = to_cloud(less_sharp, nless_sharp);
  h->o.flat = to_cloud(flat, nflat);
  h->o.lessFlat = to_cloud(less_flat, nless_flat);
  return 0;
}
int32_t oracle_odom_solve(oracle_odom* h) {
  h->o.solve();
  return 0;
}
int32_t oracle_odom_set_prior(oracle_odom* h, const double* q, const double* t) {
  h->o.has_prior = q && t;
  if (h->o.has_prior) {
    for (int i = 0; i < 4; ++i) h->o.prior_q[i] = q[i];
    for (int i = 0; i < 3; ++i) h->o.prior_t[i] = t[i];
  }
  return 0;
}
int32_t oracle_odom_output(oracle_odom* h, double* q_w, double* t_w, double* q_lc, double* t_lc) {
  q_w[0] = h->o.q_w.x; q_w[1] = h->o.q_w.y; q_w[2] = h->o.q_w.z; q_w[3] = h->o.q_w.w;
  t_w[0] = h->o.t_w.x; t_w[1] = h->o.t_w.y; t_w[2] = h->o.t_w.z;
  for (int i = 0; i < 4; ++i) q_lc[i] = h->o.para_q[i];
  for (int i = 0; i < 3; ++i) t_lc[i] = h->o.para_t[i];
  return (h->o.frameCount % h->o.mapping_skip_frame == 0) ? 0 : 1;
}
static const Cloud& od_cloud(oracle_odom* h, int which) {
  return which == 0 ? h->o.cornerLast : (which == 1 ? h->o.surfLast : h->o.fullRes);
}
int32_t oracle_odom_count(oracle_odom* h, int32_t which) {
  return static_cast<int32_t>(od_cloud(h, which).size());
}
int32_t oracle_odom_copy(oracle_odom* h, int32_t which, float* out) {
  from_cloud(od_cloud(h, which), out);
  return static_cast<int32_t>(od_cloud(h, which).size());
}
int32_t oracle_odom_stats(oracle_odom* h, int32_t* corr, oracle_lm_stats* lm) {
  for (int i = 0; i < 4; ++i) corr[i] = h->o.corr[i];
  lm[0] = h->o.lm[0];
  lm[1] = h->o.lm[1];
  return 0;
}
double oracle_odom_ms(oracle_odom* h) { return h->o.ms; }

// ---- mapping
struct oracle_map {
  LaserMapping m;
};
oracle_map* oracle_map_create(float line_res, float plane_res) {
  auto* h = new oracle_map;
  h->m.lineRes = line_res;
  h->m.planeRes = plane_res;
  return h;
}
void oracle_map_destroy(oracle_map* h) { delete h; }
int32_t oracle_map_input(oracle_map* h, const float* corner, int32_t nc, const float* surf,
                         int32_t ns, const float* full, int32_t nf, const double* q_wodom,
                         const double* t_wodom, int32_t skip_frame) {
  h->m.input(to_cloud(corner, nc), to_cloud(surf, ns), to_cloud(full, nf),
             Quat{q_wodom[0], q_wodom[1], q_wodom[2], q_wodom[3]},
             V3{t_wodom[0], t_wodom[1], t_wodom[2]}, skip_frame != 0);
  return 0;
}
int32_t oracle_map_solve(oracle_map* h) {
  if (!h->m.skip) h->m.solve();
  return 0;
}
int32_t oracle_map_pose(oracle_map* h, double* q_w, double* t_w) {
  for (int i = 0; i < 4; ++i) q_w[i] = h->m.parameters[i];
  for (int i = 0; i < 3; ++i) t_w[i] = h->m.parameters[4 + i];
  return 0;
}
int32_t oracle_map_get_stats(oracle_map* h, oracle_map_stats* st) {
  *st = h->m.st;
  return 0;
}
int32_t oracle_map_get_state(oracle_map* h, int32_t* cen, double* q, double* t) {
  cen[0] = h->m.cenW; cen[1] = h->m.cenH; cen[2] = h->m.cenD;
  q[0] = h->m.q_wmap_wodom.x; q[1] = h->m.q_wmap_wodom.y; q[2] = h->m.q_wmap_wodom.z; q[3] = h->m.q_wmap_wodom.w;
  t[0] = h->m.t_wmap_wodom.x; t[1] = h->m.t_wmap_wodom.y; t[2] = h->m.t_wmap_wodom.z;
  return 0;
}
int32_t oracle_map_set_state(oracle_map* h, const int32_t* cen, const double* q, const double* t) {
  h->m.cenW = cen[0]; h->m.cenH = cen[1]; h->m.cenD = cen[2];
  h->m.q_wmap_wodom = {q[0], q[1], q[2], q[3]};
  h->m.t_wmap_wodom = {t[0], t[1], t[2]};
  return 0;
}
int32_t oracle_map_cube_count(oracle_map* h, int32_t which, int32_t cube) {
  if (cube < 0 || cube >= LaserMapping::N) return -1;
  return static_cast<int32_t>((which == 0 ? h->m.cornerArr : h->m.surfArr)[cube].size());
}
int32_t oracle_map_cube_copy(oracle_map* h, int32_t which, int32_t cube, float* out) {
  if (cube < 0 || cube >= LaserMapping::N) return -1;
  const Cloud& c = (which == 0 ? h->m.cornerArr : h->m.surfArr)[cube];
  from_cloud(c, out);
  return static_cast<int32_t>(c.size());
}
int32_t oracle_map_cube_set(oracle_map* h, int32_t which, int32_t cube, const float* pts, int32_t n) {
  if (cube < 0 || cube >= LaserMapping::N) return -1;
  (which == 0 ? h->m.cornerArr : h->m.surfArr)[cube] = to_cloud(pts, n);
  return n;
}
int32_t oracle_map_factor_count(oracle_map* h, int32_t round) {
  return static_cast<int32_t>(h->m.factors[round & 1].size());
}
int32_t oracle_map_factors(oracle_map* h, int32_t round, double* out) {
  const auto& fs = h->m.factors[round & 1];
  for (size_t i = 0; i < fs.size(); ++i) {
    double* r = out + i * 10;
    r[0] = fs[i].type;
    for (int k = 0; k < 3; ++k) {
      r[1 + k] = fs[i].p[k];
      r[4 + k] = fs[i].a[k];
      r[7 + k] = fs[i].b[k];
    }
  }
  return static_cast<int32_t>(fs.size());
}
int32_t oracle_map_round_pose(oracle_map* h, int32_t round, double* x7) {
  for (int i = 0; i < 7; ++i) x7[i] = h->m.roundPose[round & 1][i];
  return 0;
}

}  // extern "C"
