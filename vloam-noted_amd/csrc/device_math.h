// device_math.h — geometry shared by the LOAM kernels (gfx950).
//
// Everything here decides discrete outcomes (which map points are neighbours, whether a
// neighbourhood is a line / plane, which voxel a point falls in), so it is written with the
// same operation order as the reference (Eigen 3.3 generic paths, FLANN L2_Simple, PCL
// VoxelGrid) and compiled with -ffp-contract=off: results are bit-identical to the CPU
// oracle's restatement (oracle/loam_oracle.cpp), which is written independently.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace loam {

struct dq {  // quaternion, xyzw storage (para_q / parameters[0..3])
  double x, y, z, w;
};
struct d3 {
  double x, y, z;
};

__host__ __device__ inline d3 cross3(const d3& a, const d3& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Eigen QuaternionBase::_transformVector (Quaternion.h): uv = vec x v; uv += uv;
// v + w * uv + vec x uv
__host__ __device__ inline d3 qrot(const dq& q, const d3& v) {
  d3 qv{q.x, q.y, q.z};
  d3 uv = cross3(qv, v);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  d3 c = cross3(qv, uv);
  return {(v.x + q.w * uv.x) + c.x, (v.y + q.w * uv.y) + c.y, (v.z + q.w * uv.z) + c.z};
}

// Eigen quat_product (generic path)
__host__ __device__ inline dq qmul(const dq& a, const dq& b) {
  dq r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

__host__ __device__ inline dq qinv(const dq& q) {
  double n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  if (n2 > 0) return {-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
  return {0, 0, 0, 0};
}

// LaserMapping::pointAssociateToMap (laser_mapping.cpp:154-164): double transform, float out
__host__ __device__ inline float4 to_map(const double* x7, float4 p) {
  dq q{x7[0], x7[1], x7[2], x7[3]};
  d3 r = qrot(q, d3{(double)p.x, (double)p.y, (double)p.z});
  return make_float4((float)(r.x + x7[4]), (float)(r.y + x7[5]), (float)(r.z + x7[6]), p.w);
}

// cube index rule of laser_mapping.cpp:228-241 / :747-756
__host__ __device__ inline int cube_of(double v, int cen) {
  int c = (int)((v + 25.0) / 50.0) + cen;
  if (v + 25.0 < 0) c--;
  return c;
}

// FLANN L2_Simple<float>: result += diff*diff per dimension, diff = query - point
__device__ inline float fdist2(float qx, float qy, float qz, float px, float py, float pz) {
  float dx = qx - px, dy = qy - py, dz = qz - pz;
  float r = 0.0f;
  r += dx * dx;
  r += dy * dy;
  r += dz * dz;
  return r;
}

// 3x3 symmetric eigensolver, cyclic Jacobi, ascending (stands in for
// SelfAdjointEigenSolver<Matrix3d>, laser_mapping.cpp:583).  Same sequence as the oracle.
__device__ inline void eig3(const double Ain[3][3], double evals[3], double evecs[3][3]) {
  double a[3][3], v[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      a[i][j] = Ain[i][j];
      v[i][j] = (i == j) ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
    if (off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int q = p + 1; q < 3; ++q) {
        double apq = a[p][q];
        if (apq != 0.0) {
          double app = a[p][p], aqq = a[q][q];
          double theta = (aqq - app) / (2.0 * apq);
          double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
          if (theta < 0.0) t = -t;
          double c = 1.0 / sqrt(t * t + 1.0);
          double s = t * c;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            double akp = a[k][p], akq = a[k][q];
            a[k][p] = c * akp - s * akq;
            a[k][q] = s * akp + c * akq;
          }
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            double apk = a[p][k], aqk = a[q][k];
            a[p][k] = c * apk - s * aqk;
            a[q][k] = s * apk + c * aqk;
          }
          a[p][q] = 0.0;
          a[q][p] = 0.0;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            double vkp = v[k][p], vkq = v[k][q];
            v[k][p] = c * vkp - s * vkq;
            v[k][q] = s * vkp + c * vkq;
          }
        }
      }
    }
  }
  int o0 = 0, o1 = 1, o2 = 2;
  // stable ascending insertion sort of 3 (same comparisons as the oracle)
  if (a[o1][o1] < a[o0][o0]) { int t = o0; o0 = o1; o1 = t; }
  if (a[o2][o2] < a[o1][o1]) {
    int t = o1; o1 = o2; o2 = t;
    if (a[o1][o1] < a[o0][o0]) { int u = o0; o0 = o1; o1 = u; }
  }
  const int ord[3] = {o0, o1, o2};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    evals[i] = a[ord[i]][ord[i]];
#pragma unroll
    for (int k = 0; k < 3; ++k) evecs[k][i] = v[k][ord[i]];
  }
}

// 5x3 least squares A n = -1, column-pivoted Householder QR (stands in for
// ColPivHouseholderQR, laser_mapping.cpp:655).  Same sequence as the oracle.
__device__ inline void lsq53(const double Ain[5][3], double x[3]) {
  double A[5][3];
  double b[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    b[i] = -1.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) A[i][j] = Ain[i][j];
  }
  int perm[3] = {0, 1, 2};
  double diag[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int best = k;
    double bestn = -1.0;
#pragma unroll
    for (int j = k; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int i = k; i < 5; ++i) s += A[i][j] * A[i][j];
      if (s > bestn) {
        bestn = s;
        best = j;
      }
    }
    if (best != k) {
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        double t = A[i][k];
        A[i][k] = A[i][best];
        A[i][best] = t;
      }
      int t = perm[k];
      perm[k] = perm[best];
      perm[best] = t;
    }
    double c0 = A[k][k];
    double tail = 0.0;
#pragma unroll
    for (int i = k + 1; i < 5; ++i) tail += A[i][k] * A[i][k];
    double tau, beta;
    double ess[5] = {0, 0, 0, 0, 0};
    if (tail <= 2.2250738585072014e-308) {
      tau = 0.0;
      beta = c0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
#pragma unroll
      for (int i = k + 1; i < 5; ++i) ess[i] = A[i][k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    diag[k] = beta;
    A[k][k] = beta;
#pragma unroll
    for (int i = k + 1; i < 5; ++i) A[i][k] = 0.0;
#pragma unroll
    for (int j = k + 1; j < 3; ++j) {
      double s = A[k][j];
#pragma unroll
      for (int i = k + 1; i < 5; ++i) s += ess[i] * A[i][j];
      s *= tau;
      A[k][j] -= s;
#pragma unroll
      for (int i = k + 1; i < 5; ++i) A[i][j] -= s * ess[i];
    }
    {
      double s = b[k];
#pragma unroll
      for (int i = k + 1; i < 5; ++i) s += ess[i] * b[i];
      s *= tau;
      b[k] -= s;
#pragma unroll
      for (int i = k + 1; i < 5; ++i) b[i] -= s * ess[i];
    }
  }
  double z[3] = {0, 0, 0};
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    if (diag[k] == 0.0) {
      z[k] = 0.0;
      continue;
    }
    double s = b[k];
#pragma unroll
    for (int j = k + 1; j < 3; ++j) s -= A[k][j] * z[j];
    z[k] = s / A[k][k];
  }
  // x[perm[k]] = z[k] (perm is a permutation of 0..2)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (perm[k] == 0) x[0] = z[k];
    if (perm[k] == 1) x[1] = z[k];
    if (perm[k] == 2) x[2] = z[k];
  }
}

// laser_mapping.cpp:557-603 — line test + two points on the line; nb in kNN order
__device__ inline bool edge_from_nbrs(const float nb[5][3], d3& pa, d3& pb) {
  double cx = 0, cy = 0, cz = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    cx = cx + (double)nb[j][0];
    cy = cy + (double)nb[j][1];
    cz = cz + (double)nb[j][2];
  }
  cx = cx / 5.0;
  cy = cy / 5.0;
  cz = cz / 5.0;
  double C[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    double d[3] = {(double)nb[j][0] - cx, (double)nb[j][1] - cy, (double)nb[j][2] - cz};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
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

// laser_mapping.cpp:642-680 — plane fit + flatness check
__device__ inline bool plane_from_nbrs(const float nb[5][3], d3& n, double& d) {
  double A[5][3];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    A[j][0] = nb[j][0];
    A[j][1] = nb[j][1];
    A[j][2] = nb[j][2];
  }
  double x[3];
  lsq53(A, x);
  double nn = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  double negdot = 1 / nn;
  n = {x[0] / nn, x[1] / nn, x[2] / nn};
  d = negdot;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if (fabs(n.x * nb[j][0] + n.y * nb[j][1] + n.z * nb[j][2] + negdot) > 0.2) ok = false;
  }
  return ok;
}

}  // namespace loam
