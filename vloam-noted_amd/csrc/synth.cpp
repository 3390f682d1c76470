// synth.cpp — synthetic HDL-64E street scenes for tests and bench.
//
// KITTI bags are unavailable offline, so every configuration runs on a procedurally
// generated street: ground plane z = -1.73 m, building facades at |y| = 12 m with recessed
// windows and alleys (back walls at |y| = 30 m), poles at |y| = 9 m, parked-car boxes at
// |y| = 7 m.  The scene is a pure function of (seed, x) — infinite and deterministic.
//
// Sensor: 64 lasers; upper block 1.98 - k/3 deg, lower block -8.87 - k/2 deg (offset a few
// hundredths of a degree from the reference's scanID boundaries so the ring rule of
// scan_registration.cpp:241-254 is unambiguous), n_az azimuths per revolution clockwise,
// range noise N(0, 0.02 m), max range 100 m.  Output order is ring-major (KITTI-like).
// synth_frame_ex's flags switch on the edge cases (boundary elevations, per-laser azimuth
// offsets, azimuth-interleaved order, 1 cm quantization) for the parity tests.
#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline double u01(uint64_t h) { return (h >> 11) * (1.0 / 9007199254740992.0); }
inline double hrand(uint64_t seed, int64_t a, int64_t b) {
  return u01(mix64(seed ^ mix64((uint64_t)a * 0x100000001b3ULL + (uint64_t)b)));
}

struct Rng {
  uint64_t s;
  double uni() {
    s = mix64(s);
    return u01(s);
  }
  double gauss() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

constexpr double kGround = -1.73;
constexpr double kFacade = 12.0, kRecess = 0.35, kBack = 30.0, kBuildH = 15.0;
constexpr double kPoleY = 9.0, kPoleR = 0.15, kPoleH = 6.0, kPoleSlot = 15.0;
constexpr double kCarY = 7.0, kCarW = 1.8, kCarL = 4.5, kCarH = 1.5, kCarSlot = 9.0;
constexpr double kBldSlot = 48.0, kAlleyW = 6.0;
constexpr double kMaxRange = 100.0;

struct Scene {
  uint64_t seed;
  // side: 0 for y > 0, 1 for y < 0
  bool alley(int side, double x) const {
    int64_t k = (int64_t)std::floor(x / kBldSlot);
    double off = 10.0 + 25.0 * hrand(seed, 100 + side, k);
    double lx = x - k * kBldSlot;
    return lx >= off && lx < off + kAlleyW;
  }
  // window test on facade coordinates (x along street, z height)
  bool window(int side, double x, double z) const {
    int64_t col = (int64_t)std::floor(x / 4.0);
    int64_t flr = (int64_t)std::floor((z - kGround) / 3.5);
    if (flr < 1 || flr > 3) return false;
    if (hrand(seed, 200 + side, col * 7 + flr) < 0.25) return false;
    double lx = x - col * 4.0, lz = (z - kGround) - flr * 3.5;
    double w0 = 0.6 + 0.4 * hrand(seed, 300 + side, col);
    return lx > w0 && lx < 4.0 - w0 && lz > 0.9 && lz < 2.7;
  }
  bool pole(int side, int64_t k, double& px) const {
    if (hrand(seed, 400 + side, k) < 0.15) return false;
    px = k * kPoleSlot + 2.0 + 11.0 * hrand(seed, 500 + side, k);
    return true;
  }
  bool car(int side, int64_t k, double& cx) const {
    if (hrand(seed, 600 + side, k) < 0.35) return false;
    cx = k * kCarSlot + 0.5 + 3.5 * hrand(seed, 700 + side, k);
    return true;
  }
};

// nearest hit distance along unit ray (o, d); returns +inf on miss
double cast(const Scene& S, const double o[3], const double d[3]) {
  double best = INFINITY;
  // ground
  if (d[2] < -1e-9) {
    double t = (kGround - o[2]) / d[2];
    if (t > 0 && t < best) best = t;
  }
  // facades / alleys / back walls / window recesses
  for (int side = 0; side < 2; ++side) {
    double sgn = side == 0 ? 1.0 : -1.0;
    if (d[1] * sgn <= 1e-9) continue;
    double t = (sgn * kFacade - o[1]) / d[1];
    if (t > 0 && t < best) {
      double x = o[0] + t * d[0], z = o[2] + t * d[2];
      if (z < kGround + kBuildH) {
        if (S.alley(side, x)) {
          double tb = (sgn * kBack - o[1]) / d[1];
          double zb = o[2] + tb * d[2];
          if (tb < best && zb < kGround + kBuildH) best = tb;
        } else if (S.window(side, x, z)) {
          double tr = (sgn * (kFacade + kRecess) - o[1]) / d[1];
          if (tr < best) best = tr;
        } else {
          best = t;
        }
      }
    }
  }
  // poles: vertical cylinders along the |y| = 9 line
  for (int side = 0; side < 2; ++side) {
    double sgn = side == 0 ? 1.0 : -1.0;
    if (std::fabs(d[1]) < 1e-9) continue;
    double tc = (sgn * kPoleY - o[1]) / d[1];
    if (tc <= 0) continue;
    double xc = o[0] + tc * d[0];
    double span = 0.5 + kPoleR * std::fabs(std::hypot(d[0], d[1]) / d[1]);
    int64_t k0 = (int64_t)std::floor((xc - span - 13.0) / kPoleSlot);
    int64_t k1 = (int64_t)std::floor((xc + span) / kPoleSlot);
    for (int64_t k = k0; k <= k1; ++k) {
      double px;
      if (!S.pole(side, k, px)) continue;
      double py = sgn * kPoleY;
      double ox = o[0] - px, oy = o[1] - py;
      double a = d[0] * d[0] + d[1] * d[1];
      double b = 2 * (ox * d[0] + oy * d[1]);
      double c = ox * ox + oy * oy - kPoleR * kPoleR;
      double disc = b * b - 4 * a * c;
      if (disc < 0 || a < 1e-12) continue;
      double t = (-b - std::sqrt(disc)) / (2 * a);
      if (t > 0 && t < best) {
        double z = o[2] + t * d[2];
        if (z > kGround && z < kGround + kPoleH) best = t;
      }
    }
  }
  // parked cars: axis-aligned boxes in the |y| in [6.1, 7.9] lane
  for (int side = 0; side < 2; ++side) {
    double sgn = side == 0 ? 1.0 : -1.0;
    double y0 = sgn * kCarY - kCarW / 2, y1 = sgn * kCarY + kCarW / 2;
    double ty0, ty1;
    if (std::fabs(d[1]) < 1e-12) {
      if (o[1] < y0 || o[1] > y1) continue;
      ty0 = 0;
      ty1 = kMaxRange;
    } else {
      ty0 = (y0 - o[1]) / d[1];
      ty1 = (y1 - o[1]) / d[1];
      if (ty0 > ty1) std::swap(ty0, ty1);
    }
    if (ty1 <= 0 || ty0 >= best) continue;
    double xa = o[0] + std::max(ty0, 0.0) * d[0], xb = o[0] + std::min(ty1, kMaxRange) * d[0];
    if (xa > xb) std::swap(xa, xb);
    int64_t k0 = (int64_t)std::floor((xa - kCarL - 4.0) / kCarSlot);
    int64_t k1 = (int64_t)std::floor(xb / kCarSlot);
    if (k1 - k0 > 40) k1 = k0 + 40;
    for (int64_t k = k0; k <= k1; ++k) {
      double cx;
      if (!S.car(side, k, cx)) continue;
      double lo[3] = {cx, y0, kGround}, hi[3] = {cx + kCarL, y1, kGround + kCarH};
      double tmin = 0, tmax = best;
      bool hit = true;
      for (int a = 0; a < 3 && hit; ++a) {
        if (std::fabs(d[a]) < 1e-12) {
          if (o[a] < lo[a] || o[a] > hi[a]) hit = false;
        } else {
          double t0 = (lo[a] - o[a]) / d[a], t1 = (hi[a] - o[a]) / d[a];
          if (t0 > t1) std::swap(t0, t1);
          tmin = std::max(tmin, t0);
          tmax = std::min(tmax, t1);
          if (tmin > tmax) hit = false;
        }
      }
      if (hit && tmin > 0 && tmin < best) best = tmin;
    }
  }
  return best;
}

void rotz_y_x(double yaw, double pitch, double roll, double R[3][3]) {
  double cy = std::cos(yaw), sy = std::sin(yaw), cp = std::cos(pitch), sp = std::sin(pitch),
         cr = std::cos(roll), sr = std::sin(roll);
  R[0][0] = cy * cp; R[0][1] = cy * sp * sr - sy * cr; R[0][2] = cy * sp * cr + sy * sr;
  R[1][0] = sy * cp; R[1][1] = sy * sp * sr + cy * cr; R[1][2] = sy * sp * cr - cy * sr;
  R[2][0] = -sp;     R[2][1] = cp * sr;                R[2][2] = cp * cr;
}

void mat_to_quat(const double R[3][3], double q[4]) {
  double tr = R[0][0] + R[1][1] + R[2][2];
  double x, y, z, w;
  if (tr > 0) {
    double s = std::sqrt(tr + 1.0) * 2;
    w = 0.25 * s; x = (R[2][1] - R[1][2]) / s; y = (R[0][2] - R[2][0]) / s; z = (R[1][0] - R[0][1]) / s;
  } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
    double s = std::sqrt(1.0 + R[0][0] - R[1][1] - R[2][2]) * 2;
    w = (R[2][1] - R[1][2]) / s; x = 0.25 * s; y = (R[0][1] + R[1][0]) / s; z = (R[0][2] + R[2][0]) / s;
  } else if (R[1][1] > R[2][2]) {
    double s = std::sqrt(1.0 + R[1][1] - R[0][0] - R[2][2]) * 2;
    w = (R[0][2] - R[2][0]) / s; x = (R[0][1] + R[1][0]) / s; y = 0.25 * s; z = (R[1][2] + R[2][1]) / s;
  } else {
    double s = std::sqrt(1.0 + R[2][2] - R[0][0] - R[1][1]) * 2;
    w = (R[1][0] - R[0][1]) / s; x = (R[0][2] + R[2][0]) / s; y = (R[1][2] + R[2][1]) / s; z = 0.25 * s;
  }
  q[0] = x; q[1] = y; q[2] = z; q[3] = w;
}

}  // namespace

extern "C" {

// ground-truth sensor pose of a frame: x = f * speed, gentle lateral weave and yaw wobble
void synth_pose(uint64_t seed, double frame, double speed, double* q_xyzw, double* t_xyz) {
  double ph = 2.0 * M_PI * u01(mix64(seed + 17));
  // start from rest: quadratic ramp to `speed` m/frame over the first 20 frames
  double x = frame < 20.0 ? speed * frame * frame / 40.0 : speed * (frame - 10.0);
  double y = 2.0 * std::sin(2.0 * M_PI * frame / 500.0 + ph);
  double dy = 2.0 * (2.0 * M_PI / 500.0) * std::cos(2.0 * M_PI * frame / 500.0 + ph) / speed;
  double yaw = std::atan(dy) + (2.0 * M_PI / 180.0) * std::sin(2.0 * M_PI * frame / 170.0 + ph);
  double pitch = (0.3 * M_PI / 180.0) * std::sin(2.0 * M_PI * frame / 90.0);
  double roll = (0.2 * M_PI / 180.0) * std::sin(2.0 * M_PI * frame / 60.0 + 1.0);
  double R[3][3];
  rotz_y_x(yaw, pitch, roll, R);
  mat_to_quat(R, q_xyzw);
  t_xyz[0] = x;
  t_xyz[1] = y;
  t_xyz[2] = 0.0;
}

// Edge-case modes of synth_frame_ex (flags), the input shapes the reference's scan
// registration and odometry see on real sensors but the default street avoids:
//   SYNTH_COLUMN_MAJOR  azimuth-interleaved output (one column of 64 lasers after another, the
//                       order of raw HDL-64E packets) instead of ring-major
//   SYNTH_LASER_AZ      per-laser azimuth offsets of up to +-4 deg (the HDL-64E rotational
//                       corrections): rings start at different azimuths, so with column-major
//                       order points before the halfPassed latch fall below startOri and get
//                       relTime < 0, int(intensity) = scanID - 1 (scan_registration.cpp:263-296)
//   SYNTH_BOUNDARY      laser elevations exactly on the ring rule's boundaries and cut-offs
//                       (scan_registration.cpp:241-254: 2 - (k + 1/2)/3, -8.83 - (k + 1/2)/2,
//                       2, -8.83, -24.33): a point's ring is decided by the last bits of
//                       atan / sqrt / the division
//   SYNTH_QUANTIZE      coordinates rounded to 1 cm: equal curvatures (std::sort ties of
//                       :365-366) and points on VoxelGrid leaf boundaries
//   SYNTH_VLP16         a 16-laser sensor (VLP-16: -15 + 2k deg), for the N_SCANS == 16 ring rule
//                       (scan_registration.cpp:225-230); with SYNTH_BOUNDARY the elevations sit
//                       on its boundaries (-16 + 2k: (angle + 15) / 2 + 0.5 = k exactly) and the
//                       +15 deg cut-off
//   SYNTH_HDL32         a 32-laser sensor (HDL-32E: -92/3 + 4k/3 deg) for N_SCANS == 32
//                       (:231-236); without SYNTH_BOUNDARY offset by half a ring pitch, with it
//                       exactly HDL-32E's, where (angle + 92/3) * 3/4 = k is the boundary
constexpr int32_t SYNTH_COLUMN_MAJOR = 1, SYNTH_LASER_AZ = 2, SYNTH_BOUNDARY = 4, SYNTH_QUANTIZE = 8,
                  SYNTH_VLP16 = 16, SYNTH_HDL32 = 32;

int32_t synth_frame_ex(uint64_t seed, int32_t frame, int32_t n_az, double speed, int32_t flags, float* out_xyz,
                       double* pose7);

// one revolution: writes up to 64*n_az points (16 / 32 * n_az for SYNTH_VLP16 / SYNTH_HDL32) (x,y,z, stride 3) in the SENSOR frame,
// ring-major; returns the number of returns.  pose7 = q(x,y,z,w), t(x,y,z) ground truth.
int32_t synth_frame(uint64_t seed, int32_t frame, int32_t n_az, double speed, float* out_xyz,
                    double* pose7) {
  return synth_frame_ex(seed, frame, n_az, speed, 0, out_xyz, pose7);
}

int32_t synth_frame_ex(uint64_t seed, int32_t frame, int32_t n_az, double speed, int32_t flags, float* out_xyz,
                       double* pose7) {
  Scene S{seed};
  double q[4], t[3];
  synth_pose(seed, frame, speed, q, t);
  if (pose7) {
    for (int i = 0; i < 4; ++i) pose7[i] = q[i];
    for (int i = 0; i < 3; ++i) pose7[4 + i] = t[i];
  }
  // rotation matrix from quaternion
  double x = q[0], y = q[1], z = q[2], w = q[3];
  double R[3][3] = {{1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)},
                    {2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)},
                    {2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)}};
  Rng rng{mix64(seed * 1000003ULL + (uint64_t)frame)};
  double az0 = 2.0 * M_PI * u01(mix64(seed ^ (uint64_t)frame * 77ULL)) / n_az;
  const int lasers = (flags & SYNTH_VLP16) ? 16 : (flags & SYNTH_HDL32) ? 32 : 64;
  const bool bnd = (flags & SYNTH_BOUNDARY) != 0;
  double ce[64], se[64], daz[64];
  for (int ring = 0; ring < lasers; ++ring) {
    double elev = ring < 32 ? (1.98 - ring / 3.0) : (-8.87 - (ring - 32) * 0.5);
    if (lasers == 16) {
      elev = bnd ? -16.0 + 2.0 * (ring + 1) : -15.0 + 2.0 * ring + 0.01;
    } else if (lasers == 32) {
      elev = -92.0 / 3.0 + (ring + (bnd ? 0.0 : 0.5)) * 4.0 / 3.0;
    } else if (bnd) {
      elev = ring < 32 ? 2.0 - (ring + 0.5) / 3.0 : -8.83 - (ring - 32 + 0.5) / 2.0;
      if (ring == 0) elev = 2.0;
      if (ring == 32) elev = -8.83;
      if (ring == 63) elev = -24.33;
    }
    const double el = elev * M_PI / 180.0;
    ce[ring] = std::cos(el);
    se[ring] = std::sin(el);
    // offsets falling with the laser index (plus jitter): in a column-major frame the first
    // returning laser leads, and the first columns of the lasers after it lie before startOri
    daz[ring] = (flags & SYNTH_LASER_AZ)
                    ? (M_PI / 180.0) * (4.0 - 8.0 * ring / (lasers - 1.0) + 0.5 * (2.0 * hrand(seed, 900, ring) - 1.0))
                    : 0.0;
  }
  int32_t n = 0;
  const bool cm = (flags & SYNTH_COLUMN_MAJOR) != 0;
  for (int outer = 0; outer < (cm ? n_az : lasers); ++outer) {
    for (int inner = 0; inner < (cm ? lasers : n_az); ++inner) {
      const int ring = cm ? inner : outer, a = cm ? outer : inner;
      double az = -(az0 + 2.0 * M_PI * a / n_az + daz[ring]);  // clockwise
      double ds[3] = {ce[ring] * std::cos(az), ce[ring] * std::sin(az), se[ring]};
      double dw[3] = {R[0][0] * ds[0] + R[0][1] * ds[1] + R[0][2] * ds[2],
                      R[1][0] * ds[0] + R[1][1] * ds[1] + R[1][2] * ds[2],
                      R[2][0] * ds[0] + R[2][1] * ds[1] + R[2][2] * ds[2]};
      double r = cast(S, t, dw);
      double noise = 0.02 * rng.gauss();
      if (!(r < kMaxRange)) continue;
      r += noise;
      float p[3] = {static_cast<float>(r * ds[0]), static_cast<float>(r * ds[1]), static_cast<float>(r * ds[2])};
      if (flags & SYNTH_QUANTIZE)
        for (float& v : p) v = static_cast<float>(std::round(static_cast<double>(v) * 100.0) / 100.0);
      out_xyz[3 * n + 0] = p[0];
      out_xyz[3 * n + 1] = p[1];
      out_xyz[3 * n + 2] = p[2];
      ++n;
    }
  }
  return n;
}

}  // extern "C"
