// Compiles the header-only shim (include/loam_core.hpp) with plain g++ against the built
// library: version, defaults, argument errors, and (without a GPU) the loud no-device error.
// With a GPU (argv[1] = "1"): six synthetic HDL-64E frames through the shim's
// ScanRegistration -> LaserOdometry -> LaserMapping with host clouds between the stages, the
// way the reference nodes call them (lidar_odometry_mapping.cpp:40-176), against the CPU oracle
// pipeline (test infrastructure, linked for the comparison only): poses within 1e-4; once with
// the blocking solveMapping and once with the frames queued (solveMappingAsync / waitMapping,
// frame f - 1 published while frame f runs).
#include <array>
#include <cmath>
#include <cstdio>
#include <vector>

#include "loam_core.hpp"

extern "C" {
int32_t synth_frame(uint64_t seed, int32_t frame, int32_t n_az, double speed, float* out_xyz, double* pose7);
// oracle (oracle/loam_oracle.h)
struct oracle_scanreg;
struct oracle_odom;
struct oracle_map;
oracle_scanreg* oracle_scanreg_create(int32_t n_scans, double minimum_range);
int32_t oracle_scanreg_input(oracle_scanreg* h, const float* xyz, int32_t n, int32_t stride);
int32_t oracle_scanreg_count(oracle_scanreg* h, int32_t which);
int32_t oracle_scanreg_copy(oracle_scanreg* h, int32_t which, float* out);
oracle_odom* oracle_odom_create(int32_t mapping_skip_frame);
int32_t oracle_odom_input(oracle_odom* h, const float* full, int32_t nfull, const float* sharp, int32_t nsharp,
                          const float* less_sharp, int32_t nless_sharp, const float* flat, int32_t nflat,
                          const float* less_flat, int32_t nless_flat);
int32_t oracle_odom_solve(oracle_odom* h);
int32_t oracle_odom_output(oracle_odom* h, double* q_w, double* t_w, double* q_lc, double* t_lc);
int32_t oracle_odom_count(oracle_odom* h, int32_t which);
int32_t oracle_odom_copy(oracle_odom* h, int32_t which, float* out);
oracle_map* oracle_map_create(float line_res, float plane_res);
int32_t oracle_map_input(oracle_map* h, const float* corner, int32_t nc, const float* surf, int32_t ns,
                         const float* full, int32_t nf, const double* q_wodom, const double* t_wodom, int32_t skip);
int32_t oracle_map_solve(oracle_map* h);
int32_t oracle_map_pose(oracle_map* h, double* q_w, double* t_w);
}

// the oracle pipeline's mapping poses (q xyzw, t) for frames 0 .. nf - 1
static std::vector<std::array<double, 7>> oracle_poses(int nf, int n_az) {
  oracle_scanreg* osr = oracle_scanreg_create(64, 5.0);
  oracle_odom* olo = oracle_odom_create(1);
  oracle_map* olm = oracle_map_create(0.4f, 0.8f);
  std::vector<float> xyz(64 * n_az * 3);
  double gt[7];
  std::vector<std::array<double, 7>> out;
  for (int f = 0; f < nf; ++f) {
    const int n = synth_frame(23, f, n_az, 1.0, xyz.data(), gt);
    oracle_scanreg_input(osr, xyz.data(), n, 3);
    std::vector<float> c[5];
    for (int k = 0; k < 5; ++k) {
      c[k].resize(4 * static_cast<size_t>(oracle_scanreg_count(osr, k)) + 4);
      oracle_scanreg_copy(osr, k, c[k].data());
    }
    auto cnt = [&](int k) { return oracle_scanreg_count(osr, k); };
    oracle_odom_input(olo, c[0].data(), cnt(0), c[1].data(), cnt(1), c[2].data(), cnt(2), c[3].data(), cnt(3),
                      c[4].data(), cnt(4));
    oracle_odom_solve(olo);
    double oq[4], ot[3], oqlc[4], otlc[3];
    const int oskip = oracle_odom_output(olo, oq, ot, oqlc, otlc);
    std::vector<float> cl(4 * static_cast<size_t>(oracle_odom_count(olo, 0)) + 4),
        sl(4 * static_cast<size_t>(oracle_odom_count(olo, 1)) + 4);
    oracle_odom_copy(olo, 0, cl.data());
    oracle_odom_copy(olo, 1, sl.data());
    oracle_map_input(olm, cl.data(), oracle_odom_count(olo, 0), sl.data(), oracle_odom_count(olo, 1), nullptr, 0, oq,
                     ot, oskip);
    oracle_map_solve(olm);
    std::array<double, 7> r;
    oracle_map_pose(olm, r.data(), r.data() + 4);
    out.push_back(r);
  }
  return out;
}

static double pose_diff(const double q[4], const double t[3], const std::array<double, 7>& r) {
  double d = 0.0;
  for (int i = 0; i < 3; ++i) d = std::fmax(d, std::fabs(t[i] - r[4 + i]));
  for (int i = 0; i < 4; ++i) d = std::fmax(d, std::fabs(std::fabs(q[i]) - std::fabs(r[i])));
  return d;
}

// mode BLOCKING: each frame's solveMapping blocks (the reference's facade,
// lidar_odometry_mapping.cpp:144-176); QUEUED: frame f is enqueued with solveMappingAsync and
// frame f - 1 is waited for and "published" after it (pipelined mapping); POSE:
// solveMappingPose, frame f published at once, its map update finishing beside frame f + 1
enum ShimMode { BLOCKING, QUEUED, POSE };
static int frames_through_the_shim(ShimMode mode, const std::vector<std::array<double, 7>>& ref, int n_az) {
  const bool queued = mode == QUEUED;
  static const char* const names[] = {"blocking", "queued", "pose"};
  loam_params p = loam_amd::default_params();
  p.exact_voxel_order = 1;  // free-running frames: PCL's VoxelGrid order, like the oracle
  loam_amd::ScanRegistration sr(p, 0);
  loam_amd::LaserOdometry lo(p, 0);
  loam_amd::LaserMapping lm(p, 0);
  std::vector<float> xyz(64 * n_az * 3);
  double gt[7];
  double worst = 0.0;
  const int nf = static_cast<int>(ref.size());
  auto publish = [&](int f) {  // what publish() would send for frame f
    double qm[4], tm[3];
    lm.output(qm, tm);
    const double d = pose_diff(qm, tm, ref[f]);
    worst = std::fmax(worst, d);
    const loam_map_stats st = lm.stats();
    std::printf("%s frame %d: mapping t (%.4f %.4f %.4f), LM iterations %d + %d, |d| %.3e\n",
                names[mode], f, tm[0], tm[1], tm[2], st.lm[0].iterations, st.lm[1].iterations, d);
  };
  for (int f = 0; f < nf; ++f) {
    const int n = synth_frame(23, f, n_az, 1.0, xyz.data(), gt);
    // device pipeline through the shim, host clouds between the stages
    sr.input(xyz.data(), n, 3);
    loam_amd::Cloud full, sharp, less_sharp, flat, less_flat;
    sr.output(full, sharp, less_sharp, flat, less_flat);
    lo.input(sharp, less_sharp, flat, less_flat);
    lo.solveLO();
    double q[4], t[3];
    const bool skip = lo.output(q, t);
    lm.input(lo.copy_last(0), lo.copy_last(1), q, t, skip);
    if (mode == BLOCKING) {
      lm.solveMapping();
      publish(f);
    } else if (mode == POSE) {
      lm.solveMappingPose();
      publish(f);
    } else {
      lm.solveMappingAsync();  // frame f, behind f - 1 on the device
      if (f > 0) {
        lm.waitMapping();  // frame f - 1
        publish(f - 1);
      }
    }
  }
  if (queued) {
    lm.waitMapping();
    publish(nf - 1);
  }
  return worst < 1e-4 ? 0 : 9;
}

int main(int argc, char** argv) {
  const bool expect_device = argc > 1 && argv[1][0] == '1';
  std::printf("version %d\n", loam_version());
  const loam_params p = loam_amd::default_params();
  if (p.scan_line != 64) return 2;
  try {
    loam_amd::check(loam_mapper_create(&p, 0, 0, nullptr));
    return 3;
  } catch (const loam_amd::Error& e) {
    if (e.code() != LOAM_ERR_ARG) return 4;
  }
  try {
    loam_amd::LaserOdometry o(p, 0);
    double q[4], t[3];
    o.output(q, t);
    if (!expect_device) return 7;
  } catch (const loam_amd::Error& e) {
    if (expect_device || (e.code() != LOAM_ERR_NODEVICE && e.code() != LOAM_ERR_HIP)) return 8;
  }
  try {
    loam_amd::LaserMapping m(p, 0);
    double q[4] = {0, 0, 0, 1}, t[3] = {0, 0, 0};
    m.output(q, t);
    std::printf("device ok, pose w %.1f\n", q[3]);
    if (!expect_device) return 5;
  } catch (const loam_amd::Error& e) {
    std::printf("no device: %d %s\n", e.code(), e.what());
    return (!expect_device && (e.code() == LOAM_ERR_NODEVICE || e.code() == LOAM_ERR_HIP)) ? 0 : 6;
  }
  const int n_az = 1000;
  const std::vector<std::array<double, 7>> ref = oracle_poses(6, n_az);
  for (ShimMode mode : {BLOCKING, QUEUED, POSE}) {
    const int rc = frames_through_the_shim(mode, ref, n_az);
    if (rc) return rc;
  }
  return 0;
}
