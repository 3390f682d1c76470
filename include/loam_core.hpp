// loam_core.hpp — header-only C++ shim over the C-ABI (loam_core.h) with the reference's
// class and method names, for the lidar_odometry_mapping nodes:
//   vloam::ScanRegistration  scan_registration.h:64-81   -> loam_amd::ScanRegistration
//   vloam::LaserOdometry     laser_odometry.h:70-84      -> loam_amd::LaserOdometry
//   vloam::LaserMapping      laser_mapping.h:85-100      -> loam_amd::LaserMapping
// Clouds cross the boundary as packed float4 (x, y, z, intensity) arrays. pcl::PointXYZI
// is 32 bytes, so the node packs and unpacks it (INTEGRATION.md shows the adapter). Errors
// throw loam_amd::Error carrying the LOAM_ERR_* code and loam_last_error(). There is no
// CPU fallback.
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "loam_core.h"

namespace loam_amd {

class Error : public std::runtime_error {
 public:
  Error(int32_t rc, const std::string& msg) : std::runtime_error(msg), rc_(rc) {}
  int32_t code() const { return rc_; }

 private:
  int32_t rc_;
};

inline int32_t check(int32_t rc) {
  if (rc < 0) throw Error(rc, std::string("loam: ") + loam_last_error());
  return rc;
}

inline loam_params default_params() {
  loam_params p;
  loam_params_default(&p);
  return p;
}

using Cloud = std::vector<float>;  // 4 floats per point

// ScanRegistration::input / output (scan_registration.cpp:144-577)
class ScanRegistration {
 public:
  explicit ScanRegistration(const loam_params& p = default_params(), int32_t device = 0) {
    check(loam_scanreg_create(&p, device, &h_));
  }
  ~ScanRegistration() { loam_scanreg_destroy(h_); }
  ScanRegistration(const ScanRegistration&) = delete;
  ScanRegistration& operator=(const ScanRegistration&) = delete;

  void init() {}
  void reset() {}
  // laserCloudIn: n points, `stride` floats apart (pcl::PointXYZ: stride 4)
  void input(const float* xyz, int32_t n, int32_t stride = 4) { check(loam_scanreg_input(h_, xyz, n, stride)); }
  // laserCloud, cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat, surfPointsLessFlat
  void output(Cloud& full, Cloud& sharp, Cloud& less_sharp, Cloud& flat, Cloud& less_flat) const {
    Cloud* out[5] = {&full, &sharp, &less_sharp, &flat, &less_flat};
    int32_t n[5];
    check(loam_scanreg_counts(h_, n));
    for (int k = 0; k < 5; ++k) {
      out[k]->resize(static_cast<size_t>(n[k]) * 4);
      if (n[k]) check(loam_scanreg_copy(h_, k, out[k]->data(), n[k]));
    }
  }
  // device pointer + count of one output cloud (stays valid until the next input)
  std::pair<const float*, int32_t> device_cloud(int32_t which) const {
    const float* p = nullptr;
    const int32_t n = check(loam_scanreg_device_ptr(h_, which, &p));
    return {p, n};
  }
  double ms() const { return loam_scanreg_ms(h_); }
  loam_scanreg* handle() const { return h_; }

 private:
  loam_scanreg* h_ = nullptr;
};

// LaserOdometry::init / input / solveLO / output (laser_odometry.cpp:46-679), one stream
class LaserOdometry {
 public:
  explicit LaserOdometry(const loam_params& p = default_params(), int32_t device = 0) {
    check(loam_odometry_create(&p, device, 1, &h_));
  }
  ~LaserOdometry() { loam_odometry_destroy(h_); }
  LaserOdometry(const LaserOdometry&) = delete;
  LaserOdometry& operator=(const LaserOdometry&) = delete;

  void init() { check(loam_odometry_reset(h_)); }
  void reset() {}  // laser_odometry.cpp:128-135 clears per-frame buffers only
  void input(const Cloud& sharp, const Cloud& less_sharp, const Cloud& flat, const Cloud& less_flat) {
    check(loam_odometry_input(h_, 0, sharp.data(), n(sharp), less_sharp.data(), n(less_sharp), flat.data(), n(flat),
                              less_flat.data(), n(less_flat)));
  }
  // features already in HBM (ScanRegistration::device_cloud)
  void input_device(const float* sharp, int32_t ns, const float* less_sharp, int32_t nls, const float* flat,
                    int32_t nf, const float* less_flat, int32_t nlf) {
    check(loam_odometry_input_device(h_, 0, sharp, ns, less_sharp, nls, flat, nf, less_flat, nlf));
  }
  // vloam_tf->velo_last_VOT_velo_curr for the next solveLO (detach_vo_lo = 0,
  // laser_odometry.cpp:237-250)
  void set_vo_prior(const double q_xyzw[4], const double t_xyz[3]) { check(loam_odometry_set_prior(h_, 0, q_xyzw, t_xyz)); }
  void solveLO() { check(loam_odometry_solve(h_)); }
  // q_w_curr, t_w_curr, q_last_curr, t_last_curr, skip_frame (laser_odometry.cpp:660-679)
  bool output(double q_w[4], double t_w[3], double q_lc[4] = nullptr, double t_lc[3] = nullptr) const {
    int32_t skip = 0;
    check(loam_odometry_output(h_, 0, q_w, t_w, q_lc, t_lc, &skip));
    return skip != 0;
  }
  // laserCloudCornerLast (0) / laserCloudSurfLast (1) in HBM, valid until the next solve
  std::pair<const float*, int32_t> last_cloud(int32_t which) const {
    const float* p = nullptr;
    const int32_t c = check(loam_odometry_last_cloud(h_, 0, which, &p));
    return {p, c};
  }
  Cloud copy_last(int32_t which) const {
    Cloud out(static_cast<size_t>(last_cloud(which).second) * 4);
    if (!out.empty()) check(loam_odometry_copy_last(h_, 0, which, out.data(), static_cast<int32_t>(out.size() / 4)));
    return out;
  }
  loam_odom_stats stats() const {
    loam_odom_stats st;
    check(loam_odometry_stats(h_, 0, &st));
    return st;
  }
  loam_odometry* handle() const { return h_; }

 private:
  static int32_t n(const Cloud& c) { return static_cast<int32_t>(c.size() / 4); }
  loam_odometry* h_ = nullptr;
};

// B independent LaserMapping instances in one handle (one launch sequence per solve)
class BatchMapper {
 public:
  BatchMapper(int32_t n_streams, const loam_params& p = default_params(), int32_t device = 0) : n_(n_streams) {
    check(loam_mapper_create(&p, device, n_streams, &h_));
  }
  ~BatchMapper() { loam_mapper_destroy(h_); }
  BatchMapper(const BatchMapper&) = delete;
  BatchMapper& operator=(const BatchMapper&) = delete;

  void reset() { check(loam_mapper_reset(h_)); }
  void input(int32_t stream, const Cloud& corner, const Cloud& surf, const double q_wodom[4],
             const double t_wodom[3], bool skip_frame = false) {
    check(loam_mapper_input(h_, stream, corner.data(), static_cast<int32_t>(corner.size() / 4), surf.data(),
                            static_cast<int32_t>(surf.size() / 4), q_wodom, t_wodom, skip_frame ? 1 : 0));
  }
  void input_device(int32_t stream, const float* corner, int32_t nc, const float* surf, int32_t ns,
                    const double q_wodom[4], const double t_wodom[3], bool skip_frame = false) {
    check(loam_mapper_input_device(h_, stream, corner, nc, surf, ns, q_wodom, t_wodom, skip_frame ? 1 : 0));
  }
  void solve() { check(loam_mapper_solve(h_)); }
  // solve() in two halves (loam_mapper_solve_async / _wait): enqueue the frame and return; wait
  // for the oldest frame not yet waited for.  Two frames may be in the queue: give frame f + 1's
  // input and solve_async() while frame f is in flight (on a graph-path handle, <= 4 streams, the
  // device runs f + 1 right behind f).  solve_async() throws only when it did not enqueue the
  // frame; an older frame it finished to make room that failed is reported by the next wait() /
  // solve() (LOAM_ERR_EARLIER), so a caller that re-submits on a throw never queues a frame twice.
  void solve_async() { check(loam_mapper_solve_async(h_)); }
  // solve() that returns at the poses (loam_mapper_solve_pose): the map update of the frame
  // finishes beside the next frame's stack VoxelGrid; same results, bit for bit
  void solve_pose() { check(loam_mapper_solve_pose(h_)); }
  void wait() { check(loam_mapper_wait(h_)); }
  // queue the stack VoxelGrids of the inputs given so far (they run beside the frame in flight)
  void prefetch() { check(loam_mapper_prefetch(h_)); }
  void pose(int32_t stream, double q_w[4], double t_w[3]) const { check(loam_mapper_pose(h_, stream, q_w, t_w)); }
  // /laser_cloud_map (laser_mapping.cpp:884-899)
  Cloud map(int32_t stream) const {
    const int32_t n = check(loam_mapper_map_copy(h_, stream, nullptr, 0));
    Cloud out(static_cast<size_t>(n) * 4);
    if (n) check(loam_mapper_map_copy(h_, stream, out.data(), n));
    return out;
  }
  // /velodyne_cloud_registered (:901-911)
  Cloud registered(int32_t stream, const Cloud& full_res) const {
    Cloud out(full_res.size());
    check(loam_mapper_register_cloud(h_, stream, full_res.data(), static_cast<int32_t>(full_res.size() / 4),
                                     out.data()));
    return out;
  }
  loam_map_stats stats(int32_t stream) const {
    loam_map_stats st;
    check(loam_mapper_stats(h_, stream, &st));
    return st;
  }
  Cloud cube(int32_t stream, int32_t which, int32_t cube) const {
    const int32_t n = check(loam_mapper_cube_count(h_, stream, which, cube));
    Cloud out(static_cast<size_t>(n) * 4);
    if (n) check(loam_mapper_cube_copy(h_, stream, which, cube, out.data()));
    return out;
  }
  int32_t streams() const { return n_; }
  loam_mapper* handle() const { return h_; }

 private:
  loam_mapper* h_ = nullptr;
  int32_t n_ = 0;
};

// LaserMapping::init / reset / input / solveMapping / output (laser_mapping.cpp:147-814)
class LaserMapping {
 public:
  explicit LaserMapping(const loam_params& p = default_params(), int32_t device = 0) : m_(1, p, device) {}
  void init() { m_.reset(); }
  void reset() {}  // laser_mapping.cpp:132-136 clears per-frame buffers only
  // laserCloudCornerLast, laserCloudSurfLast, q_wodom_curr, t_wodom_curr, skip_frame
  void input(const Cloud& corner_last, const Cloud& surf_last, const double q_wodom_curr[4],
             const double t_wodom_curr[3], bool skip_frame) {
    m_.input(0, corner_last, surf_last, q_wodom_curr, t_wodom_curr, skip_frame);
  }
  void solveMapping() { m_.solve(); }
  // solveMapping that returns once q_w_curr / t_w_curr are final ("Pose first"):
  // output() and stats() read at once; the cube insertion and re-VoxelGrid run on beside the
  // next frame, and laserCloudMap() waits for them
  void solveMappingPose() { m_.solve_pose(); }
  // solveMapping split so that the node publishes frame f - 1 while frame f runs (INTEGRATION.md,
  // "Pipelined mapping"): input(f); solveMappingAsync(); waitMapping() finishes f - 1, whose
  // output() / stats() / laserCloudMap() are then read.  Host clouds are copied at input().
  void solveMappingAsync() { m_.solve_async(); }
  void waitMapping() { m_.wait(); }
  void prefetch() { m_.prefetch(); }
  // q_w_curr / t_w_curr: what publish() sends on /aft_mapped_to_init (laser_mapping.cpp:816-874);
  // after waitMapping(): the frame it finished
  void output(double q_w_curr[4], double t_w_curr[3]) const { m_.pose(0, q_w_curr, t_w_curr); }
  loam_map_stats stats() const { return m_.stats(0); }
  // publish() payloads: laserCloudMap and laserCloudFullRes in the map frame
  Cloud laserCloudMap() const { return m_.map(0); }
  Cloud laserCloudFullResRegistered(const Cloud& full_res) const { return m_.registered(0, full_res); }
  BatchMapper& batch() { return m_; }

 private:
  BatchMapper m_;
};

}  // namespace loam_amd
