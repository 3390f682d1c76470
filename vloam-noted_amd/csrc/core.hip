// core.hip — parameters, errors and device checks of the C-ABI (include/loam_core.h).
#include <mutex>
#include <string>

#include "common.h"

namespace loam {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int32_t ensure_device(int32_t device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    set_error("no HIP device available (the MI355X core has no CPU fallback)");
    return LOAM_ERR_NODEVICE;
  }
  if (device < 0 || device >= n) {
    set_error("device index out of range");
    return LOAM_ERR_ARG;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    set_error("hipGetDeviceProperties failed");
    return LOAM_ERR_HIP;
  }
  std::string arch = prop.gcnArchName;
  if (arch.rfind("gfx950", 0) != 0) {
    set_error("device " + std::to_string(device) + " is " + arch + ", this build targets gfx950");
    return LOAM_ERR_NODEVICE;
  }
  return LOAM_OK;
}

}  // namespace loam

extern "C" {

void loam_params_default(loam_params* p) {
  if (!p) return;
  // loam_velodyne_HDL_64_kitti.launch:3-16, vloam_main.launch:4
  p->scan_line = 64;
  p->minimum_range = 5.0;
  p->mapping_skip_frame = 1;
  p->map_pub_number = 20;
  p->mapping_line_resolution = 0.4;
  p->mapping_plane_resolution = 0.8;
  p->detach_vo_lo = 1;
  p->verbose_level = 1;
  p->max_input_points = 262144;
  p->max_map_points = 2097152;
  p->max_submap_points = 524288;
  p->exact_voxel_order = 0;
}

const char* loam_last_error(void) { return loam::g_last_error.c_str(); }

int32_t loam_version(void) { return 100; }

}  // extern "C"
