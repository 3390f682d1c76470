// Compiles the header-only shim (include/loam_core.hpp) with plain g++ against the built
// library: version, defaults, argument errors, and (without a GPU) the loud no-device error.
#include <cstdio>

#include "loam_core.hpp"

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
    return expect_device ? 0 : 5;
  } catch (const loam_amd::Error& e) {
    std::printf("no device: %d %s\n", e.code(), e.what());
    return (!expect_device && (e.code() == LOAM_ERR_NODEVICE || e.code() == LOAM_ERR_HIP)) ? 0 : 6;
  }
}
