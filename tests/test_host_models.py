"""CPU: the host-checkable parts of the device arithmetic, against the C++ runtime itself.

- libm_f32.h (glibc's atanf / atan2f restated for the device, used by the ring rule and the
  azimuth / relTime of scan_registration.cpp:185-296) is compiled for the host and compared
  bit for bit with this container's glibc (tests/cxx/libm_f32_check.cpp).
- stdsort.h's formulation of libstdc++'s std::sort permutation (sector sort :365-366, PCL
  VoxelGrid) is run serially and compared with std::sort (tests/cxx/stdsort_model.cpp).
The GPU tests then check the device code against the oracle (which calls std::sort / glibc).
"""
import os
import subprocess

from conftest import ROOT

CXX = os.path.join(ROOT, "tests", "cxx")
CSRC = os.path.join(ROOT, "vloam-noted_amd", "csrc")


def _build_run(tmp_path, src, extra=()):
    exe = str(tmp_path / os.path.splitext(src)[0])
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, os.path.join(CXX, src), "-o", exe,
                    "-lm"], check=True, capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    return r


def test_glibc_atan2f_restatement_is_bit_exact(tmp_path):
    r = _build_run(tmp_path, "libm_f32_check.cpp", ("-D__host__=", "-D__device__=", "-I", CSRC))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_std_sort_permutation_model(tmp_path):
    r = _build_run(tmp_path, "stdsort_model.cpp")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout

