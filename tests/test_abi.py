"""CPU: the C-ABI boundary (include/loam_core.h) — library loads, exports every declared
symbol, the ctypes table matches the header, the header carries no torch/HIP types, and the
product path fails loudly (no CPU fallback) when there is no GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, gpu_available
from loam_amd import _core

HEADER = os.path.join(ROOT, "include", "loam_core.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(loam_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_api():
    names = declared()
    for must in ("loam_scanreg_create", "loam_scanreg_input", "loam_mapper_create", "loam_mapper_input",
                 "loam_mapper_solve", "loam_mapper_pose", "loam_lm_solve", "loam_voxel_grid"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(_core.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    assert sorted(_core.SIGNATURES) == declared()


def test_header_is_plain_c():
    text = open(HEADER).read()
    for bad in ("torch", "at::", "hipStream_t", "std::", "#include <hip"):
        assert bad not in text
    assert 'extern "C"' in text


def test_host_only_entry_points():
    L = _core.lib()
    assert L.loam_version() >= 100
    p = _core.default_params()
    assert p.scan_line == 64 and abs(p.mapping_line_resolution - 0.4) < 1e-12
    assert abs(p.mapping_plane_resolution - 0.8) < 1e-12 and abs(p.minimum_range - 5.0) < 1e-12
    assert p.max_map_points > 0 and p.max_submap_points > 0


def test_bad_arguments_are_rejected():
    L = _core.lib()
    h = ctypes.c_void_p()
    assert L.loam_mapper_create(None, 0, 0, ctypes.byref(h)) == -1  # NULL params = defaults; 0 streams is bad
    assert L.loam_mapper_solve(None) == -1
    assert L.loam_scanreg_destroy(None) in (0, -1)


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_no_device_fails_loudly():
    from loam_amd.mapping import BatchMapper
    from loam_amd.scanreg import ScanRegistration
    with pytest.raises(_core.LoamError) as e:
        BatchMapper(1)
    assert e.value.rc in (-5, -2)
    with pytest.raises(_core.LoamError):
        ScanRegistration()
    from loam_amd import prims
    with pytest.raises(_core.LoamError):
        prims.voxel_grid([[0, 0, 0, 0]], 0.4)


def test_cxx_shim_compiles_and_links(tmp_path):
    """include/loam_core.hpp with plain g++ (the reference nodes' compiler), linked to the library"""
    import subprocess
    lib_dir = os.path.dirname(_core.LIB_PATH)
    exe = str(tmp_path / "shim_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cxx", "shim_check.cpp"), "-o", exe, "-L", lib_dir,
                    "-lloam_core", f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath,/opt/rocm/lib"],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([exe, "1" if gpu_available() else "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "version" in r.stdout
