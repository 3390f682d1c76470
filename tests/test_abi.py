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
    """include/loam_core.hpp with plain g++ (the reference nodes' compiler), linked to the library;
    on a GPU box it runs frames through the shim's three stages (tests/cxx/shim_check.cpp)"""
    import subprocess
    lib_dir = os.path.dirname(_core.LIB_PATH)
    exe = str(tmp_path / "shim_check")
    oracle_dir = os.path.join(ROOT, "oracle", "_build")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cxx", "shim_check.cpp"), "-o", exe, "-L", lib_dir,
                    "-lloam_core", "-lloam_synth", "-L", oracle_dir, "-lloam_oracle", f"-Wl,-rpath,{lib_dir}",
                    f"-Wl,-rpath,{oracle_dir}", "-Wl,-rpath,/opt/rocm/lib"],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([exe, "1" if gpu_available() else "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "version" in r.stdout
    if gpu_available():  # four frames through the shim's three stages against the oracle
        assert "frame 3" in r.stdout


def test_new_entry_points_validate_arguments():
    """argument checks of the sharding, depth and VO entry points (before any device work)"""
    L = _core.lib()
    h = ctypes.c_void_p()
    assert L.loam_comm_create(0, 2, None, ctypes.byref(h)) == -1       # 2 ranks need callbacks
    assert L.loam_comm_create(2, 2, None, ctypes.byref(h)) == -1       # rank out of range
    assert L.loam_comm_create(0, 1, None, ctypes.byref(h)) == 0        # one rank: no callbacks needed
    assert L.loam_comm_destroy(h) == 0
    assert L.loam_mapper_create_sharded(None, 0, 1, None, ctypes.byref(h)) == -1
    xyz = (ctypes.c_float * 3)(1.0, 2.0, 3.0)
    assert L.loam_shard_owner(xyz, ctypes.c_float(0.4), 0) == -1
    assert L.loam_shard_owner(xyz, ctypes.c_float(0.0), 2) == -1
    assert L.loam_shard_owner(xyz, ctypes.c_float(0.4), 1) == 0
    dp = _core.DepthParams()
    L.loam_depth_params_default(ctypes.byref(dp))
    assert (dp.grid, dp.img_width, dp.img_height) == (5, 1242, 375)
    dp.grid = 0
    assert L.loam_depth_create(ctypes.byref(dp), 0, 1, ctypes.byref(h)) == -1
    off = (ctypes.c_int32 * 2)(0, 1)
    x = (ctypes.c_double * 6)()
    assert L.loam_vo_solve(0, 1, off, None, x, 100, None) == -1        # records missing
    assert L.loam_vo_solve(0, 1, off, None, x, 100000, None) == -1     # iteration cap
    bad = (ctypes.c_int32 * 2)(1, 0)
    assert L.loam_vo_solve(0, 1, bad, None, x, 100, None) == -1        # offsets must start at 0
    assert L.loam_vo_solve(0, 0, None, None, None, 100, None) == 0      # nothing to do
