"""pytest configuration: `gpu` marker, import paths, CPU-side builds (oracle, generator).

CPU tests (``-m "not gpu"``) cover the oracle against independent implementations and the
golden fixtures, the host logic, and that the C-ABI library loads and exports every symbol
of include/loam_core.h.  GPU tests (``-m gpu``) are the parity tests proper; they call the
HIP kernels through the C-ABI and compare with the oracle.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    # the oracle and the scene generator are plain host code: build them if missing
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "libloam_oracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "vloam-noted_amd", "loam_amd", "_lib", "libloam_synth.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "vloam-noted_amd"), "synth"], check=True,
                       stdout=subprocess.DEVNULL)
    # the HIP library (hipcc cross-compiles gfx950 without a GPU): the ABI tests load it
    if not os.path.exists(os.path.join(ROOT, "vloam-noted_amd", "loam_amd", "_lib", "libloam_core.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "vloam-noted_amd"), "-j4"], check=True,
                       stdout=subprocess.DEVNULL)


def gpu_available():
    """HIP device count through the runtime itself (no torch import: slow on a cold box)."""
    import ctypes
    if not os.path.exists("/dev/kfd"):
        return False
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
