"""The PCL-order sort's drain wait reports when it runs out (voxel_hot.h vh_drain).

A wave of the hot-pruned std::sort emulation that claims a list entry not listed yet waits while
some listed subtree is unfinished.  The wait is bounded (2^24 spins by default, which a working
workgroup cannot exhaust).  If it ever ran out, the subtree that entry would have held could stay
unsorted and a centroid would be silently wrong, so the filter raises VH_ERR_SPIN, which reaches
the caller as LOAM_ERR_SYNC with a message.  LOAM_VH_SPIN_LIMIT=0 (read once per process) makes
every such wait run out at once; the child process below runs a cloud whose sort lists many
subtrees (so some wave waits) with it, and must fail that way.  The same cloud with the default
limit gives the oracle's bits (the flag path leaves the default run unchanged).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import loam_oracle as O
from loam_amd import prims, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[2])
from loam_amd import prims
from loam_amd._core import LoamError
pts = np.load(sys.argv[1])
try:
    prims.voxel_grid_pcl(pts, 0.4)
except LoamError as e:
    print("RC", e.rc, str(e))
    sys.exit(0)
print("RC 0")
"""


def _cloud():
    # a quantized street frame: many points per 0.4 m voxel, a few thousand hot voxels, so the
    # sort partitions at the workgroup level and then drains many wave subtrees
    xyz, _ = synth.frame(6, 3, 2000, flags=synth.QUANTIZE)
    pts = np.concatenate([xyz, np.arange(len(xyz), dtype=np.float32)[:, None] % 64], 1)
    return np.ascontiguousarray(pts[:20000], dtype=np.float32)


def test_drain_spin_exhaustion_is_reported(tmp_path):
    pts = _cloud()
    path = tmp_path / "cloud.npy"
    np.save(path, pts)
    env = dict(os.environ, LOAM_VH_SPIN_LIMIT="0")
    r = subprocess.run([sys.executable, "-c", CHILD, str(path), os.path.join(ROOT, "vloam-noted_amd")],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = r.stdout.strip().splitlines()[-1]
    assert line.startswith("RC -6"), line  # LOAM_ERR_SYNC
    assert "ran out" in line, line


def test_default_limit_gives_pcl_bits():
    pts = _cloud()
    ref = O.voxel_grid(pts, 0.4)
    assert np.array_equal(prims.voxel_grid_pcl(pts, 0.4).view(np.uint32), ref.view(np.uint32))
