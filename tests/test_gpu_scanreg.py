"""GPU parity of ScanRegistration::input (scan_registration.cpp:144-513) against the oracle.

Everything is bit-exact: the ring-major cloud (xyz and intensity = scanID + 0.1 relTime, with
glibc's atan2f / atanf restated on the device, libm_f32.h), curvature, labels and the four
feature clouds.  The sector sort reproduces std::sort's order when curvatures tie (stdsort.h)
and the per-ring VoxelGrid sums in PCL's order (voxel_pcl.h).  The edge-case generator modes
(csrc/synth.cpp) feed what the default street avoids: elevations on the ring rule's
boundaries, per-laser azimuth offsets with column-major order (relTime < 0 before the
halfPassed latch), and 1 cm quantization (tied curvatures, points on leaf boundaries).
"""
import numpy as np
import pytest

import loam_oracle as O
from loam_amd import synth
from loam_amd.scanreg import ScanRegistration

pytestmark = pytest.mark.gpu


def _same_points(a, b):
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _check_frame(xyz, gpu=None, n_scans=64):
    ref = O.ScanRegistration(n_scans=n_scans)
    ref.input(xyz)
    gpu = gpu or ScanRegistration()
    gpu.input(xyz)
    for a, b in zip(gpu.output(), ref.output()):
        _same_points(a, b)
    curv, lab = gpu.curvature()
    rcurv, rlab = ref.curvature()
    assert np.array_equal(curv[5:-5].view(np.uint32), rcurv[5:-5].view(np.uint32))
    assert np.array_equal(lab[5:-5], rlab[5:-5])
    return ref


@pytest.mark.parametrize("seed,frame", [(1, 0), (2, 13), (9, 40)])
def test_scanreg_matches_oracle(seed, frame):
    xyz, _ = synth.frame(seed, frame)
    _check_frame(xyz)


MODES = {"boundary": synth.BOUNDARY, "column_major": synth.COLUMN_MAJOR | synth.LASER_AZ,
         "quantized": synth.QUANTIZE, "all": synth.BOUNDARY | synth.COLUMN_MAJOR | synth.LASER_AZ | synth.QUANTIZE}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("seed,frame", [(3, 10), (8, 77)])
def test_scanreg_edge_cases(mode, seed, frame):
    xyz, _ = synth.frame(seed, frame, 2000, flags=MODES[mode])
    ref = _check_frame(xyz)
    it = ref.cloud(0)[:, 3]
    if mode in ("column_major", "all"):  # relTime < 0 before the latch: int(intensity) = scanID - 1
        assert ((it - np.floor(it)) > 0.5).sum() > 100
    if mode in ("quantized", "all"):  # tied curvatures inside the sectors
        c, _ = ref.curvature()
        assert len(c) - len(np.unique(c)) > 300


@pytest.mark.parametrize("lasers,flags", [(16, 0), (16, synth.BOUNDARY), (32, 0), (32, synth.BOUNDARY),
                                          (16, synth.COLUMN_MAJOR | synth.LASER_AZ | synth.QUANTIZE)])
def test_scanreg_16_and_32_lines(lasers, flags):
    """the N_SCANS == 16 / 32 ring rules (scan_registration.cpp:225-236) on VLP-16 / HDL-32E
    elevations, also exactly on the rules' boundaries"""
    xyz, _ = synth.frame(5, 21, 2000, flags=flags | (synth.VLP16 if lasers == 16 else synth.HDL32))
    ref = _check_frame(xyz, ScanRegistration(scan_line=lasers), n_scans=lasers)
    ids = np.floor(ref.cloud(0)[:, 3]).astype(int)
    assert ids.max() < lasers and len(np.unique(ids)) >= (12 if lasers == 16 else 20)


@pytest.mark.parametrize("n_az", [4000, 5000])
def test_scanreg_long_tied_sectors(n_az):
    """boundary elevations merge two lasers into one ring and quantization makes the ties:
    sectors over 512 points (tie re-sort in global memory) and, at 5000 azimuths, over 1024
    (the block bitonic path, then the re-sort)"""
    xyz, _ = synth.frame(4, 5, n_az, flags=synth.BOUNDARY | synth.QUANTIZE)
    ref = _check_frame(xyz, ScanRegistration(max_input_points=400000))
    sizes = np.diff(np.flatnonzero(np.diff(np.floor(ref.cloud(0)[:, 3])) != 0))
    assert sizes.max() > 6 * (1024 if n_az == 5000 else 512)


def test_scanreg_many_long_tied_rings():
    """7000 azimuths, 1 cm quantization: every ring's sectors exceed 1024 points, so all rings'
    workgroups run the long-sector path (block bitonic, then the tie re-sort with its level
    lists in global memory) at the same time; each ring has its own list area"""
    xyz, _ = synth.frame(6, 9, 7000, flags=synth.QUANTIZE)
    ref = _check_frame(xyz, ScanRegistration(max_input_points=480000))
    ids = np.floor(ref.cloud(0)[:, 3]).astype(int)
    assert (np.bincount(ids) > 6 * 1024 + 11).sum() >= 20


def test_scanreg_curvature_exactly_threshold():
    """frame 2417 of the long stream (seed 23) has a curvature of exactly 0.1f at a sector's edge
    candidate: the reference compares the float with the double literal 0.1 (scan_registration.cpp
    :381, :443), so 0.1f > 0.1 makes it lessSharp (a float compare with 0.1f would not)"""
    xyz, _ = synth.frame(23, 2417, 2000)
    ref = _check_frame(xyz)
    c, lab = ref.curvature()
    assert np.any((c == np.float32(0.1)) & (lab == 1))


def test_scanreg_stride_and_nan():
    """(n, 4) input with NaN rows and points inside minimum_range (removeNaN + removeClosed)"""
    xyz, _ = synth.frame(4, 3)
    pts = np.concatenate([xyz, np.zeros((len(xyz), 1), np.float32)], 1)
    pts[::97, 0] = np.nan
    pts[5::211, :3] *= 0.01  # inside 5 m
    ref = O.ScanRegistration()
    ref.input(pts)
    gpu = ScanRegistration()
    gpu.input(pts)
    for a, b in zip(gpu.output(), ref.output()):
        _same_points(a, b)


def test_scanreg_small_and_empty():
    gpu = ScanRegistration()
    gpu.input(np.zeros((0, 3), np.float32))
    assert list(gpu.counts()) == [0, 0, 0, 0, 0]
    xyz, _ = synth.frame(4, 3, n_az=64)  # tiny rings: fewer than 17 points skip selection
    ref = O.ScanRegistration()
    ref.input(xyz)
    gpu.input(xyz)
    for a, b in zip(gpu.output(), ref.output()):
        _same_points(a, b)


def test_async_pinned_ingest_and_overlap():
    """loam_scanreg_input_async from the pinned buffer, overlapped with a
    mapper solve of the previous frame: the same features as the synchronous path"""
    from loam_amd.mapping import BatchMapper
    from loam_amd.scanreg import ScanRegistration
    frames = [synth.frame(4, f, 1000)[0] for f in range(4)]
    ref = ScanRegistration()
    want = []
    for xyz in frames:
        ref.input(xyz)
        want.append([ref.cloud(w) for w in range(5)])
    sr = ScanRegistration()
    m = BatchMapper(1)
    sr.input_async(frames[0])
    for f in range(len(frames)):
        got = [sr.cloud(w) for w in range(5)]  # waits for the frame
        for a, b in zip(got, want[f]):
            assert np.array_equal(a, b)
        m.input(0, got[2], got[4], np.array([0, 0, 0, 1.0]), np.zeros(3))
        if f + 1 < len(frames):
            sr.input_async(frames[f + 1])  # next frame's copy + kernels overlap this solve
        m.solve()
    sr.wait()


def test_batched_frames_match_single():
    """loam_scanreg_input_batch: scans of different sizes and shapes (quantized with tied
    curvatures, column-major with per-laser offsets, a tiny one, an empty one) in one launch
    sequence, each frame's five clouds bit-identical to the single-frame handle's, twice in a row
    (the second batch smaller: the frames past it must not leak into the counts)"""
    from loam_amd.scanreg import ScanRegistrationBatch
    clouds = [synth.frame(1, 0)[0], synth.frame(6, 3, flags=synth.QUANTIZE)[0],
              synth.frame(9, 40, flags=synth.COLUMN_MAJOR | synth.LASER_AZ)[0], synth.frame(4, 3, n_az=64)[0],
              np.zeros((0, 3), np.float32), synth.frame(2, 13)[0]]
    single = ScanRegistration()
    want = []
    for c in clouds:
        single.input(c)
        want.append(single.output())
    b = ScanRegistrationBatch(8)
    b.input_batch(clouds)
    for f, w in enumerate(want):
        assert list(b.counts(f)) == [len(x) for x in w], f
        for k in range(5):
            _same_points(b.cloud(f, k), w[k])
    b.input_batch(clouds[2:4])
    for f, w in enumerate(want[2:4]):
        for k in range(5):
            _same_points(b.cloud(f, k), w[k])
    with pytest.raises(Exception):
        b.counts(3)  # past the last launch's frames
    b.close()
    single.close()


def test_concurrent_sectors_and_reruns():
    """the six sectors of a ring pick concurrently and a sector is rerun where the flags inherited
    from the sector before hit one of its first-5-point picks (scanreg.hip sr_greedy_ring; the
    rule itself: tests/test_sr_conc_rule.py): the frames here exercise both, bit-exact"""
    gpu = ScanRegistration()
    gpu.debug_counters(reset=True)
    for seed, f, flags in [(1, 0, 0), (6, 3, synth.QUANTIZE), (9, 4, synth.COLUMN_MAJOR | synth.LASER_AZ)]:
        xyz, _ = synth.frame(seed, f, 2000, flags=flags)
        _check_frame(xyz, gpu)
    c = gpu.debug_counters()
    assert c[22] > 100, list(c)  # rings with concurrent sectors
    assert c[21] > 10, list(c)   # sector reruns
    gpu.close()
