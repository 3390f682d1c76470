"""GPU parity of the kernels behind the mapping stage, each against the CPU oracle.

Bars: VoxelGrid and kNN are index/integer decisions + float arithmetic written in the same
order on both sides -> bit-exact.  The LM normal equations are fp64 sums in a different
order (device tree reduction vs sequential) -> 1e-10 relative.  The LM solve uses normal
equations (Cholesky) on the device vs Householder QR (Ceres DENSE_QR) in the oracle ->
pose within 1e-9 and identical iteration counts.
"""
import numpy as np
import pytest

import loam_oracle as O
from loam_amd import _core, synth
from loam_amd._core import lib, ptr, check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frame_clouds():
    xyz, _ = synth.frame(3, 25)
    sr = O.ScanRegistration()
    sr.input(xyz)
    return sr.output()


def gpu_voxel(pts, leaf):
    pts = _core.f32x4(pts)
    out = np.empty_like(pts)
    n = _core.c_i32()
    check(lib().loam_voxel_grid(0, ptr(pts), len(pts), leaf, ptr(out), n))
    return out[: n.value]


@pytest.mark.parametrize("which,leaf", [(4, 0.8), (2, 0.4), (0, 0.2), (4, 0.2)])
def test_voxel_grid_bit_exact(frame_clouds, which, leaf):
    cloud = frame_clouds[which]
    if which == 0:  # one ring-sized cloud, as in scan_registration.cpp:497-501
        cloud = cloud[:1800]
    ref = O.voxel_grid(cloud, leaf)
    got = gpu_voxel(cloud, leaf)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_voxel_grid_edge_cases():
    assert gpu_voxel(np.zeros((0, 4), np.float32), 0.4).shape == (0, 4)
    one = np.array([[1.5, -2.25, 3.0, 7.0]], np.float32)
    assert np.array_equal(gpu_voxel(one, 0.4), one)
    dup = np.repeat(one, 100, axis=0)  # 100 identical points -> one centroid
    assert np.array_equal(gpu_voxel(dup, 0.4), O.voxel_grid(dup, 0.4))
    # negative coordinates straddling zero, several points per voxel
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.uniform(-3, 3, (5000, 3)), rng.uniform(0, 60, (5000, 1))], 1).astype(np.float32)
    assert np.array_equal(gpu_voxel(pts, 0.4).view(np.uint32), O.voxel_grid(pts, 0.4).view(np.uint32))


def test_knn_radius_exact(frame_clouds):
    pts = frame_clouds[2][:, :4].copy()  # lessSharp cloud
    rng = np.random.default_rng(1)
    q = pts[rng.integers(0, len(pts), 3000)].copy()
    q[:, :3] += rng.normal(0, 0.3, (len(q), 3)).astype(np.float32)
    k = 5
    idx = np.empty((len(q), k), np.int32)
    d2 = np.empty((len(q), k), np.float32)
    check(lib().loam_knn_radius(0, ptr(pts), len(pts), ptr(q), len(q), k, 1.0, ptr(idx), ptr(d2)))
    ridx, rd2 = O.knn(pts, q, k)
    valid = rd2 < 1.0
    assert np.array_equal(valid, idx >= 0)
    assert np.array_equal(idx[valid], ridx[valid])
    assert np.array_equal(d2[valid], rd2[valid])


def _factor_set(n_edge=700, n_plane=2500, seed=0):
    rng = np.random.default_rng(seed)
    f = []
    for _ in range(n_edge):
        p = rng.uniform(-30, 30, 3)
        a = p + rng.normal(0, 0.3, 3)
        d = rng.normal(0, 1, 3)
        d /= np.linalg.norm(d)
        f.append([1, *p, *(a + 0.1 * d), *(a - 0.1 * d)])
    for _ in range(n_plane):
        p = rng.uniform(-30, 30, 3)
        n = rng.normal(0, 1, 3)
        n /= np.linalg.norm(n)
        d = -float(n @ p) + rng.normal(0, 0.2)
        f.append([3, *p, *n, d, 0, 0])
    for _ in range(300):
        p = rng.uniform(-30, 30, 3)
        n = rng.normal(0, 1, 3)
        n /= np.linalg.norm(n)
        j = p + rng.normal(0, 0.2, 3)
        f.append([2, *np.float32(p), *j, *n])
    f = np.array(f, dtype=np.float64)
    f[:, 1:4] = f[:, 1:4].astype(np.float32)  # curr_point comes from float clouds
    return f


def test_lm_normal_equations(frame_clouds):
    f = _factor_set()
    x = np.array([0.01, -0.02, 0.03, 0.0, 0.5, -0.2, 0.1])
    x[:4] /= 1.0
    x[3] = np.sqrt(1 - np.sum(x[:3] ** 2))
    cost = np.empty(1); jtj = np.empty(36); jtr = np.empty(6)
    rows = check(lib().loam_lm_normal_equations(0, ptr(f), len(f), ptr(x), ptr(cost), ptr(jtj), ptr(jtr)))
    rc, rjtj, rjtr, rrows = O.lm_normal_eq(f, x)
    assert rows == rrows
    assert abs(cost[0] - rc) <= 1e-10 * abs(rc)
    assert np.max(np.abs(jtj.reshape(6, 6) - rjtj)) <= 1e-10 * np.max(np.abs(rjtj))
    assert np.max(np.abs(jtr - rjtr)) <= 1e-10 * np.max(np.abs(rjtr))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lm_solve_matches_oracle(seed):
    f = _factor_set(seed=seed)
    x0 = np.array([0.02, -0.01, 0.015, 0.0, 0.3, -0.4, 0.2])
    x0[3] = np.sqrt(1 - np.sum(x0[:3] ** 2))
    xr, str_ = O.lm_solve(f, x0, 4)
    xg = x0.copy()
    st = _core.LMStats()
    check(lib().loam_lm_solve(0, ptr(f), len(f), ptr(xg), 4, st))
    assert st.iterations == str_.iterations
    assert st.successful == str_.successful
    assert np.max(np.abs(xg - xr)) < 1e-9
    assert abs(st.final_cost - str_.final_cost) <= 1e-9 * max(1.0, str_.final_cost)


def test_lm_solve_no_factors():
    x = np.array([0, 0, 0, 1, 1, 2, 3], dtype=np.float64)
    st = _core.LMStats()
    check(lib().loam_lm_solve(0, None, 0, ptr(x), 4, st))
    assert np.array_equal(x, [0, 0, 0, 1, 1, 2, 3])
    assert st.termination == 4


def test_voxel_grid_many_unique_voxels():
    """more unique voxels than one LDS pass (12288): idx-range groups path"""
    rng = np.random.default_rng(5)
    pts = np.concatenate([rng.uniform(-20, 20, (60000, 3)), rng.uniform(0, 60, (60000, 1))], 1).astype(np.float32)
    ref = O.voxel_grid(pts, 0.5)
    got = gpu_voxel(pts, 0.5)
    assert len(ref) > 12288
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("leaf,n_new", [(0.4, 1), (0.4, 65), (0.4, 300), (0.8, 1024), (0.4, 1025),
                                        (0.8, 1500), (0.4, 2049), (0.4, 4096), (0.4, 5000)])
def test_voxel_merge_bit_exact(frame_clouds, leaf, n_new):
    """map update path: VoxelGrid(fixed ++ added) with `fixed` a VoxelGrid fixed point; the merge
    kernel (n_new <= 4096) must equal the full filter bit for bit"""
    from loam_amd import prims
    fixed = O.voxel_grid(frame_clouds[4], leaf)
    if not np.array_equal(O.voxel_grid(fixed, leaf), fixed):
        pytest.skip("content is not a fixed point")
    rng = np.random.default_rng(n_new)
    # half the new points land in occupied voxels (jittered copies), half anywhere nearby
    pick = fixed[rng.integers(0, len(fixed), n_new // 2)].copy()
    pick[:, :3] += rng.uniform(-0.05, 0.05, (len(pick), 3)).astype(np.float32)
    lo, hi = fixed[:, :3].min(0), fixed[:, :3].max(0)
    far = np.concatenate([rng.uniform(lo, hi, (n_new - len(pick), 3)),
                          rng.uniform(0, 64, (n_new - len(pick), 1))], 1).astype(np.float32)
    added = np.concatenate([pick, far]).astype(np.float32)
    got, merged = prims.voxel_merge(fixed, added, leaf)
    ref = O.voxel_grid(np.concatenate([fixed, added]), leaf)
    assert merged == (n_new <= 4096)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
