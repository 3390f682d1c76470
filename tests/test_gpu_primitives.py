"""GPU parity of the kernels behind the mapping stage, each against the CPU oracle.

Bars: VoxelGrid and kNN are index/integer decisions + float arithmetic written in the same
order on both sides -> bit-exact.  Two VoxelGrid kernels: voxel_pcl.h sums a voxel's points in
PCL's order (the libstdc++ std::sort permutation) and is bit-exact against the oracle's PCL
filter; voxel.h (the mapper's) sums them in input order and is bit-exact against the oracle in
that order and within the float summation-order bound of PCL's (helpers.py).  The LM normal equations are fp64 sums in a different
order (device tree reduction vs sequential) -> 1e-10 relative.  The LM solve uses normal
equations (Cholesky) on the device vs Householder QR (Ceres DENSE_QR) in the oracle ->
pose within 1e-9 and identical iteration counts.
"""
import numpy as np
import pytest

import loam_oracle as O
from helpers import assert_centroids_within_order_bound
from loam_amd import _core, prims, synth
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
    with O.voxel_order(1):
        ref_in = O.voxel_grid(cloud, leaf)
    ref = O.voxel_grid(cloud, leaf)
    got = gpu_voxel(cloud, leaf)
    assert got.shape == ref_in.shape
    assert np.array_equal(got.view(np.uint32), ref_in.view(np.uint32))
    assert_centroids_within_order_bound(cloud, leaf, got, ref)
    pcl = prims.voxel_grid_pcl(cloud, leaf)
    assert np.array_equal(pcl.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("n,kv", [(5, 3), (16, 2), (17, 2), (300, 7), (4000, 30), (20000, 1000), (100000, 50)])
def test_sort_perm_matches_std_sort(n, kv):
    """the device std::sort emulation (stdsort.h) against libstdc++ itself: heavy ties"""
    rng = np.random.default_rng(n)
    keys = rng.integers(0, kv, n).astype(np.uint32)
    for waves in (1, 16):
        assert np.array_equal(prims.sort_perm(keys, waves), O.std_sort_perm(keys)), waves


@pytest.mark.parametrize("pattern", range(8))
def test_sort_perm_adversarial(pattern):
    """sorted, reversed, organ-pipe and median-of-3-killer inputs: the depth-limit heap sort
    (__partial_sort) and unbalanced partitions.  Patterns 5-7 are the exact mode's cube
    re-filter: distinct sorted keys (old content) with a few random keys appended (new points),
    which drives introsort into the depth limit on segments of distinct keys (placed by rank,
    stdsort.h ss_depth_limit) and, with ties to the old keys, of tied keys (the heap itself)"""
    n = 4096
    i = np.arange(n)
    if pattern >= 5:
        rng = np.random.default_rng(pattern)
        n_old, n_new = (14000, 60) if pattern == 5 else (4300, 180)
        old = np.sort(rng.choice(1 << 22, n_old, replace=False))
        new = rng.integers(0, 1 << 22, n_new) if pattern != 7 else rng.choice(old, n_new)
        keys = np.concatenate([old, new]).astype(np.uint32)
        for waves in (1, 16):
            assert np.array_equal(prims.sort_perm(keys, waves), O.std_sort_perm(keys)), waves
        return
    if pattern == 0:
        k = i
    elif pattern == 1:
        k = n - i
    elif pattern == 2:
        k = np.where(i < n // 2, i, n - i)
    elif pattern == 3:
        k = np.where(i % 2 == 1, i, n - i)
    else:  # Musser's median-of-3 killer
        h = n // 2
        k = np.empty(n, np.int64)
        k[:h] = np.where(np.arange(h) % 2 == 0, np.arange(h) + 1, h + np.arange(h))
        k[h:] = 2 * (np.arange(n - h) + 1)
    keys = k.astype(np.uint32)
    assert np.array_equal(prims.sort_perm(keys, 16), O.std_sort_perm(keys))


def test_voxel_grid_pcl_order_large_and_tied():
    """PCL-order kernel on a quantized cloud (many points per voxel, coordinates on leaf
    boundaries) and on a 60k-point cloud (global scratch path)"""
    xyz, _ = synth.frame(6, 3, 2000, flags=synth.QUANTIZE)
    pts = np.concatenate([xyz, np.arange(len(xyz), dtype=np.float32)[:, None] % 64], 1)
    for leaf in (0.2, 0.8):
        ref = O.voxel_grid(pts, leaf)
        assert np.array_equal(prims.voxel_grid_pcl(pts, leaf).view(np.uint32), ref.view(np.uint32))
        with O.voxel_order(1):
            assert np.array_equal(gpu_voxel(pts, leaf).view(np.uint32), O.voxel_grid(pts, leaf).view(np.uint32))
        assert_centroids_within_order_bound(pts, leaf, gpu_voxel(pts, leaf), ref)


def _cube_cloud(n_old, n_single, n_pair, seed, leaf):
    """a map cube as the exact mode re-filters it: VoxelGrid output (one point per voxel, in voxel
    order) ++ new points, n_single of them in voxels of their own old point (2-member voxels) and
    n_pair pairs sharing an old point's voxel (3-member voxels)"""
    rng = np.random.default_rng(seed)
    side = int(round(n_old ** (1 / 3) * 1.6))
    xyz = rng.uniform(0, side * leaf, (n_old * 3, 3)).astype(np.float32)
    old = O.voxel_grid(np.concatenate([xyz, rng.uniform(0, 50, (len(xyz), 1)).astype(np.float32)], 1), leaf)
    pick = rng.choice(len(old), n_single + n_pair, replace=False)
    jitter = lambda: np.float32(0.01 * leaf) * rng.uniform(-1, 1, 4).astype(np.float32)  # noqa: E731
    new = [old[i] + jitter() for i in pick[:n_single]]
    new += [old[i] + jitter() for i in pick[n_single:] for _ in range(2)]
    return np.concatenate([old, np.asarray(new, np.float32)]).astype(np.float32)


@pytest.mark.parametrize("n_old,n_single,n_pair", [(13500, 50, 1), (4300, 100, 3), (2000, 5, 0), (2000, 40, 6)])
def test_voxel_grid_pcl_depth_limit(n_old, n_single, n_pair):
    """sorted content with a few points appended drives introsort into its depth limit on long
    segments (tools/introsort_stats.py: the exact mode's cube re-filters); those segments are
    sorted by (key, element) when the heap's tie order cannot show in a centroid and heap-sorted
    otherwise (stdsort.h ss_depth_limit): PCL's bits either way, LDS and global scratch paths"""
    for leaf in (0.4, 0.8):
        pts = _cube_cloud(n_old, n_single, n_pair, n_old + n_pair, leaf)
        ref = O.voxel_grid(pts, leaf)
        assert np.array_equal(prims.voxel_grid_pcl(pts, leaf).view(np.uint32), ref.view(np.uint32)), leaf


def test_voxel_grid_edge_cases():
    assert gpu_voxel(np.zeros((0, 4), np.float32), 0.4).shape == (0, 4)
    one = np.array([[1.5, -2.25, 3.0, 7.0]], np.float32)
    assert np.array_equal(gpu_voxel(one, 0.4), one)
    dup = np.repeat(one, 100, axis=0)  # 100 identical points -> one centroid
    assert np.array_equal(gpu_voxel(dup, 0.4), O.voxel_grid(dup, 0.4))
    assert np.array_equal(prims.voxel_grid_pcl(dup, 0.4), O.voxel_grid(dup, 0.4))
    assert prims.voxel_grid_pcl(np.zeros((0, 4), np.float32), 0.4).shape == (0, 4)
    # negative coordinates straddling zero, several points per voxel
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.uniform(-3, 3, (5000, 3)), rng.uniform(0, 60, (5000, 1))], 1).astype(np.float32)
    with O.voxel_order(1):
        assert np.array_equal(gpu_voxel(pts, 0.4).view(np.uint32), O.voxel_grid(pts, 0.4).view(np.uint32))
    assert np.array_equal(prims.voxel_grid_pcl(pts, 0.4).view(np.uint32), O.voxel_grid(pts, 0.4).view(np.uint32))
    # leaf too small for int32 voxel indices: PCL returns the input unchanged
    far = np.array([[-1e6, 0, 0, 1], [0, 0, 0, 2], [1e6, 1e3, 1e3, 3]], np.float32)
    assert np.array_equal(prims.voxel_grid_pcl(far, 0.01), far)


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
    with O.voxel_order(1):
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
    O.set_voxel_order(1)  # the mapper kernels' order (restored below)
    fixed = O.voxel_grid(frame_clouds[4], leaf)
    if not np.array_equal(O.voxel_grid(fixed, leaf), fixed):
        O.set_voxel_order(0)
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
    O.set_voxel_order(0)
    assert merged == (n_new <= 4096)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("kind,n,m,seed", [("cube", 13500, 400, 11), ("cube", 4300, 300, 1), ("cube", 1500, 600, 4),
                                           ("cube", 9000, 3000, 12), ("stack", 6000, 3000, 5),
                                           ("stack", 28000, 3400, 13), ("stack", 800, 790, 8)])
def test_voxel_grid_pcl_hot_voxels(kind, n, m, seed):
    """voxels of 3+ members (the ones whose centroid shows std::sort's order) on cube-shaped
    clouds (sorted content ++ new points, introsort at its depth limit, literal heap sorts) and on
    raw-feature-shaped clouds (most voxels hot): the pruned emulation of voxel_hot.h, PCL's bits"""
    from test_sort_rule import _stack_cloud, _triples_cloud
    for leaf in (0.4, 0.8):
        pts = _triples_cloud(n, m, seed, leaf) if kind == "cube" else _stack_cloud(n, m, seed, leaf)
        ref = O.voxel_grid(pts, leaf)
        assert np.array_equal(prims.voxel_grid_pcl(pts, leaf).view(np.uint32), ref.view(np.uint32)), leaf
