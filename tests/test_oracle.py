"""CPU: pin the oracle (oracle/loam_oracle.cpp) with independent implementations.

The reference has no tests or fixtures and cannot be built here, so the
oracle's restatement is checked against separately written statements of each piece:
  kNN            scipy.spatial.cKDTree + brute force  (pcl::KdTreeFLANN, laser_mapping.cpp:554/:633)
  VoxelGrid      pure-Python PCL applyFilter           (voxel_grid.hpp; laser_mapping.cpp:492-500)
  line PCA       numpy.linalg.eigh                      (laser_mapping.cpp:557-603)
  plane fit      numpy.linalg.lstsq                     (laser_mapping.cpp:642-680)
  Jacobians      central finite differences of the cost
  LM             tests/ceres_lm_np.py (numpy Ceres TR-LM) + known-answer recovery
  ScanRegistration ring ids / curvature / selection limits (scan_registration.cpp:144-513)
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

import ceres_lm_np as NP
import loam_oracle as O


# ---------------------------------------------------------------------------------- kNN
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_knn_matches_ckdtree(seed):
    rng = np.random.default_rng(seed)
    pts = np.zeros((4000, 4), np.float32)
    pts[:, :3] = rng.uniform(-10, 10, (4000, 3))
    q = np.zeros((300, 4), np.float32)
    q[:, :3] = rng.uniform(-10, 10, (300, 3))
    idx, d2 = O.knn(pts, q, 5)
    tree = cKDTree(pts[:, :3].astype(np.float64))
    dd, ii = tree.query(q[:, :3].astype(np.float64), k=5)
    assert np.array_equal(idx, ii)
    # distances are FLANN L2_Simple<float>: float32 sum of squared float32 differences
    diff = pts[idx][:, :, :3] - q[:, None, :3]
    ref = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]
    assert np.array_equal(d2, ref)
    assert np.allclose(d2, dd ** 2, rtol=1e-5, atol=1e-6)


def test_knn_ties_break_by_index():
    pts = np.zeros((6, 4), np.float32)
    pts[:, 0] = [1, -1, 1, -1, 2, 0.5]  # +-1 on the x axis: equal distances
    idx, d2 = O.knn(pts, np.zeros((1, 4), np.float32), 5)
    assert list(idx[0]) == [5, 0, 1, 2, 3]


# ---------------------------------------------------------------------------- VoxelGrid
def voxel_grid_py(pts, leaf, pcl_order=False):
    """pcl::VoxelGrid<PointXYZI>::applyFilter restated in float32 numpy; a voxel's points are
    summed in input order, or (pcl_order) in the order std::sort leaves (idx, point) pairs
    compared by idx (the permutation taken from libstdc++ itself, oracle_std_sort_perm)"""
    p = pts.astype(np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = p[:, :3].min(0), p[:, :3].max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(p[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = O.std_sort_perm(idx.astype(np.uint32)) if pcl_order else np.argsort(idx, kind="stable")
    out = []
    i = 0
    while i < len(order):
        j = i
        s = np.zeros(4, np.float32)
        while j < len(order) and idx[order[j]] == idx[order[i]]:
            s = (s + p[order[j]]).astype(np.float32)
            j += 1
        out.append(s / np.float32(j - i))
        i = j
    return np.array(out, np.float32)


@pytest.mark.parametrize("leaf", [0.2, 0.4, 0.8])
def test_voxel_grid_matches_python(leaf):
    rng = np.random.default_rng(int(leaf * 10))
    pts = np.zeros((3000, 4), np.float32)
    pts[:, :3] = rng.uniform(-3, 3, (3000, 3))
    pts[:, 3] = rng.uniform(0, 64, 3000)
    assert np.array_equal(O.voxel_grid(pts, leaf), voxel_grid_py(pts, leaf, pcl_order=True))
    with O.voxel_order(1):
        assert np.array_equal(O.voxel_grid(pts, leaf), voxel_grid_py(pts, leaf))


def test_std_sort_perm_is_a_sorting_permutation():
    """the oracle's PCL sort: a permutation, keys ascending, and NOT the stable one on ties"""
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 20, 5000).astype(np.uint32)
    perm = O.std_sort_perm(keys)
    assert sorted(perm) == list(range(len(keys)))
    assert np.all(np.diff(keys[perm].astype(np.int64)) >= 0)
    assert not np.array_equal(perm, np.argsort(keys, kind="stable"))


def test_voxel_grid_overflow_returns_input():
    pts = np.zeros((3, 4), np.float32)
    pts[:, 0] = [-1e6, 0, 1e6]
    pts[:, 1] = [-1e6, 0, 1e6]
    pts[:, 2] = [-1e6, 0, 1e6]
    assert np.array_equal(O.voxel_grid(pts, 0.01), pts)


# ------------------------------------------------------------------- correspondence geometry
def test_edge_pca_matches_eigh():
    rng = np.random.default_rng(3)
    n_ok = 0
    for _ in range(200):
        c = rng.uniform(-20, 20, 3)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        spread = rng.uniform(0.02, 0.4)
        nb = np.zeros((5, 4), np.float32)
        nb[:, :3] = c + np.outer(rng.uniform(-0.5, 0.5, 5), d) + rng.normal(0, spread, (5, 3))
        ok, a, b = O.edge_from_nbrs(nb)
        P = nb[:, :3].astype(np.float64)
        ctr = P.sum(0) / 5.0
        Z = P - ctr
        w, V = np.linalg.eigh(Z.T @ Z)
        ok_ref = w[2] > 3 * w[1]
        if abs(w[2] - 3 * w[1]) < 1e-9 * w[2]:
            continue  # knife edge
        assert ok == ok_ref
        if ok:
            n_ok += 1
            v = V[:, 2]
            assert np.allclose(a + b, 2 * ctr, atol=1e-9)
            u = (a - b) / 0.2
            assert abs(abs(u @ v) - 1.0) < 1e-8
    assert n_ok > 20


def test_plane_fit_matches_lstsq():
    rng = np.random.default_rng(4)
    n_ok = n_bad = 0
    for _ in range(200):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        c = rng.uniform(-20, 20, 3)
        u = np.cross(n, rng.normal(size=3))
        v = np.cross(n, u)
        nb = np.zeros((5, 4), np.float32)
        nb[:, :3] = (c + np.outer(rng.uniform(-1, 1, 5), u) + np.outer(rng.uniform(-1, 1, 5), v)
                     + np.outer(rng.normal(0, rng.choice([0.01, 0.3]), 5), n))
        ok, nn, d = O.plane_from_nbrs(nb)
        A = nb[:, :3].astype(np.float64)
        sol = np.linalg.lstsq(A, -np.ones(5), rcond=None)[0]
        d_ref = 1.0 / np.linalg.norm(sol)
        n_ref = sol * d_ref
        ok_ref = bool(np.all(np.abs(A @ n_ref + d_ref) <= 0.2))
        if np.min(np.abs(np.abs(A @ n_ref + d_ref) - 0.2)) < 1e-9:
            continue
        assert ok == ok_ref
        if ok:
            n_ok += 1
            assert np.allclose(nn, n_ref, atol=1e-9) and abs(d - d_ref) < 1e-9 * max(1, abs(d_ref))
        else:
            n_bad += 1
    assert n_ok > 20 and n_bad > 20


# ------------------------------------------------------------------------- LM / Jacobians
@pytest.mark.parametrize("kind", [2, 3])
def test_gradient_matches_finite_differences(kind):
    rng = np.random.default_rng(10 + kind)
    F, xt = NP.make_problem(rng, 15, 40, kind=kind)
    x = NP.plus(xt, rng.normal(0, 0.02, 6))
    cost, jtj, jtr, m = O.lm_normal_eq(F, x)
    assert m == 3 * 15 + 40
    c_np, f_np, J_np = NP.evaluate(F, x)
    assert abs(cost - c_np) < 1e-12 * max(1, c_np)
    assert np.allclose(jtj, J_np.T @ J_np, rtol=1e-10, atol=1e-10)
    h = 1e-6
    g_fd = np.empty(6)
    for c in range(6):
        e = np.zeros(6)
        e[c] = h
        g_fd[c] = (O.lm_normal_eq(F, NP.plus(x, e))[0] - O.lm_normal_eq(F, NP.plus(x, -e))[0]) / (2 * h)
    assert np.allclose(jtr, g_fd, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("seed", range(8))
def test_lm_matches_numpy_ceres(seed):
    rng = np.random.default_rng(100 + seed)
    F, xt = NP.make_problem(rng, 30, 90, kind=3 if seed % 2 else 2)
    x0 = NP.plus(xt, np.concatenate([rng.normal(0, 0.02, 3), rng.normal(0, 0.3, 3)]))
    x_o, st = O.lm_solve(F, x0)
    x_n, sn = NP.lm_solve(F, x0)
    assert (st.iterations, st.successful, st.invalid, st.termination) == \
        (sn["iterations"], sn["successful"], sn["invalid"], sn["termination"])
    assert np.allclose(x_o, x_n, atol=1e-10)
    assert abs(st.initial_cost - sn["initial_cost"]) <= 1e-12 * sn["initial_cost"]
    assert abs(st.final_cost - sn["final_cost"]) <= 1e-10 * max(1.0, sn["final_cost"])


def test_lm_known_answer_recovery():
    rng = np.random.default_rng(7)
    F, xt = NP.make_problem(rng, 60, 200, noise=0.0)
    F = F.copy()
    # noise-free and no outliers: rebuild the perturbed rows from the truth
    R = NP.quat_to_R(xt[:4])
    for r in F:
        if r[0] == 1:
            c = (r[4:7] + r[7:10]) / 2
            d = (r[4:7] - r[7:10]) / 0.2
            r[1:4] = R.T @ (c + 0.3 * d - xt[4:])
        else:
            n, d0 = r[4:7], r[7]
            w = R @ r[1:4] + xt[4:]
            w = w - (n @ w + d0) * n
            r[1:4] = R.T @ (w - xt[4:])
    x0 = NP.plus(xt, np.array([0.03, -0.02, 0.04, 0.3, -0.2, 0.1]))
    x, st = O.lm_solve(F, x0, max_iter=30)
    assert st.final_cost < 1e-16
    ang = 2 * np.arccos(min(1.0, abs(float(x[:4] @ xt[:4]))))
    assert ang < 1e-8 and np.linalg.norm(x[4:] - xt[4:]) < 1e-8


def test_lm_no_factors():
    x0 = np.array([0, 0, 0, 1.0, 1, 2, 3])
    x, st = O.lm_solve(np.zeros((0, 10)), x0)
    assert np.array_equal(x, x0) and st.iterations == 0


# --------------------------------------------------------------------- ScanRegistration
@pytest.fixture(scope="module")
def scan():
    from loam_amd import synth
    xyz, _ = synth.frame(3, 5, 1000)
    sr = O.ScanRegistration()
    sr.input(xyz)
    return xyz, sr.output(), sr.curvature()


def test_scanreg_ring_ids(scan):
    """scanID rule of scan_registration.cpp:241-254 (64 lines, lower rings > 50 dropped)"""
    xyz, clouds, _ = scan
    full = clouds[0]
    ring = np.floor(full[:, 3]).astype(int)
    p = full[:, :3].astype(np.float64)
    ang = np.degrees(np.arctan(p[:, 2] / np.hypot(p[:, 0], p[:, 1])))
    ref = np.where(ang >= -8.83, ((2 - ang) * 3.0 + 0.5).astype(int),
                   32 + ((-8.83 - ang) * 2.0 + 0.5).astype(int))
    assert np.array_equal(ring, ref)
    assert ring.max() <= 50 and np.all(np.diff(ring) >= 0)  # ring-major output
    # intensity = scanID + scanPeriod * relTime; ori may pass endOri by the pi/2 latch
    # tolerance (scan_registration.cpp:262-290) and endOri - startOri >= pi: relTime <= 1.5
    rel = full[:, 3] - ring
    assert np.all((rel >= 0) & (rel <= 0.15 + 1e-6))
    # range filter (removeClosedPointCloud, MINIMUM_RANGE 5 m)
    assert np.all((p ** 2).sum(1) >= 25.0 - 1e-3)


def test_scanreg_curvature_and_selection(scan):
    _, clouds, (curv, lab) = scan
    full = clouds[0]
    ring = np.floor(full[:, 3]).astype(int)
    L = full[:, :3]
    n = len(full)
    d = np.roll(L, 5, 0)  # L[i-5] + ... + L[i-1] - 10 L[i] + L[i+1] + ... + L[i+5], in order
    for k in (4, 3, 2, 1):
        d = d + np.roll(L, k, 0)
    d = d - np.float32(10) * L
    for k in (1, 2, 3, 4, 5):
        d = d + np.roll(L, -k, 0)
    c_ref = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]
    sl = slice(5, n - 5)
    assert np.array_equal(curv[sl], c_ref[sl])
    # selection limits per ring sector (scan_registration.cpp:381-470)
    sharp, less_sharp, flat = clouds[1], clouds[2], clouds[3]
    assert len(sharp) <= 2 * 6 * 51 and len(flat) <= 4 * 6 * 51
    assert np.all(curv[lab == 2] > 0.1) and np.all(curv[lab == -1] < 0.1)
    for r in np.unique(ring):
        assert (lab[ring == r] == 2).sum() <= 12 and (lab[ring == r] == -1).sum() <= 24
        assert (lab[ring == r] >= 1).sum() <= 120
    assert len(less_sharp) == (lab >= 1).sum()
