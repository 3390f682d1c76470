"""GPU: the visual-odometry pose solve (loam_vo_solve; VisualOdometry::solveNlsAll,
visual_odometry.cpp:304-509) against the oracle (Jet autodiff + Ceres TR-LM restatement):
identical iteration / success / invalid / termination counts and the solution within 1e-9
(analytic Jacobians vs Jets differ in rounding only), for single and batched problems, the
committed fixture, a known motion, and the empty problem."""
import os

import numpy as np
import pytest

import loam_oracle as O
from loam_amd import vo
from vo_problems import make_problem

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vo.npz")


def same(st, ost):
    return [st.iterations, st.successful, st.invalid, st.termination] == \
        [ost.iterations, ost.successful, ost.invalid, ost.termination]


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    F, _ = make_problem(rng, noise=2e-3 * (seed + 1))
    x0 = np.zeros(6) if seed % 2 == 0 else np.array([0.008, -0.018, 0.004, 0.04, -0.01, -0.85])
    x, st = vo.solve([F], [x0])
    ox, ost = O.vo_solve(F, x0, 100)
    assert same(st[0], ost), (st[0].iterations, ost.iterations, st[0].termination, ost.termination)
    assert np.abs(x[0] - ox).max() < 1e-9
    assert abs(st[0].final_cost - ost.final_cost) <= 1e-9 * ost.final_cost


def test_batched_problems():
    probs, x0s = [], []
    for k in range(12):
        rng = np.random.default_rng(100 + k)
        F, _ = make_problem(rng, n32=300 + 50 * k, n22=200, w=rng.normal(0, 0.02, 3), t=(0.0, 0.0, -1.0 + 0.05 * k))
        probs.append(F)
        x0s.append(np.zeros(6))
    probs.append(np.zeros((0, 10)))  # an empty problem in the batch
    x0s.append(np.full(6, 0.5))
    x, st = vo.solve(probs, x0s)
    for k, F in enumerate(probs[:-1]):
        ox, ost = O.vo_solve(F, x0s[k], 100)
        assert same(st[k], ost), k
        assert np.abs(x[k] - ox).max() < 1e-9, k
    assert st[-1].termination == 4 and np.array_equal(x[-1], np.full(6, 0.5))


def test_fixture_and_known_motion():
    g = np.load(GOLDEN)
    x, st = vo.solve([g["factors"]], [g["x0"]], int(g["max_iter"]))
    assert [st[0].iterations, st[0].successful, st[0].invalid, st[0].termination] == list(g["stats"])
    assert np.abs(x[0] - g["x"]).max() < 1e-9
    F, xt = make_problem(np.random.default_rng(2), noise=0.0, outliers=0.0)
    x, _ = vo.solve([F])
    assert np.abs(x[0] - xt).max() < 1e-8


def test_factors_from_matches():
    """vo_factors: CostFunctor32 where the previous point has a depth, CostFunctor22 elsewhere"""
    from loam_amd.depth import KITTI_P_RECT0
    rng = np.random.default_rng(9)
    prev = np.stack([rng.uniform(0, 1242, 50), rng.uniform(0, 375, 50)], 1)
    curr = prev + rng.normal(0, 2, (50, 2))
    d0 = np.where(rng.random(50) < 0.6, rng.uniform(5, 40, 50), -1.0)
    F = vo.vo_factors(prev, curr, d0, KITTI_P_RECT0)
    assert np.array_equal(F[:, 0] == 4, d0 > 0)
    x, st = vo.solve([F])
    assert st[0].termination in (0, 1, 2, 3)
