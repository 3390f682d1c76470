"""CPU: the visual-odometry LM oracle (oracle_vo_solve: Jet autodiff through CostFunctor32 /
CostFunctor22 + Ceres TR-LM on Euclidean parameters, visual_odometry.cpp:304-509) against
finite differences of a numpy restatement of the functors, a known-answer motion, and the
committed fixture."""
import os

import numpy as np
import pytest

import loam_oracle as O
from vo_problems import make_problem, normal_equations_fd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vo.npz")


@pytest.mark.parametrize("x", [np.array([0.02, -0.01, 0.03, 0.1, -0.05, -0.8]), np.zeros(6),
                               np.array([1e-9, 0.0, -2e-9, 0.0, 0.0, -1.0])])
def test_normal_equations_match_finite_differences(x):
    F, _ = make_problem(np.random.default_rng(1), n32=60, n22=40)
    cost, jtj, jtr, m = O.vo_normal_eq(F, x)
    assert m == 2 * 60 + 40
    fc, fjtj, fjtr = normal_equations_fd(F, x)
    assert abs(cost - fc) <= 1e-12 * max(1.0, abs(fc))
    scale = np.abs(fjtj).max()
    assert np.abs(jtj - fjtj).max() <= 1e-5 * scale
    assert np.abs(jtr - fjtr).max() <= 1e-5 * max(1e-12, np.abs(fjtr).max()) + 1e-12


def test_known_motion_recovered():
    F, xt = make_problem(np.random.default_rng(2), noise=0.0, outliers=0.0)
    x, st = O.vo_solve(F, np.zeros(6), 100)
    assert np.abs(x - xt).max() < 1e-8, (x, xt)
    assert st.successful >= 1 and st.termination in (1, 2, 3)


def test_no_factors():
    x, st = O.vo_solve(np.zeros((0, 10)), np.ones(6), 100)
    assert st.termination == 4 and np.array_equal(x, np.ones(6))


def test_oracle_reproduces_fixture():
    g = np.load(GOLDEN)
    x, st = O.vo_solve(g["factors"], g["x0"], int(g["max_iter"]))
    assert np.array_equal(x, g["x"])
    assert [st.iterations, st.successful, st.invalid, st.termination] == list(g["stats"])
