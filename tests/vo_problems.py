"""Synthetic visual-odometry problems (VisualOdometry::solveNlsAll residual blocks,
src/visual_odometry/src/visual_odometry.cpp:346-493) with a known camera motion, and a numpy
restatement of the two functors (ceres_cost_function.h:58-189) for finite-difference checks."""
import numpy as np
from scipy.spatial.transform import Rotation


def make_problem(rng, n32=800, n22=600, noise=1e-3, outliers=0.03, w=(0.01, -0.02, 0.005),
                 t=(0.05, -0.02, -0.9)):
    w, t = np.asarray(w, float), np.asarray(t, float)
    R = Rotation.from_rotvec(w).as_matrix()
    n = n32 + n22
    X0 = np.stack([rng.uniform(-20, 20, n), rng.uniform(-3, 3, n), rng.uniform(5, 40, n)], 1)
    X0 = X0.astype(np.float32).astype(np.float64)  # point_3d_rect0_0 is a float vector
    X1 = X0 @ R.T + t
    u1 = X1[:, :2] / X1[:, 2:3] + rng.normal(0, noise, (n, 2))
    bad = rng.random(n) < outliers
    u1[bad] += rng.normal(0, 0.05, (bad.sum(), 2))
    F = np.zeros((n, 10))
    F[:n32, 0] = 4
    F[:n32, 1:4] = X0[:n32]
    F[:n32, 4:6] = u1[:n32]
    F[n32:, 0] = 5
    F[n32:, 4:6] = X0[n32:, :2] / X0[n32:, 2:3]
    F[n32:, 7:9] = u1[n32:]
    return F, np.concatenate([w, t])


def residuals(F, x):
    R = Rotation.from_rotvec(x[:3]).as_matrix()
    t = x[3:]
    out = []
    for f in F:
        if f[0] == 4:
            P = R @ f[1:4] + t
            out.append(np.array([P[0] - P[2] * f[4], P[1] - P[2] * f[5]]))
        else:
            q = R @ np.array([f[4], f[5], 1.0])
            out.append(np.array([np.dot(np.array([f[7], f[8], 1.0]), np.cross(t, q))]))
    return out


def normal_equations_fd(F, x, h=1e-7):
    """Huber(0.1)-corrected J^T J, J^T r, cost with central-difference Jacobians"""
    rs = residuals(F, x)
    Js = [np.zeros((len(r), 6)) for r in rs]
    for k in range(6):
        e = np.zeros(6)
        e[k] = h
        rp, rm = residuals(F, x + e), residuals(F, x - e)
        for i in range(len(rs)):
            Js[i][:, k] = (rp[i] - rm[i]) / (2 * h)
    jtj, jtr, cost = np.zeros((6, 6)), np.zeros(6), 0.0
    for r, J in zip(rs, Js):
        s = float(r @ r)
        if s > 0.01:
            rho0, rho1 = 2 * 0.1 * np.sqrt(s) - 0.01, 0.1 / np.sqrt(s)
        else:
            rho0, rho1 = s, 1.0
        cost += 0.5 * rho0
        jtj += rho1 * J.T @ J
        jtr += rho1 * J.T @ r
    return cost, jtj, jtr
