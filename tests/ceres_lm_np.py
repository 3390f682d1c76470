"""Independent numpy restatement of the mapping/odometry solve — TEST INFRASTRUCTURE ONLY.

A second, separately written statement of Ceres 2.0's TrustRegionMinimizer with the
LevenbergMarquardt strategy as the reference configures it (laser_mapping.cpp:709-717,
laser_odometry.cpp:500-509: DENSE_QR, max_num_iterations = 4, HuberLoss(0.1),
EigenQuaternionParameterization), used to pin the C++ oracle (oracle/loam_oracle.cpp
lm_solve), since the reference itself cannot be built here.

Deliberately different arithmetic from the oracle: residuals and Jacobians are vectorized
(rotation matrix instead of the quaternion sandwich), the damped step comes from
numpy.linalg.lstsq (SVD) on [J_scaled; D] instead of Householder QR.  Agreement is to
~1e-12, not bit-exact.

Factor rows (10 doubles): type, p[3], a[3], b[3] —
  1 edge   (lidarFactor.hpp:14-60 LidarEdgeFactor):    r = ((lp - a) x (lp - b)) / |a - b|
  2 plane  (lidarFactor.hpp:62-104 LidarPlaneFactor):  r = (lp - j) . n   (a = j, b = n)
  3 plane  (lidarFactor.hpp:106-144 LidarPlaneNormFactor): r = n . lp + d  (a = n, b[0] = d)
with lp = R(q) p + t, x = (qx, qy, qz, qw, tx, ty, tz).
"""
import numpy as np


def quat_to_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def quat_mul(a, b):
    """Hamilton product, xyzw storage"""
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def plus(x, d):
    """EigenQuaternionParameterization::Plus (q' = [sin|d|/|d| d, cos|d|] * q) + Euclidean t"""
    nd = np.linalg.norm(d[:3])
    q = x[:4]
    if nd > 0:
        dq = np.concatenate([np.sin(nd) / nd * d[:3], [np.cos(nd)]])
        q = quat_mul(dq, q)
    return np.concatenate([q, x[4:] + d[3:]])


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def residuals(F, x, jac=True):
    """raw residuals (M,) , row -> factor id, and local Jacobian (M, 6) w.r.t. (dtheta, dt)"""
    R = quat_to_R(x[:4])
    t = x[4:]
    rs, Js, fid = [], [], []
    for k, f in enumerate(F):
        typ, p, a, b = int(f[0]), f[1:4], f[4:7], f[7:10]
        Rp = R @ p
        lp = Rp + t
        # d lp / d dtheta for the left-multiplied quaternion increment = -2 [Rp]x
        dlp = np.hstack([-2.0 * skew(Rp), np.eye(3)])
        if typ == 1:
            dn = np.linalg.norm(a - b)
            r = np.cross(lp - a, lp - b) / dn
            drdlp = skew(b - a) / dn  # d (u x w) / d lp with u = lp - a, w = lp - b
            rs.extend(r)
            Js.extend(drdlp @ dlp)
            fid.extend([k] * 3)
        elif typ == 2:
            rs.append(np.dot(lp - a, b))
            Js.append(b @ dlp)
            fid.append(k)
        else:
            rs.append(np.dot(a, lp) + b[0])
            Js.append(a @ dlp)
            fid.append(k)
    return np.array(rs), np.array(fid), (np.array(Js) if jac else None)


def huber(s, a=0.1):
    """ceres::HuberLoss rho(s), rho'(s) for squared norm s"""
    b = a * a
    big = s > b
    r = np.sqrt(np.where(big, s, 1.0))
    rho0 = np.where(big, 2 * a * r - b, s)
    rho1 = np.where(big, np.maximum(np.finfo(float).tiny, a / r), 1.0)
    return rho0, rho1


def evaluate(F, x, jac=True):
    """cost (0.5 sum rho), Corrector-scaled residuals / Jacobian (ceres/corrector.cc: rho'' < 0)"""
    r, fid, J = residuals(F, x, jac)
    sq = np.bincount(fid, weights=r * r, minlength=len(F))
    rho0, rho1 = huber(sq)
    cost = 0.5 * rho0.sum()
    if not jac:
        return cost, None, None
    sc = np.sqrt(rho1)[fid]
    return cost, r * sc, J * sc[:, None]


def lm_solve(F, x0, max_iter=4):
    """returns x (best), dict(iterations, successful, invalid, termination, initial_cost, final_cost)"""
    F = np.asarray(F, dtype=np.float64).reshape(-1, 10)
    x = np.array(x0, dtype=np.float64)
    if len(F) == 0:
        return x, dict(iterations=0, successful=0, invalid=0, termination=4, initial_cost=0.0,
                       final_cost=0.0)
    radius, dec = 1e4, 2.0
    cost, f, J = evaluate(F, x)
    stats = dict(iterations=0, successful=0, invalid=0, termination=0, initial_cost=cost)
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))  # Jacobi scaling, fixed at iteration 0
    J = J * scale

    def gmax_of(xx, JJ, ff):
        g = JJ.T @ ff
        return np.abs(xx - plus(xx, -g)).max()

    gmax = gmax_of(x, J, f)
    best, best_cost = x.copy(), np.inf
    it, ok, reuse, invalid_run = 0, True, False, 0
    diag = None
    while True:
        if ok and cost < best_cost:
            best, best_cost = x.copy(), cost
        if it >= max_iter:
            term = 0
            break
        if ok and gmax <= 1e-10:
            term = 3
            break
        if radius <= 1e-32:
            term = 5
            break
        it += 1
        ok = False
        if not reuse:
            diag = np.clip((J * J).sum(0), 1e-6, 1e32)
        D = np.sqrt(diag / radius)
        A = np.vstack([J, np.diag(D)])
        rhs = np.concatenate([f, np.zeros(6)])
        y = np.linalg.lstsq(A, rhs, rcond=None)[0]
        reuse = True
        step = -y
        js = J @ step
        mcc = -np.sum(js * (f + js / 2.0))
        if not (np.all(np.isfinite(y)) and mcc > 0):
            stats["invalid"] += 1
            invalid_run += 1
            if invalid_run >= 5:
                term = 5
                break
            radius /= dec
            dec *= 2.0
            continue
        invalid_run = 0
        cand = plus(x, step * scale)
        cand_cost = evaluate(F, cand, jac=False)[0]
        if np.linalg.norm(x - cand) <= 1e-8 * (np.linalg.norm(x) + 1e-8):
            term = 2
            break
        if abs(cost - cand_cost) <= 1e-6 * cost:
            term = 1
            break
        rel = (cost - cand_cost) / mcc
        if rel > 1e-3:
            x = cand
            cost, f, J = evaluate(F, x)
            J = J * scale
            gmax = gmax_of(x, J, f)
            ok = True
            stats["successful"] += 1
            radius = min(1e16, radius / max(1.0 / 3.0, 1.0 - (2.0 * rel - 1.0) ** 3))
            dec = 2.0
            reuse = False
        else:
            radius /= dec
            dec *= 2.0
    stats.update(iterations=it, termination=term, final_cost=best_cost)
    return best, stats


def make_problem(rng, n_edge=40, n_plane=120, noise=0.01, kind=3):
    """factors observed from a random scene under a random true pose; returns F, x_true"""
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    ang = rng.uniform(0.0, 0.3)
    q = np.concatenate([np.sin(ang / 2) * ax, [np.cos(ang / 2)]])
    t = rng.normal(0, 2.0, 3)
    R = quat_to_R(q)
    rows = []
    for _ in range(n_edge):  # point on a 3D line, observed in the body frame
        c = rng.uniform(-20, 20, 3)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        w = c + rng.uniform(-1, 1) * d + rng.normal(0, noise, 3)
        p = R.T @ (w - t)
        rows.append(np.concatenate([[1], p, c + 0.1 * d, c - 0.1 * d]))
    for _ in range(n_plane):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        c = rng.uniform(-20, 20, 3)
        u = np.cross(n, rng.normal(size=3))
        w = c + u * rng.uniform(-1, 1) + n * rng.normal(0, noise)
        p = R.T @ (w - t)
        if kind == 3:
            rows.append(np.concatenate([[3], p, n, [-np.dot(n, c), 0, 0]]))
        else:
            rows.append(np.concatenate([[2], p, c, n]))
    # a few gross outliers exercise the Huber corrector
    for r in rows[:: max(1, len(rows) // 8)]:
        r[1:4] += rng.normal(0, 0.5, 3)
    return np.array(rows), np.concatenate([q, t])
