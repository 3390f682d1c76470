"""Shared test helpers: synthetic sequences run through the CPU oracle, teacher-forcing
snapshots of the oracle mapper, pose-difference metrics."""
import numpy as np

import loam_oracle as O
from loam_amd import synth

N_CUBES = 21 * 21 * 11


def quat_angle(q1, q2):
    """rotation angle (rad) of q1^-1 q2 (xyzw)"""
    q1 = np.asarray(q1, dtype=np.float64)
    q2 = np.asarray(q2, dtype=np.float64)
    q1 = q1 / np.linalg.norm(q1)
    q2 = q2 / np.linalg.norm(q2)
    # conj(q1) * q2: w = q1.q2, v = w1 v2 - w2 v1 - v1 x v2 (atan2 keeps tiny angles exact)
    w = float(np.dot(q1, q2))
    v = q1[3] * q2[:3] - q2[3] * q1[:3] - np.cross(q1[:3], q2[:3])
    return 2.0 * np.arctan2(float(np.linalg.norm(v)), abs(w))


def snapshot(mp):
    cen, q, t = mp.get_state()
    return dict(cen=cen.copy(), q=q.copy(), t=t.copy(), corner=mp.cubes(0), surf=mp.cubes(1))


def run_sequence(seed, n_frames, n_az=2000, snapshot_frames=(), keep_features=True):
    """Oracle pipeline (scan registration -> odometry -> mapping) over a synthetic sequence.
    For frames in snapshot_frames, the mapper state BEFORE solveMapping is recorded."""
    sr, od, mp = O.ScanRegistration(), O.LaserOdometry(), O.LaserMapping()
    frames = []
    for f in range(n_frames):
        xyz, gt = synth.frame(seed, f, n_az)
        sr.input(xyz)
        od.input(*sr.output())
        od.solve()
        q, t, _, _, _ = od.output()
        corner, surf = od.cloud(0), od.cloud(1)
        rec = dict(frame=f, q_wodom=q, t_wodom=t, gt=gt)
        if keep_features:
            rec.update(corner=corner, surf=surf)
        if f in snapshot_frames:
            rec["before"] = snapshot(mp)
        mp.input(corner, surf, None, q, t)
        mp.solve()
        rec["pose"] = mp.pose()
        rec["stats"] = mp.stats()
        if f in snapshot_frames:
            rec["after"] = snapshot(mp)
            rec["factors"] = [mp.factors(0), mp.factors(1)]
            rec["round_pose"] = [mp.round_pose(0), mp.round_pose(1)]
        frames.append(rec)
    return frames


def load_state(mapper, stream, snap):
    mapper.set_state(stream, snap["cen"], snap["q"], snap["t"])
    for which, key in ((0, "corner"), (1, "surf")):
        for cube, pts in snap[key].items():
            mapper.set_cube(stream, which, cube, pts)


def voxel_members(pts, leaf):
    """PCL VoxelGrid grouping (voxel_grid.hpp): the voxel idx of every point and, per output
    voxel in increasing idx, its member count and largest |coordinate| (x, y, z, intensity)"""
    p = np.asarray(pts, np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = p[:, :3].min(0), p[:, :3].max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    div = np.floor(mx * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(p[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    uniq, inverse, counts = np.unique(idx, return_inverse=True, return_counts=True)
    amax = np.zeros((len(uniq), 4), np.float64)
    np.maximum.at(amax, inverse, np.abs(p.astype(np.float64)))
    return counts, amax


def assert_centroids_within_order_bound(pts, leaf, got, ref):
    """got and ref: VoxelGrid outputs of pts that differ only in the order a voxel's points are
    summed (float32).  Two orders of m float additions differ by at most 2 (m - 1) u sum|x_i|
    (u = 2^-24), and the division by m adds one rounding to each: per component
    |got - ref| <= (2 (m - 1) + 2) u max|x_i| * m / m.  Voxels of 1 or 2 points are exact
    (float addition commutes)."""
    got, ref = np.asarray(got, np.float32), np.asarray(ref, np.float32)
    assert got.shape == ref.shape
    m, amax = voxel_members(pts, leaf)
    assert len(m) == len(got)
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    bound = (2.0 * (m[:, None] - 1) + 2.0) * 2.0 ** -24 * amax
    assert np.all(d <= bound), float((d - bound).max())
    assert np.array_equal(got[m <= 2].view(np.uint32), ref[m <= 2].view(np.uint32))
