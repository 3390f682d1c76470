"""CPU: the decomposition behind the sharded LaserMapping, world size 2 over
gloo (127.0.0.1), with the oracle as the per-rank worker and the library's owner function.

- ownership: loam_shard_owner equals a numpy restatement (4 m voxel-aligned blocks, a voxel
  never straddles two owners), and every rank count is used;
- 5-NN: each rank's exact 5-NN over the points it owns, all-gathered and merged by (d, key),
  is the 5-NN over the whole map (the k_knn + k_nn_merge decomposition), and the 1 m
  acceptance of laser_mapping.cpp:557 / :642 is the same;
- normal equations: the rank-ordered sum of the ranks' J^T J / J^T r / cost over their factor
  shares equals the whole problem's, bit-identically on both ranks (the per-iteration
  all-reduce of the sharded LM).
The GPU side of the same decomposition is tests/test_gpu_shard.py.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def owner_np(xyz, leaf, nrank):
    """numpy restatement of comm.h shard_owner"""
    xyz = np.asarray(xyz, dtype=np.float32).reshape(-1, 3)
    inv = np.float32(1.0) / np.float32(leaf)
    bv = max(1, int(np.round(np.float32(4.0) / np.float32(leaf))))
    v = np.floor(xyz * inv).astype(np.int64)
    b = np.floor_divide(v, bv).astype(np.int64)
    u = b.astype(np.uint32)
    with np.errstate(over="ignore"):
        h = (u[:, 0] * np.uint32(73856093)) ^ (u[:, 1] * np.uint32(19349663)) ^ (u[:, 2] * np.uint32(83492791))
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return (h % np.uint32(nrank)).astype(np.int64)


def test_owner_matches_library():
    from loam_amd.mapping import shard_owner
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.uniform(-300, 300, (400, 3)), np.round(rng.uniform(-40, 40, (200, 3)) / 4) * 4,
                          np.round(rng.uniform(-40, 40, (200, 3)) / 0.4) * 0.4]).astype(np.float32)
    for leaf in (0.4, 0.8, 0.2):
        for nrank in (1, 2, 3, 8):
            ref = owner_np(pts, leaf, nrank)
            got = np.array([shard_owner(p, leaf, nrank) for p in pts])
            assert np.array_equal(got, ref), (leaf, nrank)
            if nrank > 1:
                assert len(set(ref)) == nrank
    # a voxel never straddles two owners: points of one voxel share the owner
    v = rng.integers(-200, 200, (300, 3))
    for leaf in (0.4, 0.8):
        lo = (v * np.float32(leaf)).astype(np.float32)
        inner = lo + np.float32(leaf) * rng.uniform(0.05, 0.95, (300, 3)).astype(np.float32)
        same = np.floor(lo / np.float32(leaf)) == np.floor(inner / np.float32(leaf))
        keep = same.all(axis=1)
        assert np.array_equal(owner_np(lo[keep], leaf, 8), owner_np(inner[keep], leaf, 8))


def _scene(seed=5):
    rng = np.random.default_rng(seed)
    # walls and a ground patch sampled densely enough for 5 neighbours within 1 m
    g = rng.uniform([-20, -20, -1.8], [20, 20, -1.7], (6000, 3))
    w = rng.uniform([-20, 11.9, -1.7], [20, 12.1, 4.0], (3000, 3))
    p = rng.uniform([3.0, -0.2, -1.7], [3.4, 0.2, 5.0], (800, 3))
    pts = np.concatenate([g, w, p]).astype(np.float32)
    pts = np.concatenate([pts, np.zeros((len(pts), 1), np.float32)], axis=1)
    q = pts[rng.choice(len(pts), 700, replace=False)].copy()
    q[:, :3] += rng.normal(0, 0.3, (700, 3)).astype(np.float32)
    q = np.concatenate([q, rng.uniform(-30, 30, (100, 4)).astype(np.float32)])
    return pts, q


def _factors(seed=9, n=400):
    rng = np.random.default_rng(seed)
    f = np.zeros((n, 10))
    for i in range(n):
        p = rng.uniform(-20, 20, 3)
        if i % 3 == 0:
            d = rng.normal(size=3)
            f[i] = [1, *p, *(p + rng.normal(0, 0.2, 3)), *(d / np.linalg.norm(d))]
        else:
            nrm = rng.normal(size=3)
            nrm /= np.linalg.norm(nrm)
            f[i] = [3, *p, *nrm, -float(nrm @ p) + rng.normal(0, 0.05), 0, 0]
    x = np.array([0.01, -0.02, 0.015, 1.0, 0.3, -0.2, 0.1])
    x[:4] /= np.linalg.norm(x[:4])
    return f, x


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import loam_oracle as O
    from loam_amd.comm import dist_allgather_bytes, dist_allreduce_ordered
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pts, qs = _scene()
        own = owner_np(pts[:, :3], 0.4, world) == rank
        gid = np.nonzero(own)[0]
        # this rank's exact 5-NN over its own points; key = global index
        idx, d2 = O.knn(pts[own], qs, 5)
        key = np.where(idx >= 0, gid[np.clip(idx, 0, None)], np.iinfo(np.int32).max).astype(np.int32)
        d2 = np.where(idx >= 0, d2, np.float32(np.inf)).astype(np.float32)
        rec = np.concatenate([d2.view(np.int32), key], axis=1)  # (nq, 10) int32
        allrec = dist_allgather_bytes(rec.view(np.uint8).ravel()).view(np.int32).reshape(world, len(qs), 10)
        merged = []
        for i in range(len(qs)):
            cand = []
            for r in range(world):
                cand += list(zip(allrec[r, i, :5].view(np.float32), allrec[r, i, 5:]))
            merged.append(sorted(cand)[:5])
        # the normal equations of this rank's factor share, all-reduced in rank order
        f, x = _factors()
        cost, jtj, jtr, _ = O.lm_normal_eq(f[rank::world], x)
        v = np.concatenate([[cost], jtj.ravel(), jtr])
        dist_allreduce_ordered(v)
        both = dist_allgather_bytes(v.view(np.uint8)).view(np.float64).reshape(world, -1)
        q.put((rank, merged, v, bool(np.array_equal(both[0], both[1]))))
    finally:
        dist.destroy_process_group()


def test_shard_decomposition_gloo():
    import loam_oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pts, qs = _scene()
    idx, d2 = O.knn(pts, qs, 5)
    n_ok = 0
    for rank, merged, v, identical in res:
        assert identical  # bit-identical sums on every rank
        for i in range(len(qs)):
            md = np.array([c[0] for c in merged[i]], dtype=np.float32)
            mk = np.array([c[1] for c in merged[i]])
            assert np.array_equal(md, d2[i]), i
            ok = d2[i, 4] < 1.0
            assert (md[4] < 1.0) == ok
            if ok:
                assert np.array_equal(mk, idx[i]), i
                n_ok += 1
    assert n_ok > 300
    f, x = _factors()
    cost, jtj, jtr, _ = O.lm_normal_eq(f, x)
    full = np.concatenate([[cost], jtj.ravel(), jtr])
    assert np.allclose(res[0][2], full, rtol=1e-12, atol=1e-12)
