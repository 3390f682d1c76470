"""Sizing data for a tile-decomposed kNN: on a steady-state oracle map, queries per
2 m tile and map points in each tile's 4 x 4 x 4 one-metre cells (the LDS a tile would stage).

    python tools/tile_stats.py [frames]      (CPU only: the oracle pipeline, ~20 ms per frame)

Queries: the frame's lessSharp / lessFlat features downsampled with the mapper's leaves
(0.2 / 0.4 m, voxel centroids) and moved to the map frame with the frame's final pose."""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vloam-noted_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from helpers import run_sequence  # noqa: E402
from scipy.spatial.transform import Rotation as R  # noqa: E402


def downsample(p, leaf):
    k = np.floor(p / leaf).astype(np.int64)
    _, inv = np.unique(k, axis=0, return_inverse=True)
    out = np.zeros((inv.max() + 1, 3))
    np.add.at(out, inv.ravel(), p)
    return out / np.bincount(inv.ravel())[:, None]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    f = n - 1
    seq = run_sequence(7, n, snapshot_frames=(f,))
    rec = seq[f]
    q, t = rec["pose"]
    rot = R.from_quat(q)
    for which, key, leaf in ((0, "corner", 0.2), (1, "surf", 0.4)):
        mp = np.concatenate([v[:, :3] for v in rec["after"][key].values() if len(v)])
        qs = rot.apply(downsample(rec[key][:, :3].astype(np.float64), leaf)) + t
        cells = collections.Counter(map(tuple, np.floor(mp).astype(np.int64)))
        tiles = collections.Counter(map(tuple, np.floor(qs / 2.0).astype(np.int64)))
        staged = []
        for (tx, ty, tz) in tiles:
            s = 0
            for dx in range(-1, 3):
                for dy in range(-1, 3):
                    for dz in range(-1, 3):
                        s += cells.get((2 * tx + dx, 2 * ty + dy, 2 * tz + dz), 0)
            staged.append(s)
        qpt = np.array(list(tiles.values()))
        st = np.array(staged)
        pct = lambda a: " / ".join(f"{np.percentile(a, p):.0f}" for p in (50, 90, 99, 100))  # noqa: E731
        print(f"{key}: map {len(mp)} points in {len(cells)} 1 m cells; {len(qs)} queries in {len(tiles)} 2 m tiles")
        print(f"  queries per tile  p50 / p90 / p99 / max: {pct(qpt)}")
        print(f"  staged map points p50 / p90 / p99 / max: {pct(st)}  ({16 * st.max() / 1024:.1f} KiB at the max)")
        print(f"  staged points per query (sum over tiles / queries): {st.sum() / len(qs):.1f}")


if __name__ == "__main__":
    main()
