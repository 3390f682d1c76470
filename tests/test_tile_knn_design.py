"""CPU check of the tile-decomposed kNN design: searching only a query's 2 m
tile's 4 x 4 x 4 one-metre cells gives the same accepted 5-NN as a search of the whole map.

Reference rule (laser_mapping.cpp:554-557, :633-642): the 5 nearest by FLANN's float L2, ties
to the lower submap index; a query is used only if the 5th is within 1 m (squared distance
< 1.0).  Checked on an oracle map after 40 frames with 400 queries per map, float32 distances."""
import numpy as np
import pytest

from helpers import run_sequence


def _knn5(q, pts, keys):
    d = ((pts[None, :, :] - q[:, None, :]) ** 2).sum(axis=2, dtype=np.float32)
    out = []
    for i in range(len(q)):
        o = np.lexsort((keys, d[i]))[:5]
        out.append((d[i][o], keys[o]))
    return out


@pytest.fixture(scope="module")
def steady():
    seq = run_sequence(11, 40, n_az=1000, snapshot_frames=(39,))
    return seq[39]


@pytest.mark.parametrize("key", ["corner", "surf"])
def test_tile_candidates_give_the_accepted_5nn(steady, key):
    pts = np.concatenate([v[:, :3] for v in steady["after"][key].values() if len(v)]).astype(np.float32)
    keys = np.arange(len(pts))
    rng = np.random.default_rng(3)
    q = pts[rng.choice(len(pts), 400, replace=False)] + rng.normal(0, 0.3, (400, 3)).astype(np.float32)
    full = _knn5(q, pts, keys)
    cell = np.floor(pts).astype(np.int64)
    tile = np.floor(q / 2.0).astype(np.int64)
    accepted = 0
    for i in range(len(q)):
        lo = 2 * tile[i] - 1
        m = np.all((cell >= lo) & (cell <= lo + 3), axis=1)
        d_full, k_full = full[i]
        if not d_full[4] < 1.0:
            continue  # rejected either way
        accepted += 1
        (d_t, k_t), = _knn5(q[i:i + 1], pts[m], keys[m])
        assert np.array_equal(k_t, k_full) and np.array_equal(d_t, d_full), i
    assert accepted > 50
