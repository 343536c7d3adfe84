"""Oracle pinning for descriptor matching (oracle/or_match.cpp restating features.h:224-273 with
FLANN's L2_Simple<float>): known answers and independent numpy restatements.  Parity vs real
PCL/FLANN is unpinned (no fixtures in the reference); ties and non-finite queries follow the
documented restatement choices."""
import numpy as np
import pytest

import oracle_lib as O
from match_data import fpfh_like, pair, shot_like


def l2_simple(a, b):
    """FLANN L2_Simple<float> in numpy: sequential float32 adds over the dimensions."""
    r = np.zeros(np.broadcast_shapes(a.shape[:-1], b.shape[:-1]), np.float32)
    for k in range(a.shape[-1]):
        d = (a[..., k] - b[..., k]).astype(np.float32)
        r = (r + (d * d).astype(np.float32)).astype(np.float32)
    return r


@pytest.mark.parametrize("kind", ["fpfh", "shot"])
def test_nearest_is_sequential_float_argmin(kind):
    src, tgt = pair(kind, 120, 150, seed=1)
    idx, dist = O.nearest_descriptor(src, tgt)
    full = l2_simple(src[:, None, :], tgt[None, :, :])
    ref = np.argmin(full, axis=1)  # first minimum = lowest row on ties
    assert np.array_equal(idx, ref)
    assert np.array_equal(dist.view(np.uint32), full[np.arange(len(src)), ref].view(np.uint32))


def test_permuted_copy_is_recovered_mutually():
    rng = np.random.default_rng(3)
    src = fpfh_like(rng, 200)
    perm = rng.permutation(200)
    tgt = src[perm]
    q, m = O.correspondences(src, tgt)
    assert np.array_equal(q, np.arange(200))
    assert np.array_equal(perm[m], q)


def test_ties_lowest_row_and_nonfinite_rows():
    rng = np.random.default_rng(4)
    tgt = shot_like(rng, 10)
    tgt[7] = tgt[2]          # duplicate target rows: lowest row wins
    tgt[5, 3] = np.nan       # not indexed
    src = tgt[[2, 5, 7, 0]].copy()
    src[3, 0] = np.inf       # non-finite query: no match
    idx, dist = O.nearest_descriptor(src, tgt)
    assert idx[0] == 2 and idx[2] == 2 and dist[0] == 0.0
    assert idx[1] != 5 and idx[3] == -1 and np.isnan(dist[3])
    q, m = O.correspondences(src, tgt)
    assert list(q) == [0] and list(m) == [2]  # target 2's nearest source is row 0 (tie with row 2)


def test_empty_and_mutual_definition():
    a = shot_like(np.random.default_rng(5), 5)
    assert O.correspondences(a, a[:0])[0].size == 0
    assert O.correspondences(a[:0], a)[0].size == 0
    src, tgt = pair("shot", 300, 260, seed=6)
    s2t, _ = O.nearest_descriptor(src, tgt)
    t2s, _ = O.nearest_descriptor(tgt, src)
    q, m = O.correspondences(src, tgt)
    ref = [c for c in range(len(src)) if s2t[c] >= 0 and t2s[s2t[c]] == c]
    assert list(q) == ref and np.array_equal(m, s2t[q])
