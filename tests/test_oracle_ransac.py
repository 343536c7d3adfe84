"""CPU checks of the RANSAC rejection restatement (oracle/or_ransac.cpp, SURVEY 8(f) F2;
features.h:282-297).  Parity vs real PCL is unpinned (no PCL here); these pin the restatement's
behaviour: a known rigid motion with 30 % wrong correspondences is recovered to the noise level,
every kept correspondence is a true one, RANSAC stops after few models (adaptive k), the kept
set is exactly the pairs within the inlier threshold of the returned transformation, and the
degenerate cases return the input and the identity as PCL does."""
import numpy as np

import oracle_lib as O


def _scene(n, out_frac, seed, noise=0.002):
    rng = np.random.default_rng(seed)
    src = (rng.random((n, 3)) * 2).astype(np.float32)
    th = 0.4
    R = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1.0]])
    t = np.array([0.3, -0.1, 0.2])
    tgt = (src @ R.T + t + rng.normal(0, noise, (n, 3))).astype(np.float32)
    q = np.arange(n, dtype=np.int32)
    m = q.copy()
    bad = rng.choice(n, int(out_frac * n), replace=False)
    m[bad] = rng.permutation(m[bad])
    return src, tgt, q, m, R, t


def test_recovers_rigid_motion():
    src, tgt, q, m, R, t = _scene(400, 0.3, 1)
    keep, T, it = O.ransac_rejector(src, tgt, q, m)
    assert np.abs(T[:3, :3] - R).max() < 0.02 and np.abs(T[:3, 3] - t).max() < 0.02
    assert np.all(m[keep] == q[keep])  # only true correspondences survive
    assert len(keep) > 0.6 * 400 and 1 <= it < 100
    # the kept set is exactly the pairs within the threshold of the returned model
    p = src[q] @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
    d2 = ((p - tgt[m]) ** 2).sum(1)
    inside = np.nonzero(d2 < 0.015 ** 2 * 0.999)[0]
    assert set(inside) <= set(keep)


def test_degenerate_inputs_return_the_input():
    src, tgt, q, m, _, _ = _scene(2, 0.0, 2)
    keep, T, it = O.ransac_rejector(src, tgt, q, m)
    assert np.array_equal(keep, [0, 1]) and np.array_equal(T, np.eye(4, dtype=np.float32)) and it == 0
    # targets unrelated to the sources (no rigid motion explains 3 pairs within 1.5 cm beyond
    # the sample): fewer than 3 inliers -> input unchanged, identity
    src, _, q, m, _, _ = _scene(60, 0.0, 3)
    tgt = (np.random.default_rng(9).random((60, 3)) * 50).astype(np.float32)
    keep, T, _ = O.ransac_rejector(src, tgt, q, m)
    assert len(keep) == 60 and np.array_equal(T, np.eye(4, dtype=np.float32))


def test_identical_points_cannot_be_sampled():
    # all source keypoints at one place: no sample passes isSampleGood -> no model
    src = np.zeros((10, 3), np.float32)
    tgt = np.zeros((10, 3), np.float32)
    q = np.arange(10, dtype=np.int32)
    keep, T, it = O.ransac_rejector(src, tgt, q, q)
    assert len(keep) == 10 and it == 0
