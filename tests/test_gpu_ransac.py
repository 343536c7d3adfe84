"""GPU parity: the reference's RANSAC correspondence rejection (Features<T>::filterCorrespondences,
features.h:282-297 -> CorrespondenceRejectorSampleConsensus, threshold 0.015, 1000 iterations)
through the C-ABI against the CPU restatement (oracle/or_ransac.cpp; parity vs PCL unpinned).

Bar: exact -- the same kept correspondences (positions, input order), the same transformation
(float bits) and the same number of models evaluated.  Covers synthetic rigid motions with
0-60 % wrong correspondences, thresholds and iteration caps, the degenerate cases, and the
reference's own flow on its indoor clouds: ISS keypoints -> FPFH -> findCorrespondences ->
filterCorrespondences."""
import os

import numpy as np
import pytest

import oracle_lib as O
from pcl_feature_extraction_amd import PfxError, pcd

pytestmark = pytest.mark.gpu

CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


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
    return src, tgt, q, m


def _check(ctx, src, tgt, q, m, threshold=0.015, max_iterations=1000):
    keep_o, T_o, it_o = O.ransac_rejector(src, tgt, q, m, threshold, max_iterations)
    keep_g, T_g = ctx.ransac_rejector(src, tgt, q, m, threshold, max_iterations)
    assert np.array_equal(keep_g, keep_o)
    assert np.array_equal(T_g.view(np.uint32), T_o.view(np.uint32))
    assert ctx.stat("ransac_iterations") == it_o
    return keep_o, it_o


@pytest.mark.parametrize("n,out_frac,seed", [(50, 0.0, 1), (400, 0.3, 2), (2000, 0.6, 3), (5000, 0.45, 4)])
def test_synthetic(ctx, n, out_frac, seed):
    src, tgt, q, m = _scene(n, out_frac, seed)
    keep, it = _check(ctx, src, tgt, q, m)
    assert len(keep) >= 3 and it >= 1


@pytest.mark.parametrize("threshold,max_iterations", [(0.005, 1000), (0.05, 10), (0.015, 0)])
def test_parameters(ctx, threshold, max_iterations):
    src, tgt, q, m = _scene(800, 0.5, 5)
    _check(ctx, src, tgt, q, m, threshold, max_iterations)


def test_degenerate(ctx):
    src, tgt, q, m = _scene(2, 0.0, 6)
    _check(ctx, src, tgt, q, m)
    src, _, q, m = _scene(60, 0.0, 7)
    tgt = (np.random.default_rng(9).random((60, 3)) * 50).astype(np.float32)
    _check(ctx, src, tgt, q, m)
    z = np.zeros((10, 3), np.float32)
    _check(ctx, z, z, np.arange(10, dtype=np.int32), np.arange(10, dtype=np.int32))
    with pytest.raises(PfxError) as e:
        ctx.ransac_rejector(src, tgt, q, m, threshold=0.0)
    assert e.value.code == 1


def test_reference_flow_indoor(ctx):
    """evaluation.cpp's sequence on the reference's indoor pair with its active keypoint
    detector: ISS keypoints (keypoints.h:177-189), normals + FPFH, findCorrespondences, then
    filterCorrespondences (the GPU path end to end)."""
    clouds = [pcd.read_pcd(os.path.join(CLOUDS, f"indoor_{s}.pcd")) for s in ("source", "target")]
    kps, descs = [], []
    for c in clouds:
        res = ctx.cloud_resolution(c.x, c.y, c.z)
        kp = np.asarray(ctx.iss_keypoints(c.x, c.y, c.z, 6 * res, 4 * res), np.int64)
        nx, ny, nz, _ = ctx.normals(c.x, c.y, c.z, 0.05)
        d = ctx.fpfh(c.x, c.y, c.z, nx, ny, nz, c.x[kp], c.y[kp], c.z[kp], 0.08)
        kps.append(np.stack([c.x[kp], c.y[kp], c.z[kp]], 1))
        descs.append(d)
    q, m = ctx.correspondences(descs[0], descs[1])
    assert len(q) >= 3
    _check(ctx, kps[0], kps[1], q, m)
