"""GPU parity: the reference's Harris3D keypoints (Keypoints::compute HARRIS_3D branch,
keypoints.h:150-162, with getKeypointsCloud keypoints.h:365-395) through the C-ABI against the CPU
restatement (oracle/or_keypoints.cpp orc_harris3d; parity vs real PCL unpinned: PCL adds over an
unsorted kd-tree's traversal order, the restatement over FLANN's sorted order).

Bar: bit-exact -- per-point response (float bits), the refined corners (float bits) and the
snapped keypoint indices.  Covers the reference's four clouds, NaN points and duplicates, corner
refinement on and off, thresholds, a dense blob whose refinement ball exceeds the wave sort
(ordered walk), and rejected parameters / capacity."""
import os

import numpy as np
import pytest

import oracle_lib as O
from pcl_feature_extraction_amd import PfxError, pcd

pytestmark = pytest.mark.gpu

CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


def _bits(a):
    return np.nan_to_num(np.asarray(a, np.float32), nan=-7.0).view(np.uint32)


def _check(ctx, x, y, z, threshold=1e-6, refine=True, radius=0.01):
    kp_o, resp_o, cor_o = O.harris3d(x, y, z, radius, threshold, refine)
    kp_g, resp_g, cor_g = ctx.harris3d_keypoints(x, y, z, radius, threshold, refine, details=True)
    assert np.array_equal(_bits(resp_g), _bits(resp_o)), np.nonzero(_bits(resp_g) != _bits(resp_o))[0][:10]
    assert cor_g.shape == cor_o.shape
    assert np.array_equal(_bits(cor_g), _bits(cor_o)), np.nonzero((_bits(cor_g) != _bits(cor_o)).any(1))[0][:10]
    assert np.array_equal(kp_g, kp_o)
    return len(kp_o), len(cor_o)


@pytest.mark.parametrize("name", ["indoor_source", "indoor_target", "underwater_source", "underwater_target"])
def test_reference_clouds(ctx, name):
    c = pcd.read_pcd(os.path.join(CLOUDS, name + ".pcd"))
    k, nc = _check(ctx, c.x, c.y, c.z)
    assert k > 0 and nc >= k


def _corner_scene(n, seed):
    # three planes meeting at a corner + a bumpy floor: real Harris corners
    rng = np.random.default_rng(seed)
    m = n // 4
    pts = []
    for axis in range(3):
        p = rng.random((m, 3)).astype(np.float32) * 0.3
        p[:, axis] = 0.0
        pts.append(p)
    u, v = rng.random((2, n - 3 * m)).astype(np.float32) * 0.6
    w = (0.01 * np.sin(40 * u) * np.cos(30 * v)).astype(np.float32) - 0.05
    pts.append(np.stack([u, v, w], 1))
    P = np.concatenate(pts).astype(np.float32)
    P += rng.normal(0, 1e-4, P.shape).astype(np.float32)
    return P[:, 0].copy(), P[:, 1].copy(), P[:, 2].copy()


def test_scene_with_nan_and_duplicates(ctx):
    x, y, z = _corner_scene(40000, 1)
    x[::89] = np.nan
    x[500:700], y[500:700], z[500:700] = x[900:1100], y[900:1100], z[900:1100]
    k, nc = _check(ctx, x, y, z)
    assert k > 0


@pytest.mark.parametrize("refine,threshold", [(False, 1e-6), (True, 1e-4), (True, 0.0)])
def test_parameters(ctx, refine, threshold):
    x, y, z = _corner_scene(20000, 2)
    _check(ctx, x, y, z, threshold=threshold, refine=refine)


def test_dense_blob_walks_the_ball_in_order(ctx):
    x, y, z = _corner_scene(20000, 3)
    rng = np.random.default_rng(4)
    b = (rng.random((3, 2000)) * 4e-3 + 0.1).astype(np.float32)  # 2000 points within 4 mm
    _check(ctx, np.concatenate([x, b[0]]), np.concatenate([y, b[1]]), np.concatenate([z, b[2]]))


def test_rejected_parameters_and_capacity(ctx):
    import torch
    x, y, z = _corner_scene(8000, 5)
    with pytest.raises(PfxError) as e:
        ctx.harris3d_keypoints(x, y, z, radius=0.0)
    assert e.value.code == 1
    with pytest.raises(PfxError) as e:
        ctx.harris3d_keypoints(x, y, z, non_max=False)
    assert e.value.code == 4
    dx, dy, dz = (torch.from_numpy(a).cuda() for a in (x, y, z))
    small = torch.empty(1, dtype=torch.int32, device="cuda")
    with pytest.raises(PfxError) as e:
        ctx.harris3d_keypoints_dev(dx, dy, dz, small)
    assert e.value.code == 3
    idx = torch.empty(len(x), dtype=torch.int32, device="cuda")
    k, nc = ctx.harris3d_keypoints_dev(dx, dy, dz, idx)
    kp_o, _, _ = O.harris3d(x, y, z)
    assert np.array_equal(idx[:k].cpu().numpy(), kp_o)
