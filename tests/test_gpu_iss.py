"""GPU parity: the reference's ISS keypoints (Keypoints::compute ISS branch, keypoints.h:177-189)
and Keypoints::computeCloudResolution (keypoints.h:401-428) through the C-ABI against the CPU
restatement (oracle/or_keypoints.cpp; parity vs real PCL unpinned).

Bar: bit-exact -- the resolution (double), the per-point third-eigenvalue map (double bits)
and the keypoint index list.  Covers the reference's four clouds, synthetic surfaces, NaN
points, exact duplicates, isolated outliers (the exhaustive fallback of the 2nd-NN search),
clouds so sparse the first grid certifies nothing (grid doubling), tiny clouds, a resolution
sum that is not exactly representable (sequential fallback), host and device entry points,
capacity and rejected parameters."""
import os

import numpy as np
import pytest

import oracle_lib as O
from pcl_feature_extraction_amd import PfxError, pcd

pytestmark = pytest.mark.gpu

CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


def _dev(*arrs):
    import torch
    return [torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in arrs]


def _iss_gpu(ctx, x, y, z, sal, nm):
    import torch
    dx, dy, dz = _dev(x, y, z)
    idx = torch.empty(max(len(x), 1), dtype=torch.int32, device="cuda")
    third = torch.empty(max(len(x), 1), dtype=torch.float64, device="cuda")
    k = ctx.iss_keypoints_dev(dx, dy, dz, sal, nm, idx, third=third)
    torch.cuda.synchronize()
    return idx[:k].cpu().numpy(), third[: len(x)].cpu().numpy()


def _check_cloud(ctx, x, y, z):
    res_o, _ = O.cloud_resolution(x, y, z)
    dx, dy, dz = _dev(x, y, z)
    res_g = ctx.cloud_resolution_dev(dx, dy, dz)
    assert res_g == res_o, (res_g, res_o)
    assert ctx.cloud_resolution(x, y, z) == res_o
    if res_o <= 0:
        return 0
    kp_o, th_o = O.iss_keypoints(x, y, z, 6 * res_o, 4 * res_o)
    kp_g, th_g = _iss_gpu(ctx, x, y, z, 6 * res_g, 4 * res_g)
    assert np.array_equal(th_g.view(np.uint64), th_o.view(np.uint64)), np.nonzero(th_g != th_o)[0][:10]
    assert np.array_equal(kp_g, kp_o)
    return len(kp_o)


@pytest.mark.parametrize("name", ["indoor_source", "indoor_target", "underwater_source", "underwater_target"])
def test_reference_clouds(ctx, name):
    c = pcd.read_pcd(os.path.join(CLOUDS, name + ".pcd"))
    assert _check_cloud(ctx, c.x, c.y, c.z) > 0


def _surface(n, seed):
    rng = np.random.default_rng(seed)
    u, v = rng.random((2, n)).astype(np.float32) * 2
    w = (0.2 * np.sin(3 * u) * np.cos(2 * v) + 0.002 * rng.normal(size=n)).astype(np.float32)
    return u, v, w


def test_surface_with_nan_and_duplicates(ctx):
    x, y, z = _surface(60000, 1)
    x[::97] = np.nan
    z[5::101] = np.inf
    x[1000:1300], y[1000:1300], z[1000:1300] = x[2000:2300], y[2000:2300], z[2000:2300]
    assert _check_cloud(ctx, x, y, z) > 0
    # points within ~1 cm of the x = 0 / y = 0 planes take the FLANN-ordered list path
    assert 0 < ctx.stat("iss_ordered") < len(x) // 4


def test_outliers_take_the_exhaustive_path(ctx):
    x, y, z = _surface(30000, 2)
    x[:40] = np.float32(100.0) + np.arange(40, dtype=np.float32) * np.float32(3.0)  # isolated
    _check_cloud(ctx, x, y, z)
    assert ctx.stat("resolution_brute") >= 40


def test_sparse_cloud_doubles_the_grid(ctx):
    # a thin dense strip inside a large volume: the first cell (from the bounding volume) is
    # far below the spacing of the sparse part, so most points need the larger grids
    rng = np.random.default_rng(3)
    n = 20000
    x = rng.random(n).astype(np.float32) * 50
    y = rng.random(n).astype(np.float32) * 50
    z = rng.random(n).astype(np.float32) * 50
    x[:5000] = rng.random(5000).astype(np.float32) * 0.1
    y[:5000] = rng.random(5000).astype(np.float32) * 0.1
    z[:5000] = 0.0
    _check_cloud(ctx, x, y, z)
    assert ctx.stat("resolution_rounds") > 1


def test_sequential_sum_fallback(ctx):
    # two points 1e-12 apart: the smallest term's ulp (2^-63) is so far below the total that
    # the integer sum would need more than 53 bits, so PCL's loop runs as is
    x, y, z = _surface(8000, 4)
    x[0] = y[0] = z[0] = 0.0
    x[1], y[1], z[1] = np.float32(1e-12), 0.0, 0.0
    res_o, _ = O.cloud_resolution(x, y, z)
    dx, dy, dz = _dev(x, y, z)
    assert ctx.cloud_resolution_dev(dx, dy, dz) == res_o
    assert ctx.stat("resolution_exact_sum") == 0


@pytest.mark.parametrize("n", [0, 1, 2, 5, 37])
def test_tiny_clouds(ctx, n):
    rng = np.random.default_rng(n)
    x, y, z = rng.random((3, n)).astype(np.float32)
    res_o, _ = O.cloud_resolution(x, y, z)
    assert ctx.cloud_resolution(x, y, z) == res_o
    if n:
        kp_o, th_o = O.iss_keypoints(x, y, z, 0.3, 0.2, min_neighbors=2)
        kp_g, th = ctx.iss_keypoints(x, y, z, 0.3, 0.2, min_neighbors=2, return_third=True)
        assert np.array_equal(kp_g, kp_o) and np.array_equal(th, th_o)


def test_host_entry_and_parameters(ctx):
    x, y, z = _surface(5000, 5)
    res = ctx.cloud_resolution(x, y, z)
    for (mn, t21, t32) in [(5, 0.975, 0.975), (12, 0.9, 0.8), (1, 0.99, 0.5)]:
        kp_o, th_o = O.iss_keypoints(x, y, z, 6 * res, 4 * res, mn, t21, t32)
        kp_g, th_g = ctx.iss_keypoints(x, y, z, 6 * res, 4 * res, mn, t21, t32, return_third=True)
        assert np.array_equal(kp_g, kp_o) and np.array_equal(th_g, th_o)


def test_rejected_parameters_and_capacity(ctx):
    import torch
    x, y, z = _surface(3000, 6)
    for bad in [(0.0, 0.1, 5, 0.975, 0.975), (0.1, -1.0, 5, 0.975, 0.975), (0.1, 0.1, 0, 0.975, 0.975),
                (0.1, 0.1, 5, 0.0, 0.975)]:
        with pytest.raises(PfxError) as e:
            ctx.iss_keypoints(x, y, z, bad[0], bad[1], bad[2], bad[3], bad[4])
        assert e.value.code == 1
    res = ctx.cloud_resolution(x, y, z)
    kp = ctx.iss_keypoints(x, y, z, 6 * res, 4 * res)
    assert len(kp) > 1
    dx, dy, dz = _dev(x, y, z)
    small = torch.empty(1, dtype=torch.int32, device="cuda")
    with pytest.raises(PfxError) as e:
        ctx.iss_keypoints_dev(dx, dy, dz, 6 * res, 4 * res, small)
    assert e.value.code == 3


def test_dense_cluster_at_origin_takes_the_list_path(ctx):
    # a 1 mm blob of 1500 points at the origin inside a sparse surface: its points need PCL's
    # order (coordinates near 0) and have more neighbours than the wave sort holds
    x, y, z = _surface(20000, 7)
    rng = np.random.default_rng(8)
    b = (rng.random((3, 1500)) * 1e-3).astype(np.float32)
    x = np.concatenate([x, b[0]])
    y = np.concatenate([y, b[1]])
    z = np.concatenate([z, b[2]])
    _check_cloud(ctx, x, y, z)
    assert ctx.stat("iss_ordered_lists") > 0
