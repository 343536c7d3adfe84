"""GPU parity: radius search, NormalEstimationOMP and FPFHEstimation through the C-ABI, against the
CPU restatement (oracle/, parity vs real PCL unpinned -- see oracle/or_common.h).

Bar (SURVEY section 0 / BASELINE.json north star):
  * radius-search counts, indices and squared distances: bit-exact (integer/index work);
  * normals + curvature: bit-exact (float32, same operation order as PCL's single-pass
    covariance, eigen33 and viewpoint flip -- NaN where PCL yields NaN);
  * FPFH-33: bit-exact here as well (the stated tolerance 1e-4 L2 is the ceiling, asserted too).
"""
import numpy as np
import pytest

import oracle_lib as O
from pcl_feature_extraction_amd.pcd import read_pcd

pytestmark = pytest.mark.gpu

CLOUDS = ["indoor_source", "underwater_source", "indoor_target", "underwater_target"]


def _cloud(name):
    import os
    c = read_pcd(os.path.join(os.path.dirname(__file__), "golden", "clouds", name + ".pcd"))
    return c.x, c.y, c.z


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _nan_aware_equal(a, b):
    # raw bits, NaN rows included: the product writes PCL's quiet_NaN (0x7FC00000) as the oracle does
    a = np.ascontiguousarray(np.asarray(a, np.float32))
    b = np.ascontiguousarray(np.asarray(b, np.float32))
    return a.shape == b.shape and _bits_equal(a, b)


@pytest.mark.parametrize("r", [0.05, 0.08])
def test_radius_search_exact(ctx, r):
    x, y, z = _cloud("indoor_source")
    rng = np.random.default_rng(7)
    q = rng.choice(len(x), 512, replace=False)
    cap = 2048
    c_gpu, i_gpu, d_gpu = ctx.radius_search(x, y, z, x[q], y[q], z[q], r, cap=cap)
    c_ref, i_ref, d_ref = O.radius_search(x, y, z, x[q], y[q], z[q], r, cap=cap)
    assert np.array_equal(c_gpu, c_ref)
    for j in range(len(q)):
        k = min(c_ref[j], cap)
        assert np.array_equal(i_gpu[j, :k], i_ref[j, :k]), j
        assert _bits_equal(d_gpu[j, :k], d_ref[j, :k]), j


def test_radius_search_counts_off_cloud_queries(ctx):
    x, y, z = _cloud("underwater_source")
    rng = np.random.default_rng(3)
    qx = rng.uniform(x.min() - 0.2, x.max() + 0.2, 2000).astype(np.float32)
    qy = rng.uniform(y.min() - 0.2, y.max() + 0.2, 2000).astype(np.float32)
    qz = rng.uniform(z.min() - 0.2, z.max() + 0.2, 2000).astype(np.float32)
    c_gpu, _, _ = ctx.radius_search(x, y, z, qx, qy, qz, 0.05)
    c_ref, _, _ = O.radius_search(x, y, z, qx, qy, qz, 0.05)
    assert np.array_equal(c_gpu, c_ref)


@pytest.mark.parametrize("name", CLOUDS)
def test_normals_bit_exact_full_cloud(ctx, name):
    x, y, z = _cloud(name)
    g = ctx.normals(x, y, z, 0.05)
    o = O.normals(x, y, z, 0.05)
    for a, b in zip(g, o):
        assert _nan_aware_equal(a, b)


def test_normals_edge_cases(ctx):
    rng = np.random.default_rng(11)
    # isolated points (< 3 neighbours -> NaN), exact duplicates, a plane, points on r
    iso = np.array([[10, 10, 10], [20, 20, 20], [20.01, 20, 20]], np.float32)
    dup = np.repeat(rng.uniform(0, 1, (50, 3)).astype(np.float32), 3, axis=0)
    plane = np.c_[rng.uniform(0, 1, (3000, 2)), np.full(3000, 2.0)].astype(np.float32)
    grid = np.stack(np.meshgrid(np.arange(10), np.arange(10), [0]), -1).reshape(-1, 3).astype(np.float32) * 0.05
    grid[:, 2] += 5.0
    pts = np.concatenate([iso, dup, plane, grid])
    x, y, z = pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()
    for vp in [(0, 0, 0), (0.5, 0.5, 10.0)]:
        g = ctx.normals(x, y, z, 0.05, viewpoint=vp)
        o = O.normals(x, y, z, 0.05, vp=vp)
        for a, b in zip(g, o):
            assert _nan_aware_equal(a, b)
    assert np.isnan(g[0][:3]).all()


def test_normals_every_list_path(ctx):
    """Densities that route queries through every neighbour-list path (pfx_nblist.hip): sparse
    and dense tiles, the lists that overflow a tile (k > 512 / 1024: the per-query kernel's test
    and sort), wide tiles (blocks of > 8000 candidates: lists written unsorted, then sorted in place
    by the per-query tiers, k <= 4096, <= 8192, <= 16384 in LDS, beyond in global scratch), plus
    lane-per-query and nine-lanes-per-query chains; duplicates exercise the index tie-break."""
    rng = np.random.default_rng(23)
    sparse = np.c_[rng.uniform(0, 1, (4000, 2)), np.full(4000, 1.0)]
    dense = np.c_[rng.uniform(2, 2.3, (9000, 2)), np.full(9000, 1.0)]          # k ~ 400..800
    denser = np.c_[rng.uniform(3, 3.1, (9000, 2)), np.full(9000, 1.0)]         # k ~ 1800..7000
    blob = rng.normal(0, 0.01, (1500, 3)) + [4, 4, 1]                          # k ~ 900..1500
    mid = np.repeat(rng.normal(0, 0.004, (1700, 3)) + [6, 6, 1], 3, axis=0)   # k = 5100, ties
    mid16 = np.repeat(rng.normal(0, 0.004, (3500, 3)) + [7, 7, 1], 3, axis=0)  # k = 10500 (8k-16k)
    huge = np.repeat(rng.normal(0, 0.004, (5500, 3)) + [8, 8, 1], 3, axis=0)  # k = 16500 > 16384
    pts = np.concatenate([sparse, dense, denser, blob, mid, mid16, huge]).astype(np.float32)
    x, y, z = pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()
    g = ctx.normals(x, y, z, 0.05)
    for nm in ["normals_tiles_sparse", "normals_tiles_dense", "normals_wide", "normals_single", "normals_mid8",
               "normals_mid", "normals_huge"]:
        assert ctx.stat(nm) > 0, nm
    o = O.normals(x, y, z, 0.05)
    for a, b in zip(g, o):
        assert _nan_aware_equal(a, b)


def _every_list_cloud():
    rng = np.random.default_rng(23)
    sparse = np.c_[rng.uniform(0, 1, (4000, 2)), np.full(4000, 1.0)]
    dense = np.c_[rng.uniform(2, 2.3, (9000, 2)), np.full(9000, 1.0)]
    mid8 = np.repeat(rng.normal(0, 0.004, (1700, 3)) + [6, 6, 1], 3, axis=0)   # k = 5100 (4k-8k tier)
    mid = np.repeat(rng.normal(0, 0.004, (3500, 3)) + [7, 7, 1], 3, axis=0)    # k = 10500 (8k-16k tier)
    huge = np.repeat(rng.normal(0, 0.004, (5500, 3)) + [8, 8, 1], 3, axis=0)   # k = 16500 (global scratch)
    return sparse, dense, mid8, mid, huge


def _xyz(*parts):
    pts = np.concatenate(parts).astype(np.float32)
    return pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()


def _wide_blob(rng):
    """A uniform 0.15 m cube of 13k points: every tile inside has a 3x3x3 block of > 8000
    candidates (a wide tile, k_nb_wide) while each list stays at <= ~2.5k entries (<= 4096: the
    always-launched per-query tier), so it keeps the wide-tile hint alive and no 4k-16k hint."""
    return rng.uniform(0, 0.15, (13000, 3)) + [10, 10, 1]


def test_list_tier_hints_every_path_fresh_context():
    """The 4k-8k / 8k-16k per-query list tiers and the wide-tile kernel launch only while a recent
    build of the (context, tag) had work for them (pfx_nblist.hip mid_tier_wanted).  On a fresh
    context, once hints have decayed (17 builds without such lists), a cloud that needs the skipped
    kernels must still come out exact on every path:
      * the 8k-16k tier skipped while the wide tiles and the 4k-8k tier run: the non-deferred
        catch-up proper (`_tier_catchups`) -- the lists over 8k come from wide tiles, which push
        them straight to their tier, and the huge tier, which already ran on an empty queue, is
        relaunched from the count it drained (the lists the catch-up appends were
        never fetched);
      * the wide tiles skipped too: the whole build reruns with every kernel (`_wide_reruns`);
      * the deferred check's exact rebuild."""
    import torch
    from pcl_feature_extraction_amd import Context
    sparse, dense, mid8, mid, huge = _every_list_cloud()
    wide = _wide_blob(np.random.default_rng(29))
    ex, ey, ez = _xyz(sparse, dense, mid8, mid, huge)
    ref = O.normals(ex, ey, ez, 0.05)
    dev = torch.device("cuda", 0)

    def dev_arrays(x, y, z):
        t = [torch.from_numpy(a).to(dev) for a in (x, y, z)]
        o = [torch.empty(len(x), dtype=torch.float32, device=dev) for _ in range(4)]
        torch.cuda.synchronize()  # (the context runs on its own stream)
        return t, o

    with Context(0) as c:
        def lists_only(x, y, z):  # a non-deferred build of tag "normals" (pfx_normals_lists_dev)
            (tx, ty, tz), o = dev_arrays(x, y, z)
            c.normals_lists_dev(tx, ty, tz, 0.05, *o)
            c.synchronize()

        def every_two_phase():
            (tx, ty, tz), o = dev_arrays(ex, ey, ez)
            c.normals_lists_dev(tx, ty, tz, 0.05, *o)
            c.normals_chains_dev(c, *o)
            c.synchronize()
            for a, b in zip(o, ref):
                assert _nan_aware_equal(a.cpu().numpy(), b)

        def stat(name):
            try:
                return c.stat("normals_" + name)
            except Exception:
                return 0

        every_two_phase()                          # first build: every tier, scratch allocated
        assert c.stat("normals_huge") > 0 and c.stat("normals_mid") > 0 and c.stat("normals_mid8") > 0
        assert c.stat("normals_wide") > 0
        wx, wy, wz = _xyz(sparse, mid8, wide)
        lists_only(wx, wy, wz)
        assert stat("wide") > 0 and stat("mid") == 0  # the warm-up cloud: wide tiles, no 8k-16k list
        for _ in range(17):
            lists_only(wx, wy, wz)                 # the 8k-16k hint decays, the 4k-8k and wide ones stay
        assert stat("ran_mid_tiers") & 4 and not stat("ran_mid_tiers") & 2
        cat, wre = stat("tier_catchups"), stat("wide_reruns")
        every_two_phase()                          # 8k-16k skipped: the catch-up of it, then huge again
        assert stat("tier_catchups") == cat + 1 and stat("wide_reruns") == wre
        px, py, pz = _xyz(sparse)
        for _ in range(17):
            lists_only(px, py, pz)                 # every hint decays
        cat, wre = stat("tier_catchups"), stat("wide_reruns")
        every_two_phase()                          # wide tiles skipped: the build reruns with everything
        assert stat("wide_reruns") == wre + 1
        for _ in range(17):
            lists_only(px, py, pz)
        g = c.normals(ex, ey, ez, 0.05)            # deferred build (normals_dev): check + exact rebuild
        for a, b in zip(g, ref):
            assert _nan_aware_equal(a, b)


def test_normals_speculative_grid_and_list_check():
    """normals_dev builds the grid on the previous call's widened bounds and validates grid and
    lists in one readback (pfx_normals.hip normals_dev): a scan outside the hint, a list buffer
    too small and the first very long lists each rerun the exact path, bit-exact either way."""
    from pcl_feature_extraction_amd import Context
    x, y, z = _cloud("underwater_source")
    rng = np.random.default_rng(5)
    blob = np.repeat(rng.normal(0, 0.004, (5500, 3)) + [x.mean(), y.mean(), z.mean()], 3, axis=0)  # k > 16384
    with Context(0) as c:
        def reruns():
            try:
                return c.stat("normals_speculative_reruns")
            except Exception:  # (no normal estimation on this context yet)
                return 0

        def run(px, py, pz):
            before = reruns()
            g = c.normals(px, py, pz, 0.05)
            o = O.normals(px, py, pz, 0.05)
            for a, b in zip(g, o):
                assert _nan_aware_equal(a, b)
            return reruns() - before
        assert run(x, y, z) in (0, 1)     # first call: exact bounds (a fresh list buffer may be short)
        assert run(x, y, z) == 0          # inside the hint
        sx = (x + 5.0).astype(np.float32)
        assert run(sx, y, z) == 1         # outside the hint: rerun on exact bounds
        assert run(sx, y, z) == 0
        bx, by, bz = (np.concatenate([a, b]).astype(np.float32) for a, b in zip((sx, y, z), blob.T + [[5.0], [0], [0]]))
        assert run(bx, by, bz) == 1       # first very long lists (scratch allocated by the rerun)
        assert run(bx, by, bz) == 0


def test_normals_empty_and_tiny(ctx):
    e = np.zeros(0, np.float32)
    g = ctx.normals(e, e, e, 0.05)
    assert all(len(a) == 0 for a in g)
    one = np.array([1.0], np.float32)
    g = ctx.normals(one, one, one, 0.05)
    assert np.isnan(g[0]).all()


@pytest.mark.parametrize("name", ["indoor_source", "underwater_target"])
def test_fpfh_keypoints_union_path(ctx, name):
    """Features<FPFHSignature33>::compute with keypoints != surface (features.h:175-196)."""
    x, y, z = _cloud(name)
    nx, ny, nz, _ = O.normals(x, y, z, 0.05)
    rng = np.random.default_rng(5)
    q = np.sort(rng.choice(len(x), 300, replace=False))
    g = ctx.fpfh(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08)
    o = O.fpfh(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08)
    assert _nan_aware_equal(g, o)
    l2 = np.sqrt(np.nansum((g.astype(np.float64) - o) ** 2, axis=1))
    assert l2.max() <= 1e-4


def test_fpfh_same_as_surface(ctx):
    """PCL's input == surface branch (config 2 shape), on a 20k-point crop of indoor."""
    x, y, z = _cloud("indoor_source")
    sel = np.arange(0, len(x), 5)
    x, y, z = x[sel].copy(), y[sel].copy(), z[sel].copy()
    nx, ny, nz, _ = ctx.normals(x, y, z, 0.05)
    g = ctx.fpfh(x, y, z, nx, ny, nz, None, None, None, 0.05, same_as_surface=True)
    o = O.fpfh(x, y, z, nx, ny, nz, x, y, z, 0.05, same_as_surface=True)
    assert _nan_aware_equal(g, o)


def test_fpfh_isolated_query_is_nan(ctx):
    x, y, z = _cloud("underwater_source")
    nx, ny, nz, _ = O.normals(x, y, z, 0.05)
    qx = np.array([x[0], 100.0], np.float32)
    qy = np.array([y[0], 100.0], np.float32)
    qz = np.array([z[0], 100.0], np.float32)
    g = ctx.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.08)
    o = O.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.08)
    assert np.isnan(g[1]).all() and np.isnan(o[1]).all()
    assert _nan_aware_equal(g, o)


def test_config1_normals_fpfh_all_points():
    """BASELINE configs[1]: 100k-point synthetic room (seed 1), NormalEstimation + FPFH (r 0.05)
    at every point (input == surface: PCL's all-points SPFH branch)."""
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.synth import synth_room
    x, y, z, _ = synth_room(100_000, 1)
    with Context(0) as c:
        g = c.normals(x, y, z, 0.05)
        o = O.normals(x, y, z, 0.05, threads=8)
        for a, b in zip(g, o):
            assert _nan_aware_equal(a, b)
        d = c.fpfh(x, y, z, g[0], g[1], g[2], None, None, None, 0.05, same_as_surface=True)
    od = O.fpfh(x, y, z, o[0], o[1], o[2], x, y, z, 0.05, same_as_surface=True, threads=8)
    assert _nan_aware_equal(d, od)


def test_fpfh_deferred_pair_queue_overflow(ctx, monkeypatch):
    """Pairs the fast binning path cannot certify are queued for the exact path; past the
    queue's capacity the SPFH kernel runs the exact path in place -- same descriptors."""
    x, y, z = _cloud("indoor_source")
    nx, ny, nz, _ = O.normals(x, y, z, 0.05)
    rng = np.random.default_rng(6)
    q = np.sort(rng.choice(len(x), 400, replace=False))
    base = ctx.fpfh(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08)
    assert ctx.stat("fpfh_spfh_exact_pairs") > 4 and ctx.stat("fpfh_spfh_inline_exact") == 0
    monkeypatch.setenv("PFX_FPFH_SLOW_CAP", "4")
    g = ctx.fpfh(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08)
    assert ctx.stat("fpfh_spfh_exact_pairs") == 4 and ctx.stat("fpfh_spfh_inline_exact") > 0
    assert _nan_aware_equal(g, base)
    assert _nan_aware_equal(g, O.fpfh(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08))


def _shell(n, radius, seed, centre=(0.3, -0.2, 1.5)):
    """n points on a sphere shell of the given radius (float32 SoA) plus outward normals."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    p = (np.asarray(centre) + radius * v).astype(np.float32)
    return p[:, 0].copy(), p[:, 1].copy(), p[:, 2].copy(), v.astype(np.float32)


def test_radius_search_beyond_lds_capacity(ctx):
    """PCL's radiusSearch (max_nn = 0) returns every neighbour: lists longer than the LDS
    capacity (16,384) are ordered by the global-scratch pass, bit-exact like the rest."""
    rng = np.random.default_rng(11)
    n = 20_000
    c = np.array([0.1, 0.2, 1.0])
    p = (c + rng.uniform(-0.015, 0.015, (n, 3))).astype(np.float32)
    x, y, z = p[:, 0].copy(), p[:, 1].copy(), p[:, 2].copy()
    q = np.array([0, 17, 19_999])
    cap = n
    c_gpu, i_gpu, d_gpu = ctx.radius_search(x, y, z, x[q], y[q], z[q], 0.05, cap=cap)
    c_ref, i_ref, d_ref = O.radius_search(x, y, z, x[q], y[q], z[q], 0.05, cap=cap)
    assert (c_ref > 16384).all()
    assert np.array_equal(c_gpu, c_ref)
    for j in range(len(q)):
        k = c_ref[j]
        assert np.array_equal(i_gpu[j, :k], i_ref[j, :k]), j
        assert _bits_equal(d_gpu[j, :k], d_ref[j, :k]), j


def test_fpfh_weighting_beyond_lds_capacity(ctx):
    """A keypoint with more neighbours than the weighting kernel's LDS capacity (8,192) is
    weighted by the global-scratch pass: same descriptor bits as the restatement."""
    x, y, z, nv = _shell(17_000, 0.045, 5)
    nx, ny, nz = nv[:, 0].copy(), nv[:, 1].copy(), nv[:, 2].copy()
    qx = np.array([0.3, x[0]], np.float32)
    qy = np.array([-0.2, y[0]], np.float32)
    qz = np.array([1.5, z[0]], np.float32)
    g = ctx.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.05)
    assert ctx.stat("fpfh_weight_global") == 1
    o = O.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.05, threads=8)
    assert _nan_aware_equal(g, o)


def _disc(n, radius, seed, centre=(0.2, -0.1, 1.2)):
    """n points spread over a slightly rough disc (their distances to the centre spread evenly in
    d2, as a surface neighbourhood's) plus jittered upward normals."""
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0.0, 2.0 * np.pi, n)
    rad = radius * np.sqrt(rng.uniform(0.0, 1.0, n))
    p = np.stack([centre[0] + rad * np.cos(ang), centre[1] + rad * np.sin(ang),
                  centre[2] + 1e-3 * rng.standard_normal(n)], axis=1).astype(np.float32)
    v = np.stack([0.05 * rng.standard_normal(n), 0.05 * rng.standard_normal(n), np.ones(n)], axis=1)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = v.astype(np.float32)
    return p[:, 0].copy(), p[:, 1].copy(), p[:, 2].copy(), v[:, 0].copy(), v[:, 1].copy(), v[:, 2].copy()


def test_fpfh_weighting_global_pass_spread(ctx):
    """A keypoint whose neighbourhood outgrows the weighting kernel's LDS (8,192) with its
    distances spread evenly in d2, as a surface's (the shell test's centre has them all equal): a
    disc whose 20,000 points all neighbour its centre, weighted by the global-scratch pass, gives
    the restatement's descriptor bits."""
    x, y, z, nx, ny, nz = _disc(20_000, 0.04, 21)
    qx = np.array([0.2, x[5], 0.2 + 0.02], np.float32)
    qy = np.array([-0.1, y[5], -0.1], np.float32)
    qz = np.array([1.2, z[5], 1.2], np.float32)
    o = O.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.05, threads=8)
    g = ctx.fpfh(x, y, z, nx, ny, nz, qx, qy, qz, 0.05)
    assert ctx.stat("fpfh_weight_global") >= 1
    assert _nan_aware_equal(g, o)


def test_fpfh_same_as_surface_dev_reuses_normal_lists():
    """Device API, Features::compute's sequence (features.h:187-195): normals then FPFH
    (pfx_fpfh_after_normals_dev) on the same device cloud at the same radius reuse the normals'
    FLANN-ordered lists for the weighting; another radius builds its own.  Both bit-exact against
    the restatement."""
    import torch
    from pcl_feature_extraction_amd import Context
    x, y, z = _cloud("indoor_source")
    x, y, z = x[::3].copy(), y[::3].copy(), z[::3].copy()
    n = len(x)
    dev = torch.device("cuda", 0)
    dx, dy, dz = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    nx, ny, nz, cv = (torch.empty(n, device=dev) for _ in range(4))
    out = torch.empty((n, 33), device=dev)
    with Context(0) as c:
        c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        c.normals_dev(dx, dy, dz, 0.05, nx, ny, nz, cv)
        c.fpfh_dev(dx, dy, dz, nx, ny, nz, dx, dy, dz, 0.05, out, same_as_surface=True, after_normals=True)
        torch.cuda.synchronize(dev)
        assert c.stat("fpfh_weight_lists_reused") == 1
        g5 = out.cpu().numpy()
        c.fpfh_dev(dx, dy, dz, nx, ny, nz, dx, dy, dz, 0.06, out, same_as_surface=True, after_normals=True)
        torch.cuda.synchronize(dev)
        assert c.stat("fpfh_weight_lists_reused") == 0
        g6 = out.cpu().numpy()
    on = O.normals(x, y, z, 0.05)
    for a, b in zip((nx, ny, nz, cv), on):
        assert _nan_aware_equal(a.cpu().numpy(), b)
    assert _nan_aware_equal(g5, O.fpfh(x, y, z, on[0], on[1], on[2], x, y, z, 0.05, same_as_surface=True))
    assert _nan_aware_equal(g6, O.fpfh(x, y, z, on[0], on[1], on[2], x, y, z, 0.06, same_as_surface=True))


def test_fpfh_dev_does_not_reuse_lists_of_rewritten_buffers():
    """equal pointers do not prove equal contents.  Normals on scan A, then scan B
    written into the same device buffers, then pfx_fpfh_dev (same_as_surface) with B's normals:
    the result is B's descriptors (no stale lists), and a second after_normals call cannot
    reuse lists that were consumed."""
    import torch
    from pcl_feature_extraction_amd import Context
    xa, ya, za = (a[::3].copy() for a in _cloud("indoor_source"))
    xb, yb, zb = (a[::3].copy() for a in _cloud("indoor_target"))
    n = min(len(xa), len(xb))
    xa, ya, za, xb, yb, zb = (a[:n].copy() for a in (xa, ya, za, xb, yb, zb))
    dev = torch.device("cuda", 0)
    dx, dy, dz = (torch.from_numpy(a).to(dev) for a in (xa, ya, za))
    nx, ny, nz, cv = (torch.empty(n, device=dev) for _ in range(4))
    out = torch.empty((n, 33), device=dev)
    onb = O.normals(xb, yb, zb, 0.05)
    with Context(0) as c:
        c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        c.normals_dev(dx, dy, dz, 0.05, nx, ny, nz, cv)  # scan A's lists held by c
        for d, h in zip((dx, dy, dz), (xb, yb, zb)):
            d.copy_(torch.from_numpy(h).to(dev))           # scan B into the same buffers
        for d, h in zip((nx, ny, nz), onb[:3]):
            d.copy_(torch.from_numpy(h).to(dev))
        c.fpfh_dev(dx, dy, dz, nx, ny, nz, dx, dy, dz, 0.05, out, same_as_surface=True)
        torch.cuda.synchronize(dev)
        assert c.stat("fpfh_weight_lists_reused") == 0
        gb = out.cpu().numpy()
        c.normals_dev(dx, dy, dz, 0.05, nx, ny, nz, cv)
        c.fpfh_dev(dx, dy, dz, nx, ny, nz, dx, dy, dz, 0.05, out, same_as_surface=True, after_normals=True)
        c.fpfh_dev(dx, dy, dz, nx, ny, nz, dx, dy, dz, 0.05, out, same_as_surface=True, after_normals=True)
        torch.cuda.synchronize(dev)
        assert c.stat("fpfh_weight_lists_reused") == 0  # the first call consumed them
        gb2 = out.cpu().numpy()
    ref = O.fpfh(xb, yb, zb, onb[0], onb[1], onb[2], xb, yb, zb, 0.05, same_as_surface=True)
    assert _nan_aware_equal(gb, ref)
    assert _nan_aware_equal(gb2, ref)


def test_fpfh_speculative_surface_grid():
    """pfx_fpfh_prepare_dev builds FPFH's surface grid on the previous scan's widened bounds (no
    bounds readback); its first consumer validates the grid and rebuilds it exactly when a point
    lies outside.  Descriptors through the prepared path equal the host API's on a fresh context
    for a first scan (exact build), a scan inside the bounds (speculative grid kept) and a scan
    moved by 3 m (speculative grid rebuilt)."""
    import torch
    from pcl_feature_extraction_amd import Context
    x, y, z = _cloud("indoor_source")
    dev = torch.device("cuda", 0)
    scans = [(x, y, z), (x + 0.01, y, z), (x + 3.0, y, z)]
    q = np.arange(0, len(x), 97)
    with Context(0) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        for i, (sx, sy, sz) in enumerate(scans):
            sx, sy, sz = (np.ascontiguousarray(a, np.float32) for a in (sx, sy, sz))
            t = [torch.from_numpy(a).to(dev) for a in (sx, sy, sz)]
            nrm = [torch.empty_like(t[0]) for _ in range(4)]
            qs = [a[q].contiguous() for a in t]
            out = torch.empty((len(q), 33), dtype=torch.float32, device=dev)
            ctx.fpfh_prepare_dev(*t, 0.08)
            ctx.normals_dev(*t, 0.05, *nrm)
            ctx.fpfh_prepare_queries_dev(*t, *qs, 0.08)
            ctx.fpfh_dev(*t, *nrm[:3], *qs, 0.08, out)
            torch.cuda.synchronize(dev)
            got = out.cpu().numpy()
            with Context(0) as fresh:
                n_h = fresh.normals(sx, sy, sz, 0.05)
                ref = fresh.fpfh(sx, sy, sz, n_h[0], n_h[1], n_h[2], sx[q], sy[q], sz[q], 0.08)
            assert _nan_aware_equal(got, ref), i
            try:
                reruns = ctx.stat("fpfh_speculative_reruns")
            except Exception:  # (no rerun yet: the statistic does not exist)
                reruns = 0
            assert reruns == (1 if i == 2 else 0), (i, reruns)
