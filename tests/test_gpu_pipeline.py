"""The device-resident pass (pipeline.py) end to end: the overlapped two-stream schedule used by
bench.py equals the sequential narf_fpfh, and both equal the oracle on the same scan."""
import numpy as np
import pytest

import oracle_lib as O
from parity import bits_equal

pytestmark = pytest.mark.gpu


def test_overlapped_pass_matches_sequential_and_oracle():
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc, narf_fpfh
    from pcl_feature_extraction_amd.synth import synth_room
    n = 150_000
    x, y, z, _ = synth_room(n, 21)
    dev = torch.device("cuda", 0)
    outs = []
    for overlapped in (False, True):
        b = alloc(torch, n, dev, max_keypoints=4096)
        b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
        ctx, ctx_n = Context(0), Context(0)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        if overlapped:
            run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
            kp, k = run(b)
            run.close()
        else:
            kp, k = narf_fpfh(ctx, b)
        torch.cuda.synchronize(dev)
        outs.append((np.asarray(kp), k, np.stack([t.cpu().numpy() for t in (b.nx, b.ny, b.nz, b.curv)]),
                     b.desc[:k].cpu().numpy()))
        ctx.close(); ctx_n.close()
    (kp0, k0, n0, d0), (kp1, k1, n1, d1) = outs
    assert np.array_equal(kp0, kp1) and k0 == k1 and k0 > 0
    assert bits_equal(n0, n1)
    assert bits_equal(d0, d1)
    # against the CPU restatement
    okp = O.narf_keypoints(x, y, z)
    assert np.array_equal(kp1, okp)
    onx, ony, onz, oc = O.normals(x, y, z, 0.05)
    on = np.stack([onx, ony, onz, oc])
    assert bits_equal(n1, on)
    rows = okp[okp < n]
    od = O.fpfh(x, y, z, onx, ony, onz, x[rows], y[rows], z[rows], 0.08)
    assert bits_equal(d1, od)


def test_two_phase_normals_and_support_mask():
    """pfx_normals_lists_dev + two complementary pfx_normals_chains_dev passes on two contexts
    (two streams) == pfx_normals_dev; pfx_fpfh_support_mask_dev == the r-neighbours of the
    r-neighbourhoods of the queries (oracle radius search)."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.synth import synth_room
    n = 120_000
    x, y, z, _ = synth_room(n, 33)
    dev = torch.device("cuda", 0)
    X, Y, Z = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    ref = [torch.empty(n, device=dev) for _ in range(4)]
    out = [torch.empty(n, device=dev) for _ in range(4)]
    qi = np.arange(0, n, 997)
    Q = [t[torch.from_numpy(qi).to(dev)].contiguous() for t in (X, Y, Z)]
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    with Context(0) as a, Context(0) as b:
        a.normals_dev(X, Y, Z, 0.05, *ref)
        a.fpfh_support_mask_dev(X, Y, Z, *Q, 0.08, mask)
        b.normals_lists_dev(X, Y, Z, 0.05, *out)
        b.synchronize()
        a.normals_chains_dev(b, *out, mask=mask, want=1)
        b.normals_chains_dev(b, *out, mask=mask, want=0)
        a.synchronize(); b.synchronize()
    for r, o in zip(ref, out):
        r, o = r.cpu().numpy(), o.cpu().numpy()
        assert bits_equal(r, o)
    cnt, idx, _ = O.radius_search(x, y, z, x[qi], y[qi], z[qi], 0.08, cap=4096)
    assert cnt.max() <= 4096
    S = np.unique(idx[idx >= 0])
    cnt2, idx2, _ = O.radius_search(x, y, z, x[S], y[S], z[S], 0.08, cap=8192)
    assert cnt2.max() <= 8192
    expect = np.zeros(n, np.uint8)
    expect[np.unique(idx2[idx2 >= 0])] = 1
    assert np.array_equal(mask.cpu().numpy(), expect)


def test_support_ball_mask():
    """pfx_fpfh_support_ball_dev: exactly the points within 2r of a query (float squared distance
    in FLANN's order against (2r)^2 (1 + 1e-5)), a superset of the exact support mask."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.synth import synth_room
    n = 120_000
    x, y, z, _ = synth_room(n, 34)
    dev = torch.device("cuda", 0)
    X, Y, Z = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    qi = np.arange(0, n, 1499)
    Q = [t[torch.from_numpy(qi).to(dev)].contiguous() for t in (X, Y, Z)]
    ball = torch.empty(n, dtype=torch.uint8, device=dev)
    exact = torch.empty(n, dtype=torch.uint8, device=dev)
    r = 0.08
    with Context(0) as a:
        a.fpfh_support_ball_dev(X, Y, Z, *Q, r, ball)
        a.fpfh_support_mask_dev(X, Y, Z, *Q, r, exact)
        a.synchronize()
    ball, exact = ball.cpu().numpy(), exact.cpu().numpy()
    lim = np.float32(4.0 * r * r * (1.0 + 1e-5))
    expect = np.zeros(n, np.uint8)
    for q in qi:
        dx, dy, dz = x[q] - x, y[q] - y, z[q] - z
        d2 = ((np.float32(0) + dx * dx) + dy * dy) + dz * dz
        expect[d2 <= lim] = 1
    assert np.array_equal(ball, expect)
    assert np.all(ball[exact == 1] == 1) and exact.sum() > 0


def test_subset_normals_equal_full_estimation():
    """pfx_normals_subset_dev with want = 1 then 0 (grid prepared ahead, a ragged random mask
    incl. non-finite points) == pfx_normals_dev bit for bit; entries outside a subset untouched."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.synth import synth_room
    n = 120_000
    x, y, z, _ = synth_room(n, 35)
    x[::777] = np.nan
    dev = torch.device("cuda", 0)
    X, Y, Z = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    ref = [torch.empty(n, device=dev) for _ in range(4)]
    out = [torch.full((n,), 5.0, device=dev) for _ in range(4)]
    rng = np.random.default_rng(4)
    m = (rng.random(n) < 0.3).astype(np.uint8)
    M = torch.from_numpy(m).to(dev)
    with Context(0) as a, Context(0) as b:
        a.normals_dev(X, Y, Z, 0.05, *ref)
        b.normals_prepare_dev(X, Y, Z, 0.05)
        b.normals_subset_dev(X, Y, Z, 0.05, M, 1, *out)
        b.synchronize()
        half = out[0].cpu().numpy()
        assert np.all(half[m == 0] == 5.0)  # untouched
        b.normals_subset_dev(X, Y, Z, 0.05, M, 0, *out)
        a.synchronize(); b.synchronize()
    for r, o in zip(ref, out):
        r, o = r.cpu().numpy(), o.cpu().numpy()
        assert bits_equal(r, o)


@pytest.mark.parametrize("mode", [1, 2])
def test_support_first_pass_matches_default(mode):
    """OverlappedNarfFpfh with support_first (the support's normals -- subset lists and chains
    (1), or every list then a workgroup-partitioned chain pass (2) -- then FPFH beside the rest)
    gives the default schedule's keypoints, every normal and every descriptor bit for bit."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc
    from pcl_feature_extraction_amd.synth import synth_room
    n = 150_000
    x, y, z, _ = synth_room(n, 22)
    dev = torch.device("cuda", 0)
    outs = []
    for first in (0, mode):
        b = alloc(torch, n, dev, max_keypoints=4096)
        b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
        ctx, ctx_n = Context(0), Context(0)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
        run.support_first = first
        for _ in range(2):  # (the second pass reuses every buffer)
            kp, k = run(b)
        run.check()
        run.close()
        torch.cuda.synchronize(dev)
        outs.append((np.asarray(kp), k, np.stack([t.cpu().numpy() for t in (b.nx, b.ny, b.nz, b.curv)]),
                     b.desc[:k].cpu().numpy()))
        ctx.close(); ctx_n.close()
    (kp0, k0, n0, d0), (kp1, k1, n1, d1) = outs
    assert np.array_equal(kp0, kp1) and k0 == k1 and k0 > 0
    assert bits_equal(n0, n1)
    assert bits_equal(d0, d1)


def test_split_check_pass_matches_default_with_reruns():
    """OverlappedNarfFpfh with split_check (pfx_normals_launch_dev, FPFH queued behind it, then
    pfx_normals_finish_dev): equal to the default schedule bit for bit on a sequence of scans
    whose third one lies outside the second's widened bounds (the launched estimation is rerun
    exactly and FPFH after it)."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc
    from pcl_feature_extraction_amd.synth import synth_room
    n = 150_000
    x, y, z, _ = synth_room(n, 23)
    x2, y2, z2, _ = synth_room(n, 24)
    scans = [(x, y, z), (x2, y2, z2), (x2 + 5.0, y2, z2)]  # the third: a sensor moved by 5 m
    dev = torch.device("cuda", 0)
    res = {}
    for split in (False, True):
        b = alloc(torch, n, dev, max_keypoints=4096)
        ctx, ctx_n = Context(0), Context(0)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
        run.split_check = split
        outs = []
        for sx, sy, sz in scans:
            for t, a in zip((b.x, b.y, b.z), (sx, sy, sz)):
                t.copy_(torch.from_numpy(np.ascontiguousarray(a, np.float32)))
            kp, k = run(b)
            torch.cuda.synchronize(dev)
            outs.append((np.asarray(kp), k, np.stack([t.cpu().numpy() for t in (b.nx, b.ny, b.nz, b.curv)]),
                         b.desc[:k].cpu().numpy()))
        run.check()
        if split:
            assert ctx_n.stat("normals_speculative_reruns") >= 1
        run.close()
        ctx.close(); ctx_n.close()
        res[split] = outs
    for (kp0, k0, n0, d0), (kp1, k1, n1, d1) in zip(res[False], res[True]):
        assert np.array_equal(kp0, kp1) and k0 == k1
        assert bits_equal(n0, n1)
        assert bits_equal(d0, d1)


@pytest.mark.parametrize("shot_prep_first", [True, False])
def test_overlapped_shot_matches_sequential(shot_prep_first):
    """OverlappedNarfFpfh.shot (normals on the side stream beside NARF, SHOT's surface grid
    prepared ahead: before the estimation, its list kernels gated on it, or after NARF) ==
    pipeline.narf_shot on one stream, descriptors and frames bit for bit."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc, alloc_shot, narf_shot
    from pcl_feature_extraction_amd.synth import synth_seabed
    n = 150_000
    x, y, z, _ = synth_seabed(n, 31)
    dev = torch.device("cuda", 0)
    sample = torch.from_numpy(np.sort(np.random.default_rng(2).choice(n, 500, replace=False))).to(dev)
    outs = []
    for overlapped in (False, True):
        b = alloc(torch, n, dev, max_keypoints=4096)
        s = alloc_shot(torch, 8192, dev)
        b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
        ctx, ctx_n = Context(0), Context(0)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        if overlapped:
            run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
            run.shot_prep_first = shot_prep_first
            rows = run.shot(b, s, sample)
            run.close()
        else:
            rows = narf_shot(ctx, b, s, sample)
        torch.cuda.synchronize(dev)
        outs.append((rows, s.desc[:rows].cpu().numpy(), s.rf[:rows].cpu().numpy()))
        ctx.close(); ctx_n.close()
    (r0, d0, f0), (r1, d1, f1) = outs
    assert r0 == r1 and r0 >= 500
    assert bits_equal(d0, d1)
    assert bits_equal(f0, f1)


@pytest.mark.parametrize("launch_first,prep_first,grid_first", [(False, 2, False), (True, 0, False), (True, 1, False),
                                                                 (True, 2, True)])
def test_launch_order_variants_match_default(launch_first, prep_first, grid_first):
    """OverlappedNarfFpfh's launch-order attributes (every selectable schedule
    pinned): the estimation issued by the worker thread instead of the caller (launch_first =
    False) and FPFH's surface grid queued after NARF (prep_first 0) or after the estimation's
    launch (1), and the estimation's grid queued ahead of FPFH's rather than built inside its
    launch (grid_first = True), give the default schedule's keypoints, normals and descriptors
    bit for bit."""
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc
    from pcl_feature_extraction_amd.synth import synth_room
    n = 150_000
    x, y, z, _ = synth_room(n, 25)
    dev = torch.device("cuda", 0)
    outs = []
    for variant in (None, (launch_first, prep_first, grid_first)):
        b = alloc(torch, n, dev, max_keypoints=4096)
        b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
        ctx, ctx_n = Context(0), Context(0)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
        if variant is not None:
            run.launch_first, run.prep_first, run.grid_first = variant
        for _ in range(2):  # (the second pass reuses every buffer and the speculative grids)
            kp, k = run(b)
        run.check()
        run.close()
        torch.cuda.synchronize(dev)
        outs.append((np.asarray(kp), k, np.stack([t.cpu().numpy() for t in (b.nx, b.ny, b.nz, b.curv)]),
                     b.desc[:k].cpu().numpy()))
        ctx.close(); ctx_n.close()
    (kp0, k0, n0, d0), (kp1, k1, n1, d1) = outs
    assert np.array_equal(kp0, kp1) and k0 == k1 and k0 > 0
    assert bits_equal(n0, n1)
    assert bits_equal(d0, d1)
