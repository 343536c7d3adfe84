"""Run-to-run determinism: list offsets, arena slots and work-queue
order depend on scheduling (wave-aggregated / per-workgroup atomics), the outputs must not.
Each workload runs twice on one context and once more on a fresh context; every output is
compared bit for bit (NaN payloads included)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else (np.uint64 if a.dtype == np.float64 else a.dtype))


def _same(outs):
    ref = outs[0]
    for o in outs[1:]:
        assert len(o) == len(ref)
        for a, b in zip(ref, o):
            a, b = np.asarray(a), np.asarray(b)
            assert a.shape == b.shape and np.array_equal(_bits(a), _bits(b))


def _three_runs(fn):
    from pcl_feature_extraction_amd import Context
    outs = []
    with Context(0) as c:
        outs.append(fn(c))
        outs.append(fn(c))
    with Context(0) as c:
        outs.append(fn(c))
    _same(outs)
    return outs[0]


def test_overlapped_narf_normals_fpfh_is_deterministic():
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc
    from pcl_feature_extraction_amd.synth import synth_room
    n = 300_000
    x, y, z, _ = synth_room(n, 5)
    dev = torch.device("cuda", 0)
    b = alloc(torch, n, dev, max_keypoints=4096)
    b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
    outs = []
    for fresh in (False, False, True):
        if fresh or not outs:
            ctx, ctx_n = Context(0), Context(0)
            ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
        for t in (b.nx, b.ny, b.nz, b.curv, b.desc):
            t.fill_(-1.0)
        kp, k = run(b)
        torch.cuda.synchronize(dev)
        outs.append((np.asarray(kp), np.array([k]), *[t.cpu().numpy() for t in (b.nx, b.ny, b.nz, b.curv)],
                     b.desc[:k].cpu().numpy()))
        if fresh or len(outs) == 2:
            run.close(); ctx.close(); ctx_n.close()
    _same(outs)
    assert outs[0][1][0] > 0


def test_iss_is_deterministic():
    from pcl_feature_extraction_amd.synth import synth_room
    x, y, z, _ = synth_room(200_000, 8)

    def run(c):
        res = c.cloud_resolution(x, y, z)
        kp, third = c.iss_keypoints(x, y, z, 6 * res, 4 * res, return_third=True)
        return np.array([res]), np.asarray(kp), np.asarray(third)
    out = _three_runs(run)
    assert len(out[1]) > 0


def test_harris3d_is_deterministic():
    from pcl_feature_extraction_amd.synth import synth_room
    x, y, z, _ = synth_room(200_000, 9)

    def run(c):
        kp, resp, cor = c.harris3d_keypoints(x, y, z, 0.01, 1e-6, True, details=True)
        return np.asarray(kp), np.asarray(resp), np.asarray(cor)
    out = _three_runs(run)
    assert len(out[0]) > 0


def test_shot_and_match_are_deterministic():
    from pcl_feature_extraction_amd.synth import synth_seabed
    x, y, z, _ = synth_seabed(150_000, 3)
    q = np.arange(0, len(x), 61)

    def run(c):
        nx, ny, nz, cv = c.normals(x, y, z, 0.05)
        d, rf = c.shot(x, y, z, nx, ny, nz, x[q], y[q], z[q], 0.08)
        ok = np.isfinite(d).all(axis=1)
        qi, mi = c.correspondences(d[ok][::2], d[ok][1::2])
        return nx, ny, nz, cv, d, rf, qi, mi
    _three_runs(run)
