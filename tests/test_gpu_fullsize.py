"""Parity at BASELINE.json's full sizes: the bench workloads themselves (1M-point scans through the
device-resident pass) against the CPU restatement on the same scan.  The oracle finishes these in
seconds with OpenMP threads, so the check is bit-exact rather than a property test.

  configs[2]: synth_room(1M, seed 2), NARF(support 0.2) + normals(r 0.05) + FPFH(r 0.08)
  configs[3]: synth_seabed(1M, seed 3), NARF + normals + SHOT-352(r 0.08) at the keypoints and a
              fixed 10k-point sample (bench.py's sample)
"""
import numpy as np
import pytest

import oracle_lib as O
from parity import bits_equal

pytestmark = pytest.mark.gpu

N = 1_000_000
THREADS = 16


def _same(a, b):
    return bits_equal(a, b)  # raw bits, NaN rows included


def _scan(torch, dev, x, y, z, max_keypoints=1 << 16):
    from pcl_feature_extraction_amd.pipeline import alloc
    b = alloc(torch, len(x), dev, max_keypoints=max_keypoints)
    for t, a in ((b.x, x), (b.y, y), (b.z, z)):
        t.copy_(torch.from_numpy(a))
    return b


def test_config2_room_narf_fpfh_full_size():
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh
    from pcl_feature_extraction_amd.synth import synth_room
    x, y, z, _ = synth_room(N, 2)
    dev = torch.device("cuda", 0)
    b = _scan(torch, dev, x, y, z)
    with Context(0) as ctx, Context(0) as ctx_n:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
        try:
            kp, k = run(b)
        finally:
            run.close()
        torch.cuda.synchronize(dev)
    okp = O.narf_keypoints(x, y, z, threads=THREADS)
    assert np.array_equal(np.asarray(kp), okp) and k > 0
    on = O.normals(x, y, z, 0.05, threads=THREADS)
    for t, o in zip((b.nx, b.ny, b.nz, b.curv), on):
        assert _same(t.cpu().numpy(), o)
    rows = okp[okp < N]
    od = O.fpfh(x, y, z, on[0], on[1], on[2], x[rows], y[rows], z[rows], 0.08, threads=THREADS)
    d = b.desc[:k].cpu().numpy()
    assert _same(d, od)
    ok = ~np.isnan(od).any(axis=1)
    assert ok.any() and np.allclose(d[ok].sum(axis=1), 300.0, atol=2e-3)  # 3 x 100 per histogram


def test_config3_seabed_shot_full_size():
    import torch
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import alloc_shot, narf_shot
    from pcl_feature_extraction_amd.synth import synth_seabed
    x, y, z, _ = synth_seabed(N, 3)
    dev = torch.device("cuda", 0)
    b = _scan(torch, dev, x, y, z)
    s = alloc_shot(torch, 1 << 16, dev)
    sample_np = np.sort(np.random.default_rng(10).choice(N, 10_000, replace=False))
    sample = torch.from_numpy(sample_np.astype(np.int64)).to(dev)
    with Context(0) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        rows = narf_shot(ctx, b, s, sample)
        torch.cuda.synchronize(dev)
    okp = O.narf_keypoints(x, y, z, threads=THREADS)
    q = np.r_[okp[okp < N], sample_np]
    assert rows == len(q)
    on = O.normals(x, y, z, 0.05, threads=THREADS)
    for t, o in zip((b.nx, b.ny, b.nz, b.curv), on):
        assert _same(t.cpu().numpy(), o)
    od, orf = O.shot(x, y, z, on[0], on[1], on[2], x[q], y[q], z[q], 0.08, threads=THREADS)
    assert _same(s.desc[:rows].cpu().numpy(), od)
    assert _same(s.rf[:rows].cpu().numpy(), orf)
