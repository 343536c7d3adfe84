"""The device-resident pass (pipeline.py) end to end: the overlapped two-stream schedule used by
bench.py equals the sequential narf_fpfh, and both equal the oracle on the same scan."""
import numpy as np
import pytest

import oracle_lib as O

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
        outs.append((np.asarray(kp), k, b.nx.cpu().numpy(), b.desc[:k].cpu().numpy()))
        ctx.close(); ctx_n.close()
    (kp0, k0, n0, d0), (kp1, k1, n1, d1) = outs
    assert np.array_equal(kp0, kp1) and k0 == k1 and k0 > 0
    assert np.array_equal(np.nan_to_num(n0, nan=7).view(np.uint32), np.nan_to_num(n1, nan=7).view(np.uint32))
    assert np.array_equal(np.nan_to_num(d0, nan=7).view(np.uint32), np.nan_to_num(d1, nan=7).view(np.uint32))
    # against the CPU restatement
    okp = O.narf_keypoints(x, y, z)
    assert np.array_equal(kp1, okp)
    onx, ony, onz, _ = O.normals(x, y, z, 0.05)
    assert np.array_equal(np.nan_to_num(n1, nan=7).view(np.uint32), np.nan_to_num(onx, nan=7).view(np.uint32))
    rows = okp[okp < n]
    od = O.fpfh(x, y, z, onx, ony, onz, x[rows], y[rows], z[rows], 0.08)
    assert np.array_equal(np.nan_to_num(d1, nan=7).view(np.uint32), np.nan_to_num(od, nan=7).view(np.uint32))
