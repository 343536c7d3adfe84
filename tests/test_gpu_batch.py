"""configs[4] on the GPU: the batch of 8 room scans (seeds 100-107)
through bench.py's batch path at world 1 -- pipeline.BatchNarfFpfh (scan i's FPFH and scan i+1's
NARF under scan i+1's normal estimation) followed by dist.gather_to_root over a real
torch.distributed process group (RCCL) -- the per-scan loop of evaluation.cpp:272-852.

Bar: every gathered scan's (K_s x 33 descriptors, K_s cloud indices) equals a single-scan
pipeline.narf_fpfh run on fresh contexts bit for bit, and two scans equal the CPU restatement
(oracle/, parity vs real PCL unpinned: DESIGN.md) -- at 200k points per scan (every scan against a
fresh single-scan pass), and at configs[4]'s own 1M points per scan (both batch paths, two scans
against the oracle)."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

N_SCAN = 200_000
SEEDS = [100 + i for i in range(8)]


def _bits(a):  # raw bits, NaN rows included (PCL's quiet_NaN on every side)
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_config4_batch_gather_matches_single_scan_and_oracle():
    import torch
    import torch.distributed as dist
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.dist import gather_to_root, in_scan_order, owned_scans
    from pcl_feature_extraction_amd.pipeline import BatchNarfFpfh, alloc, keypoint_rows, narf_fpfh
    from pcl_feature_extraction_amd.synth import synth_room

    dev = torch.device("cuda", 0)
    clouds = [synth_room(N_SCAN, s)[:3] for s in SEEDS]
    mine = owned_scans(len(SEEDS), 1, 0)
    assert mine == list(range(8))

    def load(c):
        b = alloc(torch, N_SCAN, dev, max_keypoints=4096)
        for t, a in zip((b.x, b.y, b.z), c):
            t.copy_(torch.from_numpy(a))
        return b

    # the batch path, as bench.py runs it on a rank that owns all 8 scans
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        scans = [load(c) for c in clouds]
        ctx, ctx_n = Context(0), Context(0)
        run = BatchNarfFpfh(torch, ctx, ctx_n, dev)
        res = run(scans)
        run.check()
        blocks = [(b.desc[:k], torch.from_numpy(keypoint_rows(kp, N_SCAN).astype(np.int32)).to(dev))
                  for b, (kp, k) in zip(scans, res)]
        got = in_scan_order(gather_to_root(torch, dist, blocks, 33, dev, len(mine)), len(SEEDS), 1)
        torch.cuda.synchronize(dev)
        got = [(d.cpu().numpy(), i.cpu().numpy()) for d, i in got]
        kps = [np.asarray(kp) for kp, _ in res]
        run.close()
        ctx.close()
        ctx_n.close()
    finally:
        dist.destroy_process_group()

    assert all(len(i) > 0 for _, i in got)  # every scan yields keypoints at this size
    # each scan == a single-scan sequential pass on fresh contexts
    for s, c in enumerate(clouds):
        b = load(c)
        with Context(0) as one:
            one.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            kp, k = narf_fpfh(one, b)
            torch.cuda.synchronize(dev)
        assert np.array_equal(np.asarray(kp), kps[s]), s
        d, i = got[s]
        assert d.shape == (k, 33) and np.array_equal(i, keypoint_rows(kp, N_SCAN).astype(np.int32)), s
        assert np.array_equal(_bits(d), _bits(b.desc[:k].cpu().numpy())), s
    # two scans against the CPU restatement
    for s in (0, 5):
        x, y, z = clouds[s]
        okp = O.narf_keypoints(x, y, z)
        assert np.array_equal(kps[s], okp), s
        nx, ny, nz, _ = O.normals(x, y, z, 0.05, threads=16)
        rows = keypoint_rows(okp, N_SCAN)
        od = O.fpfh(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08, threads=16)
        assert np.array_equal(_bits(got[s][0]), _bits(od)), s
        assert np.array_equal(got[s][1], rows.astype(np.int32)), s


N_FULL = 1_000_000


def test_config4_full_size_batch_both_paths_and_oracle():
    """configs[4] at its own size on the one GPU: the 8 x 1M-point room scans (seeds 100-107)
    through bench.py's batch path (BatchNarfFpfh + dist.gather_to_root over RCCL at world 1) and
    through the C-ABI batch (pfx_batch_narf_fpfh: host scans in, scan-order rows out): both agree
    bit for bit on every scan, and scans 0 and 5 equal the CPU restatement at full size
    (keypoints, descriptor rows, cloud indices)."""
    import torch
    import torch.distributed as dist
    from pcl_feature_extraction_amd import Batch, Context
    from pcl_feature_extraction_amd.dist import gather_to_root, in_scan_order
    from pcl_feature_extraction_amd.pipeline import BatchNarfFpfh, alloc, keypoint_rows
    from pcl_feature_extraction_amd.synth import synth_room

    dev = torch.device("cuda", 0)
    clouds = [tuple(np.ascontiguousarray(a) for a in synth_room(N_FULL, s)[:3]) for s in SEEDS]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        scans = []
        for c in clouds:
            b = alloc(torch, N_FULL, dev, max_keypoints=4096)
            for t, a in zip((b.x, b.y, b.z), c):
                t.copy_(torch.from_numpy(a))
            scans.append(b)
        ctx, ctx_n = Context(0), Context(0)
        run = BatchNarfFpfh(torch, ctx, ctx_n, dev)
        res = run(scans)
        run.check()
        blocks = [(b.desc[:k], torch.from_numpy(keypoint_rows(kp, N_FULL).astype(np.int32)).to(dev))
                  for b, (kp, k) in zip(scans, res)]
        got = in_scan_order(gather_to_root(torch, dist, blocks, 33, dev, len(SEEDS)), len(SEEDS), 1)
        torch.cuda.synchronize(dev)
        got = [(d.cpu().numpy(), i.cpu().numpy()) for d, i in got]
        kps = [np.asarray(kp) for kp, _ in res]
        run.close()
        ctx.close()
        ctx_n.close()
        del scans, blocks
    finally:
        dist.destroy_process_group()
    with Batch([0]) as bt:
        cab = bt.narf_fpfh(clouds)
    assert len(cab) == len(SEEDS)
    for s in range(len(SEEDS)):
        assert len(got[s][1]) > 0, s
        assert np.array_equal(cab[s][1], got[s][1]), s
        assert np.array_equal(_bits(cab[s][0]), _bits(got[s][0])), s
    for s in (0, 5):
        x, y, z = clouds[s]
        okp = O.narf_keypoints(x, y, z, threads=16)
        assert np.array_equal(kps[s], okp), s
        nx, ny, nz, _ = O.normals(x, y, z, 0.05, threads=16)
        rows = keypoint_rows(okp, N_FULL)
        od = O.fpfh(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08, threads=16)
        assert np.array_equal(got[s][1], rows.astype(np.int32)), s
        assert np.array_equal(_bits(got[s][0]), _bits(od)), s
