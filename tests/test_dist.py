"""Multi-process data path of bench.py (N > 1) on CPU: gloo, world_size 2 and 3, the same
gather_descriptors() the RCCL run uses (pcl_feature_extraction_amd/dist.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pcl_feature_extraction_amd.dist import gather_descriptors


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, ks, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = ks[rank]
        desc = torch.full((max(k, 1) + 3, 33), -1.0)  # rows beyond k are garbage, must not travel
        desc[:k] = torch.arange(k * 33, dtype=torch.float32).reshape(k, 33) + 1000.0 * rank
        got = gather_descriptors(torch, dist, desc, k)
        out_q.put((rank, [g.clone() for g in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ks", [[5, 0], [3, 7, 1]])
def test_gather_descriptors_gloo(ks):
    world = len(ks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        got = results[rank]
        assert [g.shape[0] for g in got] == ks
        for src, k in enumerate(ks):
            want = torch.arange(k * 33, dtype=torch.float32).reshape(k, 33) + 1000.0 * src
            assert torch.equal(got[src], want)
