"""Multi-process data path of bench.py (N > 1) on CPU, gloo: the gather of per-scan descriptor
blocks to rank 0 (pcl_feature_extraction_amd/dist.py, the code the RCCL run uses) and the
self-launcher that lets the driver call `bench.py --gpus N` directly
(pcl_feature_extraction_amd/launch.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pcl_feature_extraction_amd.dist import gather_descriptors, gather_to_root, in_scan_order, owned_scans

HERE = os.path.dirname(os.path.abspath(__file__))


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
        # gather_to_root: this rank owns scans rank, rank + world, ... with k + scan rows each
        n_scans = 2 * world + 1
        mine = owned_scans(n_scans, world, rank)
        blocks = [(torch.full((k + s % 3, 33), float(s)), torch.arange(k + s % 3, dtype=torch.int32) + 100 * s)
                  for s in mine]
        root = gather_to_root(torch, dist, blocks, 33, torch.device("cpu"), -(-n_scans // world))
        if root is not None:
            root = [(d.numpy().copy(), i.numpy().copy()) for d, i in in_scan_order(root, n_scans, world)]
        # numpy, not tensors: torch shares tensor storage through file descriptors served by this
        # process, which may already have exited when the parent unpickles them
        out_q.put((rank, [g.numpy().copy() for g in got], root))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ks", [[5, 0], [3, 7, 1]])
def test_gather_gloo(ks):
    world = len(ks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {r: (g, root) for r, g, root in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        got, root = results[rank]
        assert [g.shape[0] for g in got] == ks
        for src, k in enumerate(ks):
            want = torch.arange(k * 33, dtype=torch.float32).reshape(k, 33) + 1000.0 * src
            assert torch.equal(torch.from_numpy(got[src]), want)
        assert (root is None) == (rank != 0)
    n_scans = 2 * world + 1
    root = results[0][1]
    assert len(root) == n_scans
    for s, (d, i) in enumerate(root):
        k = ks[s % world] + s % 3
        assert torch.equal(torch.from_numpy(d), torch.full((k, 33), float(s)))
        assert torch.equal(torch.from_numpy(i), torch.arange(k, dtype=torch.int32) + 100 * s)


def test_owned_scans_round_robin():
    for world in (1, 2, 3, 4, 8):
        got = sorted(s for r in range(world) for s in owned_scans(8, world, r))
        assert got == list(range(8))
        assert max(len(owned_scans(8, world, r)) for r in range(world)) == -(-8 // world)


@pytest.mark.parametrize("world", [2, 3])
def test_self_launcher_gather_equals_single_rank(tmp_path, world):
    """`script --gpus N` without torch.distributed.run spawns N ranks itself (bench.py's path);
    the batch gathered on rank 0 equals the single-rank concatenation in scan order."""
    script = os.path.join(HERE, "helpers", "batch_gather_cpu.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    one, many = tmp_path / "one.npz", tmp_path / "many.npz"
    subprocess.run([sys.executable, script, "--gpus", "1", "--scans", "8", "--out", str(one)], env=env,
                   check=True, timeout=120)
    subprocess.run([sys.executable, script, "--gpus", str(world), "--scans", "8", "--out", str(many)], env=env,
                   check=True, timeout=180)
    a, b = np.load(one), np.load(many)
    assert int(b["world"]) == world and int(a["world"]) == 1
    assert np.array_equal(a["rows"], b["rows"]) and a["rows"].sum() > 0
    assert np.array_equal(a["desc"], b["desc"]) and np.array_equal(a["idx"], b["idx"])
