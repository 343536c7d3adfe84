"""CPU rehearsal of bench.py's multi-GPU batch path (tests/test_dist.py): the same self-launcher
(pcl_feature_extraction_amd/launch.py) and the same round-robin scan ownership + gather to rank 0
(pcl_feature_extraction_amd/dist.py) over gloo, with a deterministic per-scan stand-in for the
descriptor computation (K_s x 33 rows and K_s indices derived from the scan's seed).

    python tests/helpers/batch_gather_cpu.py --gpus N --scans S --out result.npz
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def scan_blocks(seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    k = int(rng.integers(0, 9))          # 0 rows happens: a scan without keypoints
    return rng.standard_normal((k, 33)).astype(np.float32), rng.integers(0, 1_000_000, k).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scans", type=int, default=8)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    from pcl_feature_extraction_amd import launch
    if launch.needs_spawn(args.gpus):
        sys.exit(launch.spawn(args.gpus, os.path.abspath(__file__), sys.argv[1:]))

    import numpy as np
    import torch
    import torch.distributed as dist

    from pcl_feature_extraction_amd.dist import gather_to_root, in_scan_order, owned_scans
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    try:
        mine = owned_scans(args.scans, world, rank)
        blocks = [tuple(torch.from_numpy(a) for a in scan_blocks(100 + s)) for s in mine]
        if world > 1:
            got = gather_to_root(torch, dist, blocks, 33, torch.device("cpu"), -(-args.scans // world))
        else:
            got = [blocks]
        if rank == 0:
            ordered = in_scan_order(got, args.scans, world)
            np.savez(args.out, desc=np.concatenate([d.numpy().reshape(-1, 33) for d, _ in ordered]),
                     idx=np.concatenate([i.numpy() for _, i in ordered]),
                     rows=np.array([d.shape[0] for d, _ in ordered]), world=world)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
