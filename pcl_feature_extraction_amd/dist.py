"""Multi-GPU data path of the scan batch: one process per GPU, scans dealt
round-robin over the ranks, each rank processes its scans end to end (no halo, no exchange
inside a scan), and the per-scan descriptor matrices are collected on rank 0 after compute.

The reference keeps every scan's K_s x 33 descriptors in host memory of one process
(evaluation.cpp:272-852 loops over the scans and hands them to its matching stage); here the
scans live on G devices, so after compute

  1. one all_gather of a small int64 count vector (scans held + K_s per scan) per rank, so every
     rank knows every message size (K_s differ per scan), then
  2. grouped point-to-point sends of each rank's packed K x 33 float descriptors and K int32
     cloud indices to rank 0 (torch.distributed.batch_isend_irecv: ncclSend/ncclRecv in one
     group over RCCL/xGMI; gloo on CPU) -- a gather to the root, no padding, no all-to-all.

Nothing here touches a GPU by itself: the tensors' device decides (CUDA with nccl, CPU with
gloo), which is what lets tests/test_dist.py run the same code on CPU.
"""
from __future__ import annotations


def owned_scans(n_scans: int, world: int, rank: int) -> list:
    """Scan indices rank `rank` processes: round-robin, scan s on rank s % world."""
    return list(range(rank, n_scans, world))


def gather_to_root(torch, dist, blocks, dim: int, device, max_per_rank: int, root: int = 0, group=None):
    """Collect every rank's per-scan (desc [K_s, dim] float32, idx [K_s] int32) blocks on `root`.

    `blocks` lists this rank's scans in owned order; `max_per_rank` bounds len(blocks) on every
    rank (ceil(n_scans / world)).  Returns, on root, a list over ranks of lists of (desc, idx)
    (root's own blocks are returned as given); None on the other ranks."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(blocks) > max_per_rank:
        raise ValueError(f"{len(blocks)} scans on rank {rank} > max_per_rank {max_per_rank}")
    if world == 1:
        return [list(blocks)]
    counts = torch.full((max_per_rank + 1,), -1, dtype=torch.int64, device=device)
    counts[0] = len(blocks)
    for i, (d, _) in enumerate(blocks):
        counts[1 + i] = int(d.shape[0])
    every = [torch.empty_like(counts) for _ in range(world)]
    dist.all_gather(every, counts, group=group)
    table = [[int(v) for v in t.tolist()] for t in every]   # one host read of a tiny vector
    per_rank_k = [c[1:1 + c[0]] for c in table]

    ops = []
    recv = {}
    if rank == root:
        for r in range(world):
            tot = sum(per_rank_k[r])
            if r == root or tot == 0:
                continue
            rd = torch.empty((tot, dim), dtype=torch.float32, device=device)
            ri = torch.empty((tot,), dtype=torch.int32, device=device)
            recv[r] = (rd, ri)
            ops.append(dist.P2POp(dist.irecv, rd, r, group=group))
            ops.append(dist.P2POp(dist.irecv, ri, r, group=group))
    elif sum(per_rank_k[rank]) > 0:
        sd = torch.cat([d.reshape(-1, dim) for d, _ in blocks]).contiguous()
        si = torch.cat([i.reshape(-1) for _, i in blocks]).to(torch.int32).contiguous()
        ops.append(dist.P2POp(dist.isend, sd, root, group=group))
        ops.append(dist.P2POp(dist.isend, si, root, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != root:
        return None
    out = []
    for r in range(world):
        if r == root:
            out.append(list(blocks))
            continue
        ks = per_rank_k[r]
        if r not in recv:
            out.append([(torch.empty((0, dim), dtype=torch.float32, device=device),
                         torch.empty((0,), dtype=torch.int32, device=device)) for _ in ks])
            continue
        rd, ri = recv[r]
        parts, o = [], 0
        for k in ks:
            parts.append((rd[o:o + k], ri[o:o + k]))
            o += k
        out.append(parts)
    return out


def in_scan_order(per_rank, n_scans: int, world: int) -> list:
    """Root's gather result (list over ranks of owned-order blocks) -> list over scans."""
    out = [None] * n_scans
    for r, parts in enumerate(per_rank):
        for s, blk in zip(owned_scans(n_scans, world, r), parts):
            out[s] = blk
    return out


def gather_descriptors(torch, dist, desc, k: int, group=None):
    """All ranks: returns [desc_r[:k_r] for r in ranks] (one all_gather of the counts and one of
    the blocks padded to max k).  Kept for callers that want the matrices on every rank; the
    batch path uses gather_to_root."""
    world = dist.get_world_size(group)
    dev = desc.device
    kk = torch.tensor([int(k)], device=dev, dtype=torch.int64)
    ks = [torch.zeros_like(kk) for _ in range(world)]
    dist.all_gather(ks, kk, group=group)
    counts = [int(t.item()) for t in ks]
    kmax = max(max(counts), 1)
    send = torch.zeros((kmax, desc.shape[1]), device=dev, dtype=desc.dtype)
    if k > 0:
        send[:k] = desc[:k]
    recv = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(recv, send, group=group)
    return [r[:c] for r, c in zip(recv, counts)]
