#!/usr/bin/env python3
"""Headline benchmark: Mpoints/s through NARF keypoints + FPFH descriptors on a 1M-point cloud
(BASELINE.json metric; configs[2] at N = 1, configs[4] = one 1M-point scan per GPU at N > 1).

One step = the reference's (Narf, FPFH) pass over one scan (pcl_feature_extraction_amd/pipeline.py):
range image -> border extraction -> NARF interest + NMS + greedy selection -> keypoint mapping ->
normals of the whole cloud (r = 0.05) -> FPFH at the keypoints (r = 0.08), inputs resident in HBM.
At N > 1 every rank processes its own scan and the descriptor matrices are gathered on every rank
over RCCL (dist.gather_descriptors: all_gather of the counts and of the padded K x 33 blocks)
inside the step.

`--workload shot` measures configs[3] instead (secondary line): a 1M-point underwater-style
seabed, normals + SHOT-352 (r = 0.08) at the NARF keypoints and a fixed 10,000-point sample.
`--workload match` measures the next row of SURVEY 8(f) (F1, Features<T>::findCorrespondences,
features.h:224-253): mutual 1-NN between the SHOT-352 descriptor sets of two such scans
(descriptors computed before the timed region; one step = one correspondence search).
`--workload iss` measures F3, the reference's active ISS keypoints (Keypoints::compute ISS
branch, keypoints.h:177-189): one step = cloud resolution + ISSKeypoint3D over the 1M-point room.
`--workload harris`: F3's Harris3D branch (keypoints.h:150-162 + getKeypointsCloud) over the same
room: normals (r 0.01) + response + suppression + corner refinement + snap.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fpfh|shot] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
N_POINTS = 1_000_000
SHOT_SAMPLE = 10_000

VERBOSE_TIMERS = ["grid_bbox", "grid_build", "normals", "normals_lists_phase", "normals_tiles", "normals_lists",
                  "normals_lists_small", "normals_lists_sparse",
                  "normals_lists_dense", "normals_lists_query", "normals_chain", "normals_chain_big", "normals_long", "range_image",
                  "narf_border", "narf_interest", "narf_nms", "narf_gather", "fpfh_mark", "fpfh_spfh",
                  "fpfh_support", "fpfh_weight", "shot"]
VERBOSE_STATS = ["normals_neighbors", "normals_queries", "normals_tiles_sparse", "normals_tiles_dense",
                 "normals_single", "normals_huge", "normals_long_lists", "normals_chain_wg_staged",
                 "normals_chain_wg_table", "normals_chain_wg_lane", "normals_chain_wg_deferred", "fpfh_spfh_points", "fpfh_spfh_pairs", "fpfh_spfh_exact_pairs", "narf_candidates", "narf_keypoints",
                 "narf_interest_fullimage", "narf_interest_grown", "narf_interest_window_px",
                 "narf_interest_visits", "narf_interest_queue_grown", "fpfh_weight_kmax", "fpfh_weight_sequential",
                 "shot_neighbors"]


def cpu_baseline(x, y, z, workload, sample=None):
    """The CPU restatement (oracle/, test infrastructure) on the same scan, threads as PCL:
    NARF and FPFH single-threaded (PCL 1.7 defaults, non-OMP FPFHEstimation), normals and SHOT
    OpenMP (NormalEstimationOMP / SHOTEstimationOMP)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    t0 = time.perf_counter()
    kp = O.narf_keypoints(x, y, z, threads=1)
    t1 = time.perf_counter()
    nx, ny, nz, _ = O.normals(x, y, z, 0.05, threads=threads)
    t2 = time.perf_counter()
    rows = kp[kp < len(x)]
    if workload == "fpfh":
        desc = O.fpfh(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08, threads=1)
        feat = "FPFH 1 thread"
    else:
        rows = np.r_[rows, sample]
        desc = O.shot(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08, threads=threads)
        feat = f"SHOT {threads} threads"
    t3 = time.perf_counter()
    return dict(seconds=t3 - t0, threads=threads, outputs=(kp, (nx, ny, nz), desc),
                sample=(f"the same 1M-point scan through the CPU restatement (oracle/): NARF 1 thread "
                        f"{t1 - t0:.1f}s, normals {threads} threads {t2 - t1:.1f}s, {feat} {t3 - t2:.1f}s at "
                        f"{len(rows)} rows; real PCL is not available anywhere in this pipeline"))


def full_size_parity(outputs, kp, b, desc, rows, shot):
    """The last timed step's outputs against the CPU restatement's on the whole scan: bit-exact
    (NaN positions equal) for keypoints, normals and descriptor rows."""
    import numpy as np
    okp, onorm, odesc = outputs
    if shot:
        odesc = odesc[0]

    def same(a, c):
        a, c = np.asarray(a, np.float32), np.asarray(c, np.float32)
        return bool(a.shape == c.shape and np.array_equal(np.nan_to_num(a, nan=7).view(np.uint32),
                                                          np.nan_to_num(c, nan=7).view(np.uint32)))
    res = {"normals": all(same(t.cpu().numpy(), o) for t, o in zip((b.nx, b.ny, b.nz), onorm)),
           "descriptors": same(desc[:rows].cpu().numpy(), odesc)}
    if kp is not None:
        res["keypoints"] = bool(np.array_equal(np.asarray(kp), okp))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["fpfh", "shot", "match", "iss", "harris"], default="fpfh")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if os.environ.get("PFX_BENCH_VERBOSE"):
        os.environ["PFX_VERBOSE_STATS"] = "1"  # libpfx diagnostics (extra host syncs): verbose runs only

    import numpy as np
    import torch
    import torch.distributed as dist

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.dist import gather_descriptors
    from pcl_feature_extraction_amd.pipeline import OverlappedNarfFpfh, alloc, alloc_shot, narf_shot
    from pcl_feature_extraction_amd.synth import synth_room, synth_seabed

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.workload == "match":
        return bench_match(args, torch, dev, world, rank, local)
    if args.workload == "iss":
        return bench_iss(args, torch, dev, world, rank, local)
    if args.workload == "harris":
        return bench_harris(args, torch, dev, world, rank, local)

    shot = args.workload == "shot"
    if shot:  # configs[3]: seabed seed 3 (per-rank seeds 300 + rank at N > 1)
        x, y, z, _ = synth_seabed(N_POINTS, 3 if world == 1 else 300 + rank)
    else:     # configs[2] (seed 2) / configs[4] (seeds 100..107)
        x, y, z, _ = synth_room(N_POINTS, 2 if world == 1 else 100 + rank)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx_n = Context(local)  # normal estimation overlapped with NARF on a second stream
    run_fpfh = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
    b = alloc(torch, N_POINTS, dev)
    b.x.copy_(torch.from_numpy(x))
    b.y.copy_(torch.from_numpy(y))
    b.z.copy_(torch.from_numpy(z))
    sample_np = np.sort(np.random.default_rng(10).choice(N_POINTS, SHOT_SAMPLE, replace=False))
    if shot:
        s = alloc_shot(torch, 1 << 16, dev)
        sample = torch.from_numpy(sample_np.astype(np.int64)).to(dev)
    gathered = None
    last_kp = None

    def step():
        nonlocal gathered, last_kp
        if shot:
            rows = narf_shot(ctx, b, s, sample)
            desc = s.desc
        else:
            last_kp, rows = run_fpfh(b)
            desc = b.desc
        if world > 1:
            gathered = gather_descriptors(torch, dist, desc, rows)
        return rows

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    for c in (ctx, ctx_n):
        c.set_timing(True)
        c.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rows = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    def merged(nm):  # a stage runs on one of the two contexts (grids on both)
        a, b_ = ctx.kernel_time(nm), ctx_n.kernel_time(nm)
        return a[0] + b_[0], a[1] + b_[1]

    def stat(nm):
        for c in (ctx_n, ctx) if nm.startswith("normals") else (ctx, ctx_n):
            try:
                return c.stat(nm)
            except Exception:
                pass
        raise KeyError(nm)

    timers = {nm: merged(nm) for nm in VERBOSE_TIMERS}
    if os.environ.get("PFX_BENCH_VERBOSE"):
        rep = {nm: round(ms / args.steps, 3) for nm, (ms, _) in timers.items() if ms > 0}
        print("per-step kernel ms:", json.dumps(rep), file=sys.stderr, flush=True)
        stats = {}
        for nm in VERBOSE_STATS:
            try:
                stats[nm] = stat(nm)
            except Exception:
                pass
        print("stats:", json.dumps(stats), file=sys.stderr, flush=True)
    for c in (ctx, ctx_n):
        c.set_timing(False)
    neighbors = stat("normals_neighbors")
    long_nb, long_q = stat("normals_long_neighbors"), stat("normals_long_queries")
    # the chain stage once more, alone on the GPU (after the timed region, not part of `value`):
    # in the timed step it shares the device with NARF on the other stream
    iso_ms = None
    if rank == 0 and not shot:
        ctx_n.set_timing(True)
        ctx_n.reset_timing()
        for _ in range(3):
            ctx_n.normals_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
        torch.cuda.synchronize(dev)
        iso_ms = (ctx_n.kernel_time("normals_chain")[0] + ctx_n.kernel_time("normals_chain_big")[0]) / 3
        ctx_n.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * N_POINTS * args.steps / elapsed / 1e6
        # roofline of the neighbour-gather kernel: k_normals_chain reads every query's
        # FLANN-ordered neighbour list and gathers the neighbours' coordinates into the ordered
        # covariance chains.  Algorithmic bytes per launch = sum_q |N_0.05(q)| * 12 B (xyz) +
        # 16 B (normal + curvature out) over the queries these kernels own, i.e. every query but
        # the lists longer than 1024 (k_normals_long's, reported beside); time = their HIP-event
        # duration on the ctx stream.
        algo_bytes = (neighbors - long_nb) * 12 + (N_POINTS - long_q) * 16
        # the chain stage is k_normals_chain (LDS-staged workgroups) + k_normals_chain_big (the
        # dense workgroups it defers to a 144 KB-LDS pass), run as two masked passes per step
        # (FPFH support points on the main stream, the rest on the side stream): its time per
        # step is the sum over both contexts' launches
        chain_ms = timers["normals_chain"][0] + timers["normals_chain_big"][0]
        stage_ms = timers["normals"][0] or sum(timers[nm][0] for nm in ("normals_lists_phase", "normals_chain",
                                                                          "normals_chain_big", "normals_long"))
        chain_s = chain_ms / args.steps / 1e3
        stage_s = stage_ms / args.steps / 1e3
        achieved = algo_bytes / chain_s / 1e9 if chain_s > 0 else 0.0
        stage_gbs = algo_bytes / stage_s / 1e9 if stage_s > 0 else 0.0
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_normals_chain.json")
        if os.path.exists(pmc):  # FETCH_SIZE x2 + WRITE_SIZE of k_normals_chain (scripts/gpu_pmc.sh)
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        # basis of `achieved`: the chain kernels' own launch durations, i.e. the isolated launches
        # (normal estimation alone on the device, right after the timed region).  Inside the step
        # the two masked chain passes run on two streams next to NARF's kernels, so their event
        # durations include the CU time those share; that in-step figure is reported beside it.
        in_step = {"chain_ms_per_step": round(chain_s * 1e3, 4), "achieved": round(achieved, 2),
                   "frac": round(achieved / HBM_PEAK_GBS, 5),
                   "note": "sum of the two masked passes' event durations inside the timed step (concurrent "
                           "with NARF on the other stream)"}
        if iso_ms is not None:
            basis_ms, basis = iso_ms, "isolated launches after the timed region (normal estimation alone)"
        else:
            basis_ms, basis = chain_s * 1e3, "in-step launches"
        basis_gbs = algo_bytes / (basis_ms / 1e3) / 1e9 if basis_ms > 0 else 0.0
        roofline = {"bound": "hbm", "kernel": "k_normals_chain + k_normals_chain_big", "achieved": round(basis_gbs, 2),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(basis_gbs / HBM_PEAK_GBS, 5),
                    "traffic": traffic, "algorithmic_bytes_per_launch": int(algo_bytes),
                    "chain_ms": round(basis_ms, 4), "basis": basis,
                    "neighbors_per_launch": int(neighbors - long_nb),
                    "long_lists": {"kernel": "k_normals_long", "lists": int(long_q), "neighbors": int(long_nb),
                                   "ms_per_step": round(timers["normals_long"][0] / args.steps, 4)},
                    "in_step": in_step,
                    "stage": {"name": "normals: grid + FLANN-ordered lists + chains",
                              "avg_ms": round(stage_s * 1e3, 4), "achieved": round(stage_gbs, 2),
                              "frac": round(stage_gbs / HBM_PEAK_GBS, 5)}}
        if shot:  # SHOT kernel: sum_q |N(q)| x 24 B (xyz + normal) per launch
            shot_ms, shot_n = timers["shot"]
            shot_s = (shot_ms / max(shot_n, 1)) / 1e3
            sb = stat("shot_neighbors") * 24
            # k_shot is this workload's dominant kernel (the chains take 0.5 ms of a 7.6 ms step):
            # it heads the roofline; the chain figures stay beside it.  On this dense cloud
            # (k(0.05) ~ 390) the chain's per-neighbour gather model exceeds the HBM peak because
            # the kernel stages coordinates once per workgroup in LDS; the PMC traffic file is
            # the default workload's, so no `traffic` here.
            chain = dict(roofline, kernel="k_normals_chain + k_normals_chain_big", traffic=None,
                         note="algorithmic model = 12 B per neighbour gather; coordinates are read once "
                              "per workgroup from HBM and reused from LDS")
            chain.pop("bound")
            shot_gbs = sb / shot_s / 1e9 if shot_s > 0 else 0.0
            roofline = {"bound": "hbm", "kernel": "k_shot", "achieved": round(shot_gbs, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(shot_gbs / HBM_PEAK_GBS, 5), "traffic": None,
                        "algorithmic_bytes_per_launch": int(sb), "avg_ms": round(shot_s * 1e3, 4),
                        "note": "sum_q |N_0.08(q)| x 24 B (xyz + normal) per launch (SURVEY 8(d)); VALU/LDS-atomic "
                                "bound, not HBM", "normals_chain": chain}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(x, y, z, args.workload, sample_np)
            cpu = {"value": round(N_POINTS / cb["seconds"] / 1e6, 6), "unit": "Mpoints/s",
                   "cores": cb["threads"], "kind": "port", "sample": cb["sample"],
                   "parity": full_size_parity(cb["outputs"], last_kp, b, s.desc if shot else b.desc, rows, shot)}
        if shot:
            metric = "Mpoints/s through NARF keypoint + normals + SHOT-352 descriptor on 1M-pt underwater-style cloud"
            workload = (f"configs[3] 1M-pt synthetic seabed, NARF(support 0.2) + normals(r 0.05) + SHOT-352(r 0.08) "
                        f"at the keypoints + a fixed {SHOT_SAMPLE}-point sample")
            data = "synthetic (synth_seabed: seeded fBm height field under a pinhole camera, k(0.08)~1000)"
        else:
            metric = "Mpoints/s through NARF keypoint + FPFH descriptor on 1M-pt cloud"
            workload = ("configs[2] 1M-pt synthetic room, NARF(support 0.2) + normals(r 0.05) + FPFH(r 0.08) at "
                        "the keypoints" if world == 1 else
                        "configs[4] one 1M-pt room scan per GPU + RCCL all_gather of K x 33 descriptors")
            data = "synthetic (synth_room: seeded pinhole room scan, k(0.05)~230; see synth.py)"
        line = {
            "metric": metric,
            "value": round(value, 4),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data,
            "config": {"workload": workload, "points_per_scan": N_POINTS, "descriptor_rows": int(rows),
                       "image": "640x480", "parallelism": f"scan-per-gpu x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    run_fpfh.close()
    ctx.close()
    ctx_n.close()
    if world > 1:
        dist.destroy_process_group()


def bench_match(args, torch, dev, world, rank, local):
    """F1: Features<SHOT352>::findCorrespondences between two 1M-point seabed scans (the second
    is the first turned by 3 degrees about the optical axis, re-noised), SHOT-352 at the NARF
    keypoints + the fixed 10,000-point sample of each.  Scans are independent per rank
    (replicas, no collective)."""
    import numpy as np
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import alloc, alloc_shot, narf_shot
    from pcl_feature_extraction_amd.synth import synth_seabed

    x, y, z, _ = synth_seabed(N_POINTS, 3 + 100 * rank)
    th = np.deg2rad(3.0)
    rng = np.random.default_rng(77 + rank)
    x2 = (np.cos(th) * x - np.sin(th) * y + rng.normal(0, 1e-3, N_POINTS)).astype(np.float32)
    y2 = (np.sin(th) * x + np.cos(th) * y + rng.normal(0, 1e-3, N_POINTS)).astype(np.float32)
    z2 = (z + rng.normal(0, 1e-3, N_POINTS)).astype(np.float32)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    sample = torch.from_numpy(np.sort(np.random.default_rng(10).choice(N_POINTS, SHOT_SAMPLE, replace=False))
                              .astype(np.int64)).to(dev)
    descs = []
    for cx, cy, cz in ((x, y, z), (x2, y2, z2)):
        b = alloc(torch, N_POINTS, dev)
        b.x.copy_(torch.from_numpy(cx))
        b.y.copy_(torch.from_numpy(cy))
        b.z.copy_(torch.from_numpy(cz))
        sb = alloc_shot(torch, 1 << 16, dev)
        rows = narf_shot(ctx, b, sb, sample)
        descs.append(sb.desc[:rows].clone())
    src, tgt = descs
    q = torch.empty(len(src), dtype=torch.int32, device=dev)
    m = torch.empty(len(src), dtype=torch.int32, device=dev)
    npairs = 0
    for _ in range(args.warmup):
        npairs = ctx.correspondences_dev(src, tgt, q, m)
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    ctx.reset_timing()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        npairs = ctx.correspondences_dev(src, tgt, q, m)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ns, nt = len(src), len(tgt)
    if rank == 0:
        # MFMA work per step: two tile passes over the padded (ns x nt) grid, K = 3 x 352 (bf16 split)
        pad = lambda v: (v + 127) // 128 * 128  # noqa: E731
        flops = 2 * 2.0 * pad(ns) * pad(nt) * 3 * 352
        tb, nb = ctx.kernel_time("match_bound")
        tf, _ = ctx.kernel_time("match_filter")
        tiles_s = (tb + tf) / max(nb, 1) / 1e3
        achieved = flops / tiles_s / 1e12 if tiles_s > 0 else 0.0
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            s_np, t_np = src.cpu().numpy(), tgt.cpu().numpy()
            c0 = time.perf_counter()
            oq, om = O.correspondences(s_np, t_np, threads=threads)
            csec = time.perf_counter() - c0
            same = bool(np.array_equal(oq, q[:npairs].cpu().numpy()) and np.array_equal(om, m[:npairs].cpu().numpy()))
            cpu = {"value": round(ns * nt / csec / 1e6, 3), "unit": "Mpairs/s", "cores": threads, "kind": "port",
                   "sample": (f"the same {ns} x {nt} SHOT-352 sets through the CPU restatement (oracle/or_match.cpp: "
                              f"exhaustive L2_Simple 1-NN both directions, OpenMP), {csec:.1f}s"),
                   "parity": {"correspondences": same}}
        line = {
            "metric": "Mpairs/s descriptor matching (Features::findCorrespondences, SHOT-352 mutual 1-NN)",
            "value": round(world * ns * nt * args.steps / elapsed / 1e6, 3),
            "unit": "Mpairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 (bf16-split MFMA bound + exact f32 L2_Simple)",
            "data": "synthetic (two synth_seabed scans, the second rotated 3 deg and re-noised)",
            "config": {"workload": "SURVEY 8(f) F1: mutual nearest SHOT-352 descriptors of two 1M-pt scans",
                       "source_rows": ns, "target_rows": nt, "correspondences": int(npairs),
                       "parallelism": f"replica x{world}"},
            "roofline": {"bound": "mfma", "kernel": "k_match_tiles<0> + k_match_tiles<1>", "achieved": round(achieved, 2),
                         "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 5),
                         "traffic": None, "flops_per_step": flops, "avg_tiles_ms": round(tiles_s * 1e3, 4),
                         "candidates": {"rows": ctx.stat("match_candidates_rows"),
                                        "cols": ctx.stat("match_candidates_cols")}},
            "cpu_baseline": cpu,
        }
        if os.environ.get("PFX_BENCH_VERBOSE"):
            rep = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4)
                   for nm in ("match", "match_bound", "match_filter", "match_exact")}
            print("per-step kernel ms:", json.dumps(rep), file=sys.stderr, flush=True)
        print(json.dumps(line), flush=True)
    ctx.close()


def bench_iss(args, torch, dev, world, rank, local):
    """Keypoints("ISS").compute over the 1M-point room scan (one per rank)."""
    import numpy as np

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import keypoints_iss
    from pcl_feature_extraction_amd.synth import synth_room

    x, y, z, _ = synth_room(N_POINTS, 2 if world == 1 else 100 + rank)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    dx, dy, dz = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    idx = torch.empty(N_POINTS, dtype=torch.int32, device=dev)
    k = 0
    for _ in range(args.warmup):
        k = keypoints_iss(ctx, dx, dy, dz, idx)
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    ctx.reset_timing()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k = keypoints_iss(ctx, dx, dy, dz, idx)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        # the scatter kernel (k_iss_cov): every point's salient neighbours' coordinates and its
        # third value; algorithmic bytes per launch = sum_q |N_6res(q)| x 12 B + N x 8 B
        nb = ctx.stat("iss_neighbors")
        ts, ns = ctx.kernel_time("iss_scatter")
        scat_s = ts / max(ns, 1) / 1e3
        algo = nb * 12 + N_POINTS * 8
        achieved = algo / scat_s / 1e9 if scat_s > 0 else 0.0
        stages = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4)
                  for nm in ("resolution", "resolution_nn2", "resolution_brute", "resolution_sum", "iss",
                             "iss_scatter", "iss_ordered", "iss_nms")}
        res = ctx.cloud_resolution_dev(dx, dy, dz)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            c0 = time.perf_counter()
            ores, _ = O.cloud_resolution(x, y, z, threads=threads)
            okp, _ = O.iss_keypoints(x, y, z, 6 * ores, 4 * ores, threads=threads)
            csec = time.perf_counter() - c0
            same = bool(ores == res and np.array_equal(okp, idx[:k].cpu().numpy()))
            cpu = {"value": round(N_POINTS / csec / 1e6, 6), "unit": "Mpoints/s", "cores": threads, "kind": "port",
                   "sample": (f"the same 1M-point scan through the CPU restatement (oracle/or_keypoints.cpp: grid "
                              f"kNN + sequential double sum, OpenMP radius searches), {csec:.1f}s"),
                   "parity": {"resolution": bool(ores == res), "keypoints": same}}
        line = {
            "metric": "Mpoints/s through ISS keypoints (Keypoints::compute ISS branch) on 1M-pt cloud",
            "value": round(world * N_POINTS * args.steps / elapsed / 1e6, 4),
            "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 search, f64 scatter + eigen",
            "data": "synthetic (synth_room: seeded pinhole room scan; see synth.py)",
            "config": {"workload": "SURVEY 8(f) F3: computeCloudResolution + ISSKeypoint3D(6 res, 4 res, 5, 0.975, "
                                   "0.975) on configs[2]'s 1M-pt room", "points_per_scan": N_POINTS,
                       "resolution": res, "keypoints": int(k), "parallelism": f"scan-per-gpu x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_iss_cov", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None, "algorithmic_bytes_per_launch": int(algo), "avg_ms": round(scat_s * 1e3, 4),
                         "neighbors_per_launch": int(nb), "stages_ms_per_step": stages,
                         "ordered_points": ctx.stat("iss_ordered"),
                         "resolution_rounds": ctx.stat("resolution_rounds"),
                         "resolution_brute": ctx.stat("resolution_brute"),
                         "resolution_exact_sum": ctx.stat("resolution_exact_sum")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()


def bench_harris(args, torch, dev, world, rank, local):
    """Keypoints("Harris3D").compute over the 1M-point room scan (one per rank)."""
    import numpy as np

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import keypoints_harris3d
    from pcl_feature_extraction_amd.synth import synth_room

    x, y, z, _ = synth_room(N_POINTS, 2 if world == 1 else 100 + rank)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    dx, dy, dz = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    idx = torch.empty(N_POINTS, dtype=torch.int32, device=dev)
    k = 0
    for _ in range(args.warmup):
        k = keypoints_harris3d(ctx, dx, dy, dz, idx)
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    ctx.reset_timing()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k = keypoints_harris3d(ctx, dx, dy, dz, idx)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        # the response kernel: every query's FLANN-ordered list (4 B entries) and its neighbours'
        # normals; algorithmic bytes per launch = sum_q |N_0.01(q)| x (4 + 12) B + N x 4 B
        nb = ctx.stat("normals_neighbors")
        tr, nr = ctx.kernel_time("harris3d_response")
        resp_s = tr / max(nr, 1) / 1e3
        algo = nb * 16 + N_POINTS * 4
        achieved = algo / resp_s / 1e9 if resp_s > 0 else 0.0
        stages = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4)
                  for nm in ("harris3d", "normals_lists_phase", "grid_bbox", "grid_build", "normals_tiles",
                             "normals_lists_small", "normals_lists_sparse", "normals_lists_dense", "normals_lists_query", "normals_chain",
                             "normals_chain_big", "normals_long", "harris3d_response", "harris3d_refine")}
        corners = ctx.stat("harris3d_corners")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            c0 = time.perf_counter()
            okp, _, _ = O.harris3d(x, y, z, 0.01, 1e-6, True, threads=threads)
            csec = time.perf_counter() - c0
            same = bool(np.array_equal(okp, idx[:k].cpu().numpy()))
            cpu = {"value": round(N_POINTS / csec / 1e6, 6), "unit": "Mpoints/s", "cores": threads, "kind": "port",
                   "sample": (f"the same 1M-point scan through the CPU restatement (oracle/or_keypoints.cpp "
                              f"orc_harris3d: OpenMP normals, responses, suppression, refinement), {csec:.1f}s"),
                   "parity": {"keypoints": same}}
        line = {
            "metric": "Mpoints/s through Harris3D keypoints (Keypoints::compute HARRIS_3D branch) on 1M-pt cloud",
            "value": round(world * N_POINTS * args.steps / elapsed / 1e6, 4),
            "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (synth_room: seeded pinhole room scan; see synth.py)",
            "config": {"workload": "SURVEY 8(f) F3: HarrisKeypoint3D(HARRIS, r 0.01, nms, threshold 1e-6, refine) + "
                                   "getKeypointsCloud on configs[2]'s 1M-pt room", "points_per_scan": N_POINTS,
                       "corners": int(corners), "keypoints": int(k), "parallelism": f"scan-per-gpu x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_harris_response + k_harris_nms", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None, "algorithmic_bytes_per_launch": int(algo), "avg_ms": round(resp_s * 1e3, 4),
                         "neighbors_per_launch": int(nb), "stages_ms_per_step": stages},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
