#!/usr/bin/env python3
"""Headline benchmark: Mpoints/s through NARF keypoint + FPFH descriptor on 1M-pt clouds
(BASELINE.json metric; configs[2] at --gpus 1, configs[4] = the fixed batch of 8 1M-pt scans
round-robin over the GPUs at N > 1).

One scan = the reference's (Narf, FPFH) pass (pcl_feature_extraction_amd/pipeline.py):
range image -> border extraction -> NARF interest + NMS + greedy selection -> keypoint mapping ->
normals of the whole cloud (r = 0.05) -> FPFH at the keypoints (r = 0.08), inputs resident in HBM
(`value`); the same step with H2D of the scan and D2H of the descriptors inside it is reported
beside it (`end_to_end_h2d_d2h`).  At N > 1 every rank processes its scans (8/N each) and the
K_s x 33 descriptor matrices + K_s indices are gathered on rank 0 over RCCL (grouped
send/recv, dist.gather_to_root) inside the step.  `bench.py --gpus N` without an external
launcher starts its N ranks itself (launch.py) before touching a GPU.

`--workload shot` measures configs[3] instead (secondary line): a 1M-point underwater-style
seabed, normals + SHOT-352 (r = 0.08) at the NARF keypoints and a fixed 10,000-point sample.
`--workload match` measures the next row of SURVEY 8(f) (F1, Features<T>::findCorrespondences,
features.h:224-253): mutual 1-NN between the SHOT-352 descriptor sets of two such scans
(descriptors computed before the timed region; one step = one correspondence search).
`--workload iss` measures F3, the reference's active ISS keypoints (Keypoints::compute ISS
branch, keypoints.h:177-189): one step = cloud resolution + ISSKeypoint3D over the 1M-point room.
`--workload harris`: F3's Harris3D branch (keypoints.h:150-162 + getKeypointsCloud) over the same
room: normals (r 0.01) + response + suppression + corner refinement + snap.
`--workload harris6d`: F3's Harris6D branch (keypoints.h:164-176) over the same room with a
procedural colour texture: normals + intensity gradients + 6x6 response + the Harris3D tail.
`--workload config1`: configs[1], the 100k-point room (seed 1), NormalEstimation (r 0.05) + FPFH
(r 0.05) at EVERY point (input == surface: PCL's all-points SPFH branch).
`--workload dense`: SURVEY 8(d)'s "dense" data point, the configs[2] pass on the same room scene
at 10x the point density (10M points, k(0.05) ~ 2,400).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fpfh|shot|...] [--scans S]
                    [--no-cpu-baseline] [--no-e2e]
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
DENSE_POINTS = 10_000_000  # SURVEY 8(d) dense variant: configs[2]'s scene at 10x density
SHOT_SAMPLE = 10_000
CYCLE_SEEDS = [2, 100, 101, 102]  # the headline's distinct scans: configs[2]'s seed first

VERBOSE_TIMERS = ["narf", "grid_bbox", "grid_build", "normals", "normals_fast", "normals_mfma", "normals_lists_phase", "normals_tiles", "normals_lists",
                  "normals_lists_small", "normals_lists_sparse",
                  "normals_lists_dense", "normals_lists_wide", "normals_lists_query", "normals_chain", "normals_chain_big", "normals_long", "range_image",
                  "narf_border", "narf_interest", "narf_nms", "narf_gather", "fpfh_mark", "fpfh_spfh",
                  "fpfh_support", "fpfh_weight", "shot"]
VERBOSE_STATS = ["normals_neighbors", "normals_queries", "normals_tiles_sparse", "normals_tiles_dense",
                 "normals_single", "normals_wide", "normals_huge", "normals_long_lists", "normals_chain_wg_staged",
                 "normals_chain_wg_table", "normals_chain_wg_lane", "normals_chain_wg_deferred", "fpfh_spfh_points", "fpfh_spfh_pairs", "fpfh_spfh_exact_pairs", "narf_candidates", "narf_keypoints",
                 "narf_interest_fullimage", "narf_interest_grown", "narf_interest_window_px",
                 "narf_interest_visits", "narf_interest_queue_grown", "fpfh_weight_kmax", "fpfh_weight_sequential",
                 "shot_neighbors"]


def host_info():
    """CPU model, logical CPUs of the machine and of this process's affinity mask."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"cpu_model": model, "nproc": os.cpu_count() or 1, "affinity_cpus": affinity}


def _cpu_timed_runs(x, y, z, workload, sample, reps, threads):
    """The timed CPU-restatement runs (in the pinned child process, see cpu_baseline)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O

    def once(cx, cy, cz, samp):
        t0 = time.perf_counter()
        kp = O.narf_keypoints(cx, cy, cz, threads=1)
        t1 = time.perf_counter()
        nx, ny, nz, _ = O.normals(cx, cy, cz, 0.05, threads=threads)
        t2 = time.perf_counter()
        rows = kp[kp < len(cx)]
        if workload == "fpfh":
            desc = O.fpfh(cx, cy, cz, nx, ny, nz, cx[rows], cy[rows], cz[rows], 0.08, threads=1)
        else:
            rows = np.r_[rows, samp]
            desc = O.shot(cx, cy, cz, nx, ny, nz, cx[rows], cy[rows], cz[rows], 0.08, threads=threads)
        t3 = time.perf_counter()
        return (t1 - t0, t2 - t1, t3 - t2), (kp, (nx, ny, nz), desc), len(rows)

    sub = slice(None, None, 10)
    once(x[sub], y[sub], z[sub], None if sample is None else sample[sample < len(x[sub])])
    times, outputs, nrows = [], None, 0
    for _ in range(reps):
        t, outputs, nrows = once(x, y, z, sample)
        times.append(t)
    # BASELINE.md's all-single-threaded figure: the normal estimation once more on one thread
    # (NARF and FPFH already run on one); one run, not a median (~35-60 s)
    single_normals = -1.0
    if workload == "fpfh" and os.environ.get("PFX_CPU_SINGLE", "1") != "0":
        t0 = time.perf_counter()
        O.normals(x, y, z, 0.05, threads=1)
        single_normals = time.perf_counter() - t0
    return times, outputs, nrows, single_normals


def cpu_child(path):
    """`bench.py --cpu-child <npz>`: the timed runs in a process of their own (no torch, no GPU),
    its OpenMP threads pinned one per core (OMP_PROC_BIND=close, OMP_PLACES=cores, set by the
    parent before this process's OpenMP runtime starts) inside the first `threads` CPUs of the
    parent's affinity mask; results back through the same npz path (+ .out.npz)."""
    import numpy as np
    f = np.load(path, allow_pickle=False)
    threads = int(f["threads"])
    try:
        cpus = sorted(os.sched_getaffinity(0))[:threads]
        os.sched_setaffinity(0, cpus)
    except (AttributeError, OSError):
        cpus = []
    sample = f["sample"] if f["has_sample"] else None
    times, (kp, nrm, desc), nrows, single_normals = _cpu_timed_runs(f["x"], f["y"], f["z"], str(f["workload"]),
                                                                    sample, int(f["reps"]), threads)
    if isinstance(desc, tuple):
        desc = desc[0]
    np.savez(path + ".out.npz", times=np.asarray(times), kp=np.asarray(kp), nx=nrm[0], ny=nrm[1], nz=nrm[2],
             desc=np.asarray(desc), nrows=nrows, cpus=np.asarray(cpus, np.int64), single_normals=single_normals)


def cpu_baseline(x, y, z, workload, sample=None, reps=5):
    """The CPU restatement (oracle/, test infrastructure) on the same scan, threads as PCL:
    NARF and FPFH single-threaded (PCL 1.7 defaults, non-OMP FPFHEstimation), normals and SHOT
    OpenMP (NormalEstimationOMP / SHOTEstimationOMP) over OMP_NUM_THREADS -- the box's CPU share
    for one GPU (16 there; its nproc reports the whole host).  SURVEY 8(d): one warm-up run (on a
    1/10 subsample of the scan: pages the code and the allocator in) and the median of `reps`
    full runs of the first scan of the timed cycle.  The runs happen in a child process whose
    OpenMP threads are pinned one per core (unpinned threads spread 8.2-12.4 s over
    five runs); the line reports every run and the spread beside the median."""
    import subprocess
    import tempfile
    import numpy as np
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    with tempfile.TemporaryDirectory(prefix="pfx_cpu_") as td:
        path = os.path.join(td, "scan.npz")
        np.savez(path, x=x, y=y, z=z, workload=workload, reps=reps, threads=threads,
                 sample=np.zeros(0, np.int64) if sample is None else np.asarray(sample), has_sample=sample is not None)
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
        subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", path], env=env, check=True)
        r = np.load(path + ".out.npz", allow_pickle=False)
        times = [tuple(float(v) for v in t) for t in r["times"]]
        desc = r["desc"]
        outputs = (r["kp"], (r["nx"], r["ny"], r["nz"]), (desc,) if workload != "fpfh" else desc)
        nrows, cpus = int(r["nrows"]), [int(c) for c in r["cpus"]]
        single_normals = float(r["single_normals"]) if "single_normals" in r.files else -1.0
    tot = [sum(t) for t in times]
    order = sorted(range(len(tot)), key=lambda i: tot[i])
    mid = order[len(order) // 2]  # the median run (reps odd)
    med = tot[mid]
    stage_med = list(times[mid])
    feat = "FPFH 1 thread" if workload == "fpfh" else f"SHOT {threads} threads"
    single = None
    if single_normals > 0:  # NARF and FPFH of the median run (one thread each) + normals on one thread
        secs = stage_med[0] + single_normals + stage_med[2]
        single = {"value": round(len(x) / secs / 1e6, 6), "unit": "Mpoints/s", "cores": 1, "seconds": round(secs, 3),
                  "normals_1_thread_s": round(single_normals, 3),
                  "note": "BASELINE.md's all-single-threaded figure: NARF + FPFH of the median run (one thread each) "
                          "+ one single-threaded run of the normal estimation on the same scan"}
    return dict(seconds=med, threads=threads, outputs=outputs, runs=[round(v, 3) for v in sorted(tot)], single=single,
                stages_s={"narf": round(stage_med[0], 3), "normals": round(stage_med[1], 3),
                          "features": round(stage_med[2], 3)},
                spread=round((max(tot) - min(tot)) / med, 4),
                pinning={"OMP_PROC_BIND": "close", "OMP_PLACES": "cores", "cpus": cpus},
                sample=(f"the first 1M-point scan of the timed cycle through the CPU restatement (oracle/), 1 warm-up "
                        f"(1/10 subsample) + median of {reps} full runs in a child process with pinned OpenMP threads: "
                        f"NARF 1 thread {stage_med[0]:.2f}s, normals {threads} threads "
                        f"{stage_med[1]:.2f}s, {feat} {stage_med[2]:.2f}s at {nrows} rows; real PCL is not available "
                        f"anywhere in this pipeline"))


def oracle_outputs(x, y, z):
    """The CPU restatement's keypoints, normals and FPFH rows of one scan (all threads, untimed):
    the checker for the cycle's other scans."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    kp = O.narf_keypoints(x, y, z, threads=threads)
    nx, ny, nz, _ = O.normals(x, y, z, 0.05, threads=threads)
    rows = kp[kp < len(x)]
    desc = O.fpfh(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08, threads=threads)
    return kp, (nx, ny, nz), desc


def full_size_parity(outputs, kp, b, desc, rows, shot, normals_mask=None):
    """The last timed step's outputs against the CPU restatement's on the whole scan: bit-exact
    (NaN positions equal) for keypoints, normals and descriptor rows (normals_mask: the normals
    compared only where it is set -- the demand-driven mode estimates no others)."""
    import numpy as np
    okp, onorm, odesc = outputs
    if shot:
        odesc = odesc[0]
    sel = slice(None) if normals_mask is None else np.asarray(normals_mask) != 0

    def same(a, c):  # raw bits, NaN rows included (PCL's quiet_NaN on both sides)
        a, c = np.ascontiguousarray(np.asarray(a, np.float32)), np.ascontiguousarray(np.asarray(c, np.float32))
        return bool(a.shape == c.shape and np.array_equal(a.view(np.uint32), c.view(np.uint32)))
    res = {"normals": all(same(t.cpu().numpy()[sel], o[sel]) for t, o in zip((b.nx, b.ny, b.nz), onorm)),
           "descriptors": same(desc[:rows].cpu().numpy(), odesc)}
    if kp is not None:
        res["keypoints"] = bool(np.array_equal(np.asarray(kp), okp))
    return res


def libpfx_sha16():
    import hashlib
    path = os.path.join(ROOT, "pcl_feature_extraction_amd", "libpfx.so")
    return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16] if os.path.exists(path) else None


def load_pmc(name):
    """Committed PMC summary (scripts/gpu_pmc.sh -> scripts/pmc_summary.py), or None; with
    `same_build` = whether it was collected on the libpfx.so this run loads."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    d["same_build"] = d.get("libpfx_sha16") is not None and d.get("libpfx_sha16") == libpfx_sha16()
    return d


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-child":  # (cpu_baseline's pinned child: no torch)
        cpu_child(sys.argv[2])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["fpfh", "shot", "match", "iss", "harris", "harris6d", "config1", "dense",
                                           "fastnormals", "demand"],
                    default="fpfh")
    ap.add_argument("--scans", type=int, default=0,
                    help="fpfh workload: scans per step (default 1 = configs[2] at --gpus 1, 8 = configs[4] at N > 1)")
    ap.add_argument("--cycle", type=int, default=4,
                    help="headline (fpfh, one scan per step at --gpus 1): distinct 1M-pt room scans cycled through "
                         "the timed steps (seeds 2, 100, 101, 102), each checked at full size against the oracle")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (H2D/D2H inside the step) leg")
    args = ap.parse_args()

    # driver-style `bench.py --gpus N` without an external launcher: start the N ranks as a child
    # torch.distributed.run BEFORE anything here touches a GPU, and exit with its code
    from pcl_feature_extraction_amd import launch
    if launch.needs_spawn(args.gpus):
        sys.exit(launch.spawn(args.gpus, os.path.abspath(__file__), sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    try:
        if args.workload == "match":
            return bench_match(args, torch, dev, world, rank, local)
        if args.workload == "iss":
            return bench_iss(args, torch, dev, world, rank, local)
        if args.workload in ("harris", "harris6d"):
            return bench_harris(args, torch, dev, world, rank, local, six=args.workload == "harris6d")
        if args.workload == "config1":
            return bench_config1(args, torch, dev, world, rank, local)
        return bench_scans(args, torch, dist, dev, world, rank, local)
    finally:
        if world > 1:
            dist.destroy_process_group()


def timed(torch, dist, dev, world, steps, fn):
    """Barrier + synchronize on both sides of exactly `steps` calls; max over ranks (seconds)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def bench_scans(args, torch, dist, dev, world, rank, local):
    """The headline (fpfh) and the configs[3] (shot) workloads.

    fpfh: a step = every scan of the batch through Keypoints("Narf") + Features<FPFH> on the rank
    that owns it (scans dealt round-robin, dist.owned_scans), then the gather of every scan's
    K_s x 33 descriptors + K_s cloud indices to rank 0 (dist.gather_to_root: RCCL grouped
    send/recv).  --gpus 1: one scan (configs[2], seed 2).  N > 1: configs[4], the fixed batch of
    8 scans (seeds 100..107), 8/N per GPU -- total work fixed, so "scaling": "strong".
    shot: configs[3], one seabed scan per rank (replicas)."""
    import numpy as np

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.dist import gather_to_root, in_scan_order, owned_scans
    from pcl_feature_extraction_amd.pipeline import (BatchNarfFpfh, DeviceRows, OverlappedNarfFpfh, alloc,
                                                     alloc_shot, narf_shot)
    from pcl_feature_extraction_amd.synth import ROOM_SCALE, synth_room, synth_seabed

    shot = args.workload == "shot"
    dense = args.workload == "dense"
    fast = args.workload == "fastnormals"
    # opt-in: normals estimated only where FPFH reads them (same keypoints and descriptors)
    demand = args.workload == "demand"
    npts = DENSE_POINTS if dense else N_POINTS
    if shot:
        n_scans, seeds = world, [3] if world == 1 else [300 + r for r in range(world)]
    else:
        n_scans = args.scans or (1 if world == 1 else 8)
        seeds = [2] if (n_scans == 1 and world == 1) else [100 + i for i in range(n_scans)]
    mine = owned_scans(n_scans, world, rank)
    # the headline cycles distinct scans (step k processes scan k mod C), so no previous-call hint
    # (speculative grid bounds, the FPFH grid built on the previous scan's bounds, list-tier hints,
    # grow-only buffers) is ever primed by the identical scan
    cycle = max(1, args.cycle) if (n_scans == 1 and world == 1 and args.workload == "fpfh") else 1
    if cycle > 1:
        seeds = CYCLE_SEEDS[:cycle]
        mine = list(range(len(seeds)))
        cycle = len(mine)
    per_rank_max = -(-n_scans // world)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx_n = Context(local)  # normal estimation overlapped with NARF on a second stream
    run_fpfh = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
    run_fpfh.fast_normals = fast
    if demand:
        run_fpfh.support_first = 1
        run_fpfh.normals_scope = "support"
    # several scans on this rank (configs[4] at N < 8): the software-pipelined batch pass (scan
    # i's FPFH and scan i+1's NARF under scan i+1's normal estimation); one scan: the overlapped pass
    run_batch = (BatchNarfFpfh(torch, ctx, ctx_n, dev, side_stream=run_fpfh.s_side)
                 if (len(mine) > 1 and not shot and cycle == 1) else None)
    scans, host = [], []
    for s in mine:
        if dense:  # the configs[2] scene (same scale s) at 10x the density
            x, y, z, _ = synth_room(npts, seeds[s], scale=ROOM_SCALE * (N_POINTS / npts) ** 0.5)
        else:
            x, y, z, _ = (synth_seabed if shot else synth_room)(npts, seeds[s])
        b = alloc(torch, npts, dev)
        for t, a in zip((b.x, b.y, b.z), (x, y, z)):
            t.copy_(torch.from_numpy(a))
        scans.append(b)
        host.append((x, y, z))
    sample_np = np.sort(np.random.default_rng(10).choice(N_POINTS, SHOT_SAMPLE, replace=False))
    if shot:
        sb = alloc_shot(torch, 1 << 16, dev)
        sample = torch.from_numpy(sample_np.astype(np.int64)).to(dev)
    state = {"kp": None, "rows": 0, "gathered": None, "i": 0, "kp_by": {}, "rows_by": {}}
    # descriptor rows' cloud indices to the device through pinned blocks (async: a pageable copy
    # would hold the host until the scan's FPFH had finished, idling the device between steps)
    dev_rows = DeviceRows(torch, dev, slots=2 * max(1, len(mine)))

    def one_scan(b, j=0):
        if shot:
            rows = run_fpfh.shot(b, sb, sample)  # (NARF || normals, then SHOT: as the headline's overlap)
            return sb.desc[:rows], None
        kp, k = run_fpfh(b)
        state["kp"] = kp
        state["kp_by"][j], state["rows_by"][j] = kp, k
        return b.desc[:k], dev_rows(kp, npts)

    def batch_scans():
        blocks = []
        for b, (kp, k) in zip(scans, run_batch(scans)):
            state["kp"] = kp
            blocks.append((b.desc[:k], dev_rows(kp, npts)))
        return blocks

    def step():
        if cycle > 1:  # one scan per step, the next of the cycle
            j = state["i"] % cycle
            state["i"] += 1
            blocks = [one_scan(scans[j], j)]
        else:
            blocks = batch_scans() if run_batch is not None else [one_scan(b, j) for j, b in enumerate(scans)]
        state["rows"] = int(blocks[-1][0].shape[0]) if blocks else 0
        if world > 1 and not shot:
            state["gathered"] = gather_to_root(torch, dist, blocks, 33, dev, per_rank_max)
        return blocks

    # warm-up; per-scan neighbour counts of the normal estimation (for the algorithmic bytes)
    nb_scan, long_scan = [], []
    for w in range(max(args.warmup, 1)):
        blocks = []
        if w == 0 or run_batch is None:
            for j, b in enumerate(scans):
                # the neighbour count of the scan, from one exact estimation (the fast mode has no
                # lists; the support-first schedule's statistics cover its last subset only)
                if w == 0 and (fast or (run_fpfh.support_first and not demand)):
                    ctx_n.normals_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
                    nb_scan.append(ctx_n.stat("normals_neighbors"))
                    long_scan.append((ctx_n.stat("normals_long_neighbors"), ctx_n.stat("normals_long_queries")))
                blocks.append(one_scan(b, j))
                if w == 0 and not fast and (demand or not run_fpfh.support_first):
                    c = ctx_n  # (the normal estimation runs on the side context in both passes)
                    nb_scan.append(c.stat("normals_neighbors"))
                    long_scan.append((c.stat("normals_long_neighbors"), c.stat("normals_long_queries")))
        else:
            blocks = batch_scans()
        if world > 1 and not shot:
            gather_to_root(torch, dist, blocks, 33, dev, per_rank_max)
    torch.cuda.synchronize(dev)
    # the same scans back to back through the single-scan overlapped pass (no cross-scan
    # pipelining), for the batch pipeline's gain; not part of `value`
    seq_ms = None
    if run_batch is not None and rank == 0:
        seq_el = timed(torch, dist, dev, 1, max(1, args.steps // 4), lambda: [one_scan(b) for b in scans])
        seq_ms = seq_el / max(1, args.steps // 4) * 1e3
    # inside the timed region only the stage timers run (one HIP-event pair per stage call: the
    # roofline's live time); the per-kernel pairs cost ~0.14 ms of host launch time per step
    # (172.1 vs 168.1 Mpoints/s), so the per-kernel breakdown comes from extra steps afterwards
    def read_timers():
        return {nm: (ctx.kernel_time(nm)[0] + ctx_n.kernel_time(nm)[0],
                     ctx.kernel_time(nm)[1] + ctx_n.kernel_time(nm)[1]) for nm in VERBOSE_TIMERS}

    for c in (ctx, ctx_n):
        c.set_timing(True, stages_only=True)
        c.reset_timing()
    elapsed = timed(torch, dist, dev, world, args.steps, step)
    # deferred errors of the stream-ordered calls (FPFH capacity), outside the timed region
    (run_batch or run_fpfh).check()
    timers = read_timers()
    detail_steps = max(3, args.steps // 4)
    for c in (ctx, ctx_n):
        c.set_timing(True)
        c.reset_timing()
    timed(torch, dist, dev, world, detail_steps, step)
    detail = read_timers()
    for c in (ctx, ctx_n):
        c.set_timing(False)

    def stat(nm):
        for c in (ctx_n, ctx) if nm.startswith("normals") else (ctx, ctx_n):
            try:
                return c.stat(nm)
            except Exception:
                pass
        raise KeyError(nm)

    if os.environ.get("PFX_BENCH_VERBOSE"):
        rep = {nm: round(ms / detail_steps, 3) for nm, (ms, _) in detail.items() if ms > 0}
        print("per-step kernel ms:", json.dumps(rep), file=sys.stderr, flush=True)
        stats = {}
        for nm in VERBOSE_STATS:
            try:
                stats[nm] = stat(nm)
            except Exception:
                pass
        print("stats:", json.dumps(stats), file=sys.stderr, flush=True)

    # gathered batch on rank 0: scan order, sizes (the descriptors themselves stay on the device)
    batch = None
    if world > 1 and not shot and rank == 0:
        ordered = in_scan_order(state["gathered"], n_scans, world)
        batch = {"scans": n_scans, "rows_per_scan": [int(d.shape[0]) for d, _ in ordered],
                 "matrix_rows": int(sum(d.shape[0] for d, _ in ordered)),
                 "finite": bool(all(torch.isfinite(d).all().item() for d, _ in ordered if d.numel()))}

    # the resident outputs of every scan of the cycle, for the full-size parity check at the end
    resident = {j: (state["kp_by"][j], state["rows_by"][j]) for j in state["kp_by"]}

    # the host-buffer leg (SURVEY 8(d) "H2D/D2H included"): each scan's xyz copied from pinned
    # host memory inside the step, descriptors + indices copied back; reported beside `value`
    e2e = None
    if not args.no_e2e and not shot and cycle > 1:
        e2e = bench_e2e_pipelined(torch, dist, dev, world, args.steps, host, cycle, npts, one_scan, alloc)
    elif not args.no_e2e and not shot:
        hx = [[torch.from_numpy(a).pin_memory() for a in h] for h in host]
        hd = [torch.empty((1 << 16, 33), dtype=torch.float32).pin_memory() for _ in scans]
        hi = [torch.empty((1 << 16,), dtype=torch.int32).pin_memory() for _ in scans]

        def step_e2e():
            blocks = []
            for j, b in enumerate(scans):
                for t, a in zip((b.x, b.y, b.z), hx[j]):
                    t.copy_(a, non_blocking=True)
                d, i = one_scan(b)
                k = int(d.shape[0])
                hd[j][:k].copy_(d, non_blocking=True)
                hi[j][:k].copy_(i, non_blocking=True)
                blocks.append((d, i))
            if world > 1:
                gather_to_root(torch, dist, blocks, 33, dev, per_rank_max)
        step_e2e()
        e_el = timed(torch, dist, dev, world, args.steps, step_e2e)
        e2e = {"value": round(n_scans * npts * args.steps / e_el / 1e6, 4), "unit": "Mpoints/s",
               "ms_per_step": round(e_el / args.steps * 1e3, 4),
               "note": ("host-pointer semantics: per scan 12 MB xyz H2D from pinned memory + K x 33 descriptors and "
                        "K indices D2H inside the timed step (SURVEY 8(d) definition); `value` is the same step with "
                        "the scan already resident in HBM")}

    # the same normal-estimation stage alone on the device (after the timed region, not part of
    # `value`): inside the step it shares the CUs with NARF on the other stream
    iso = None
    deviation = None
    if rank == 0 and fast:  # the fast mode against the product (parity-exact) path on the same scan
        b = scans[0]
        fast_n = [t.clone() for t in (b.nx, b.ny, b.nz, b.curv)]
        fast_d = b.desc[:state["rows"]].clone()
        run_fpfh.fast_normals = False
        kp_exact, k_exact = run_fpfh(b)
        torch.cuda.synchronize(dev)
        deviation = fast_deviation(torch, fast_n, fast_d, b, k_exact, np.array_equal(np.asarray(kp_exact),
                                                                                     np.asarray(state["kp"])))
        run_fpfh.fast_normals = True
    if rank == 0 and not shot and not demand:  # (demand: the full estimation would overwrite the checked normals)
        b = scans[0]
        ctx_n.set_timing(True)
        ctx_n.reset_timing()
        for _ in range(3):
            (ctx_n.normals_fast_dev if fast else ctx_n.normals_dev)(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
        torch.cuda.synchronize(dev)
        iso = {nm: ctx_n.kernel_time(nm)[0] / 3 for nm in VERBOSE_TIMERS}
        ctx_n.set_timing(False)

    if rank == 0:
        line = scans_line(args, world, n_scans, 1 if cycle > 1 else len(mine), shot, elapsed, timers, iso, nb_scan,
                          long_scan, stat, npts,
                          fast=fast, detail=detail, detail_steps=detail_steps, demand=demand)
        if deviation is not None:
            line["deviation_from_parity_path"] = deviation
        if cycle > 1:
            line["config"]["scan_cycle"] = {
                "seeds": CYCLE_SEEDS[:cycle], "scans": cycle,
                "note": (f"step k processes scan k mod {cycle} (synth_room 1M points, distinct seeds; configs[2] is seed "
                         f"2): no previous-call hint is primed by an identical scan"),
                "keypoints_per_scan": [int(len(resident[j][0])) for j in range(cycle)],
                "descriptor_rows_per_scan": [int(resident[j][1]) for j in range(cycle)]}
        line["config"]["descriptor_rows"] = state["rows"]
        if seq_ms is not None:
            line["batch_pipeline"] = {
                "scans_on_rank0": len(mine), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "back_to_back_ms_per_step": round(seq_ms, 4),
                "speedup": round(seq_ms / (elapsed / args.steps * 1e3), 4),
                "note": "BatchNarfFpfh (scan i's FPFH and scan i+1's NARF under scan i+1's normals) vs the same "
                        "scans through the single-scan overlapped pass back to back (rank 0 alone)"}
        if batch is not None:
            line["config"]["gathered_on_rank0"] = batch
            line["config"]["ranks_seen_by_rccl"] = dist.get_world_size()
            line["config"]["backend"] = dist.get_backend()
        line["end_to_end_h2d_d2h"] = e2e
        cpu = None
        if fast:
            cpu = {"value": None, "note": "see the configs[2] line: the CPU restatement is PCL's path, which this "
                                          "opt-in mode departs from by design"}
        elif world == 1 and not args.no_cpu_baseline and not dense:
            x, y, z = host[0]
            kp0, rows0 = resident[0] if cycle > 1 else (state["kp"], state["rows"])
            cb = cpu_baseline(x, y, z, "fpfh" if demand else args.workload, sample_np)
            cpu = {"value": round(npts / cb["seconds"] / 1e6, 6), "unit": "Mpoints/s",
                   "cores": cb["threads"], "kind": "port", "sample": cb["sample"], "runs_s": cb["runs"],
                   "stages_s": cb["stages_s"], "all_single_threaded": cb["single"],
                   "cores_note": ("OMP_NUM_THREADS = the box's CPU share for one GPU (16; nproc reports the whole "
                                  "host, shared by its eight GPUs' jobs): BASELINE.md's 'all host cores' for the OpenMP "
                                  "legs of a one-GPU job"),
                   "spread": cb["spread"], "pinning": cb["pinning"],
                   **host_info(),
                   "parity": full_size_parity(cb["outputs"], kp0, scans[0], sb.desc if shot else scans[0].desc, rows0,
                                              shot,
                                              normals_mask=run_fpfh._support[:npts].cpu().numpy() if demand else None)}
            if cycle > 1:  # every other scan of the timed cycle at full size (the oracle, all threads, untimed)
                cpu["parity_cycle"] = []
                for j in range(1, cycle):
                    hx_, hy_, hz_ = host[j]
                    cpu["parity_cycle"].append({"seed": CYCLE_SEEDS[j], **full_size_parity(
                        oracle_outputs(hx_, hy_, hz_), resident[j][0], scans[j], scans[j].desc, resident[j][1], False)})
                line["parity_all_scans"] = all(all(v for k, v in d.items() if k != "seed")
                                               for d in [cpu["parity"]] + cpu["parity_cycle"])
                line["parity_all_scans_note"] = (
                    "bit-exact against the CPU restatement (oracle/), itself unpinned against real PCL (absent). "
                    "The keypoints of these four rooms depend on std::sort's tie order in NarfKeypoint's greedy "
                    "selection: 6/6/11/9 tied NMS survivor pairs closer than 0.05 m, and 4/7/4/6 of their 83-89 "
                    "keypoints move between the two extreme tie orders (profiles/r05_narf_tie_report.jsonl). The GPU "
                    "path and the oracle sort with this build's libstdc++ and agree; a PCL built with another "
                    "standard library may order those ties differently. The reference's own four clouds have no ties.")
            if demand:
                cpu["note"] = ("the reference's CPU path (every normal, as PCL computes them): the descriptors and "
                               "keypoints are the outputs compared; normals compared on the support only")
        if dense:
            cpu = {"value": None, "note": "not run: the CPU restatement needs ~10 min per pass at this density "
                                          "(normals ~24.6G neighbour terms); see the configs[2] line"}
        line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    run_fpfh.close()
    if run_batch is not None:
        run_batch.close()
    ctx.close()
    ctx_n.close()


def bench_e2e_pipelined(torch, dist, dev, world, steps, host, cycle, npts, one_scan, alloc):
    """The headline with host buffers (H2D of the scan and D2H of the descriptors
    inside the timed region), as a stream of scans arriving in pinned host memory: scan k+1's
    12 MB of xyz goes to the other of two device slots on a copy stream (the DMA engine) while
    scan k computes; scan k waits only for its own copy.  Every H2D and D2H of the `steps` scans
    is inside the timed region (the first copy is not overlapped)."""
    hx = [[torch.from_numpy(a).pin_memory() for a in h] for h in host]
    slots = [alloc(torch, npts, dev) for _ in range(2)]
    hd = [torch.empty((1 << 16, 33), dtype=torch.float32).pin_memory() for _ in range(2)]
    hi = [torch.empty((1 << 16,), dtype=torch.int32).pin_memory() for _ in range(2)]
    cs = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)

    def run(n):
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        free = [None, None]

        def h2d(k):
            s = k % 2
            with torch.cuda.stream(cs):
                if free[s] is not None:  # the slot's previous scan has finished reading it
                    cs.wait_event(free[s])
                for t, a in zip((slots[s].x, slots[s].y, slots[s].z), hx[k % cycle]):
                    t.copy_(a, non_blocking=True)
                ready[s].record(cs)
        h2d(0)
        for k in range(n):
            s = k % 2
            main.wait_event(ready[s])
            if k + 1 < n:
                h2d(k + 1)
            d, i = one_scan(slots[s], k % cycle)
            m = int(d.shape[0])
            hd[s][:m].copy_(d, non_blocking=True)
            hi[s][:m].copy_(i, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(main)
            free[s] = ev
    run(2 * cycle)  # warm-up (pins the slots' grids and lists)
    el = timed(torch, dist, dev, world, 1, lambda: run(steps))
    return {"value": round(npts * steps / el / 1e6, 4), "unit": "Mpoints/s", "ms_per_step": round(el / steps * 1e3, 4),
            "note": (f"host-pointer semantics (SURVEY 8(d) definition): the same {cycle}-scan cycle arriving in pinned "
                     f"host memory -- per scan 12 MB xyz H2D (copy stream, double-buffered device slots: scan k+1's copy "
                     f"overlaps scan k's compute) and K x 33 descriptors + K indices D2H, all inside the timed region; "
                     f"`value` is the same stream with the scans already resident in HBM")}


def fast_deviation(torch, fast_n, fast_d, b, k, same_kp):
    """Opt-in MFMA normals vs the parity-exact path on one scan: normal angles (deg), curvature,
    and the FPFH rows at the same keypoints (absolute L2 and L2 relative to the row norm)."""
    import numpy as np
    F = torch.stack(fast_n[:3], 1).double().cpu().numpy()
    P = torch.stack((b.nx, b.ny, b.nz), 1).double().cpu().numpy()
    ok = np.isfinite(P[:, 0]) & np.isfinite(F[:, 0])
    ang = np.degrees(np.arccos(np.clip(np.abs(np.sum(F[ok] * P[ok], 1)), 0.0, 1.0)))
    out = {"normals_compared": int(ok.sum()),
           "nan_pattern_equal": bool(np.array_equal(np.isnan(F[:, 0]), np.isnan(P[:, 0]))),
           "angle_deg": {"p50": round(float(np.median(ang)), 5), "p99": round(float(np.percentile(ang, 99)), 4),
                         "max": round(float(ang.max()), 3)},
           "same_keypoints": bool(same_kp)}
    if same_kp and k == fast_d.shape[0] and k > 0:
        D = fast_d.double().cpu().numpy()
        E = b.desc[:k].double().cpu().numpy()
        fin = np.isfinite(D).all(1) & np.isfinite(E).all(1)
        l2 = np.linalg.norm(D[fin] - E[fin], axis=1)
        rel = l2 / np.maximum(np.linalg.norm(E[fin], axis=1), 1e-30)
        out["fpfh_rows"] = int(fin.sum())
        out["fpfh_l2"] = {"p50": round(float(np.median(l2)), 4), "max": round(float(l2.max()), 4)}
        out["fpfh_l2_rel"] = {"p50": round(float(np.median(rel)), 5), "max": round(float(rel.max()), 5)}
    return out


def scans_line(args, world, n_scans, scans_here, shot, elapsed, timers, iso, nb_scan, long_scan, stat, npts=N_POINTS,
               fast=False, detail=None, detail_steps=1, demand=False):
    """The contract line of bench_scans (rank 0), roofline over the neighbour-gather stage."""
    per_scan_calls = args.steps * scans_here  # scans this rank processes per step
    ms_per_step = elapsed / args.steps * 1e3
    value = n_scans * npts * args.steps / elapsed / 1e6
    nb = sum(nb_scan) / len(nb_scan)
    long_nb = sum(l[0] for l in long_scan) / len(long_scan)
    long_q = sum(l[1] for l in long_scan) / len(long_scan)
    # neighbour-gather bytes per scan = sum_q |N_0.05(q)| x 12 B + N x 16 B, over
    # the WHOLE stage that produces them: grid build + FLANN-ordered list builders + ordered
    # covariance chains + long lists (timer "normals": HIP events around pfx_normals_dev on its
    # stream, inside the timed step, averaged per scan)
    # (demand: the support's queries only -- the stage estimates no other normal)
    algo = nb * 12 + (stat("normals_queries") if demand else npts) * 16
    stage_ms = timers["normals_fast" if fast else "normals"][0] / max(per_scan_calls, 1)
    stage_gbs = algo / (stage_ms / 1e3) / 1e9 if stage_ms > 0 else 0.0
    parts = ("grid_bbox", "grid_build", "normals_lists_small", "normals_lists_sparse", "normals_lists_dense",
             "normals_lists_wide", "normals_lists_query", "normals_chain", "normals_chain_big", "normals_long")
    # per-kernel breakdown: extra steps with every kernel timer on (after the timed region)
    detail_calls = max(detail_steps * scans_here, 1)
    kernels = {nm: round(detail[nm][0] / detail_calls, 4) for nm in parts}
    chain_algo = (nb - long_nb) * 12 + (npts - long_q) * 16
    chain_ms = kernels["normals_chain"] + kernels["normals_chain_big"]
    chain = {"kernel": "k_normals_chain + k_normals_chain_big",
             "algorithmic_bytes_per_launch": int(chain_algo), "ms": chain_ms,
             "achieved": round(chain_algo / (chain_ms / 1e3) / 1e9, 2) if chain_ms > 0 else None}
    chain["frac"] = round(chain["achieved"] / HBM_PEAK_GBS, 5) if chain["achieved"] else None
    if chain["frac"] and chain["frac"] > 1:
        chain["note"] = ("above 1: the chains read each neighbour from the LDS-staged cell that many queries share, "
                         "so the algorithmic gather bytes exceed what HBM delivers -- these neighbourhoods are not "
                         "HBM-bound (the configs[2] line is the HBM-roofline case)")
    # the committed PMC summary was collected on configs[2]'s scan: only that line may cite it
    pmc = (load_pmc("pmc_normals_stage.json") or {}) if (npts == N_POINTS and not fast) else {}
    roofline = {"bound": "hbm", "kernel": "normals stage: grid + k_nb_tile/k_nb_query list builders + "
                                          "k_normals_chain(_big) + k_normals_long",
                "achieved": round(stage_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(stage_gbs / HBM_PEAK_GBS, 5), "traffic": pmc.get("stage_hbm_bytes_per_launch"),
                "algorithmic_bytes_per_launch": int(algo), "avg_ms": round(stage_ms, 4),
                "neighbors_per_launch": int(nb),
                "basis": "HIP events on the normal-estimation stream over the timed region, per scan (concurrent "
                         "with NARF on the other stream); kernels_ms_per_scan from extra steps with per-kernel "
                         "events (not in the timed region)",
                "kernels_ms_per_scan": kernels, "chain": chain,
                "pmc": pmc.get("kernels"),
                "traffic_source": ({"file": "profiles/pmc_normals_stage.json", "libpfx_sha16": pmc.get("libpfx_sha16"),
                                    "same_build_as_this_run": pmc.get("same_build")} if pmc else None)}
    if fast:  # the opt-in MFMA-covariance stage: grid build + k_normals_mfma (no lists)
        mf = timers["normals_mfma"][0] / max(per_scan_calls, 1)  # a stage timer: live in the timed region
        roofline.update({"kernel": "normals_fast stage: grid + k_normals_mfma (16x16x4 f32 MFMA: hit mask x "
                                   "centred candidate features; no neighbour list, not parity-exact)",
                         "kernels_ms_per_scan": {"grid_bbox": kernels["grid_bbox"], "grid_build": kernels["grid_build"],
                                                 "normals_mfma": round(mf, 4)},
                         "chain": None, "pmc": None, "traffic": None})
        roofline["mfma_kernel"] = {"kernel": "k_normals_mfma", "ms": round(mf, 4),
                                   "achieved": round(algo / (mf / 1e3) / 1e9, 2) if mf > 0 else None,
                                   "frac": round(algo / (mf / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if mf > 0 else None}
    if iso is not None:
        iso_stage = iso["normals_fast" if fast else "normals"]
        roofline["isolated"] = {"avg_ms": round(iso_stage, 4),
                                "achieved": round(algo / (iso_stage / 1e3) / 1e9, 2) if iso_stage > 0 else None,
                                "frac": round(algo / (iso_stage / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if iso_stage > 0 else None,
                                "kernels_ms": {nm: round(iso[nm], 4) for nm in (("grid_bbox", "grid_build",
                                                                                 "normals_mfma") if fast else parts)},
                                "note": "pfx_normals_dev alone on the device after the timed region (not `value`)"}
    if shot:  # configs[3]: k_shot heads the line (the dominant kernel of that step)
        shot_ms, shot_n = timers["shot"]
        shot_s = (shot_ms / max(shot_n, 1)) / 1e3
        sbytes = stat("shot_neighbors") * 24
        shot_gbs = sbytes / shot_s / 1e9 if shot_s > 0 else 0.0
        stage = roofline
        stage.pop("bound")
        roofline = {"bound": "hbm", "kernel": "SHOT stage: k_shot_ipos + k_shot_prep + k_shot_lrf + k_shot_eigen + "
                                              "k_shot_frame + k_shot_accum (+ k_shot<16384> for lists over 2,048)",
                    "achieved": round(shot_gbs, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(shot_gbs / HBM_PEAK_GBS, 5), "traffic": None,
                    "algorithmic_bytes_per_launch": int(sbytes), "avg_ms": round(shot_s * 1e3, 4),
                    "note": "sum_q |N_0.08(q)| x 24 B (xyz + normal) per launch (SURVEY 8(d)); VALU/LDS-atomic "
                            "bound, not HBM", "normals_stage": stage}
        metric = "Mpoints/s through NARF keypoint + normals + SHOT-352 descriptor on 1M-pt underwater-style cloud"
        workload = (f"configs[3] 1M-pt synthetic seabed, NARF(support 0.2) + normals(r 0.05) + SHOT-352(r 0.08) at "
                    f"the keypoints + a fixed {SHOT_SAMPLE}-point sample" + ("" if world == 1 else ", one scan per GPU"))
        data = "synthetic (synth_seabed: seeded fBm height field under a pinhole camera, k(0.08)~1000)"
        scaling = "weak"
    else:
        metric = "Mpoints/s through NARF keypoint + FPFH descriptor on 1M-pt cloud"
        if n_scans == 1 and demand:
            workload = ("configs[2] 1M-pt synthetic room, NARF(support 0.2) + FPFH(r 0.08) at the keypoints, normals "
                        "(r 0.05) estimated only on the FPFH support (every point within 0.16 of a keypoint: a "
                        "superset of the normals FPFHEstimation reads) -- same keypoints and descriptors; opt-in, "
                        "not the contract line")
        elif n_scans == 1:
            workload = ("configs[2] 1M-pt synthetic room, NARF(support 0.2) + normals(r 0.05) + FPFH(r 0.08) at "
                        "the keypoints")
        else:
            workload = (f"configs[4] batch of {n_scans} 1M-pt room scans (seeds 100..{99 + n_scans}) round-robin over "
                        f"{world} GPU(s), configs[2] work per scan, K_s x 33 descriptors + indices gathered to rank 0 "
                        f"(RCCL grouped send/recv)")
        data = "synthetic (synth_room: seeded pinhole room scan, k(0.05)~230; see synth.py)"
        scaling = "strong" if n_scans > 1 else "weak"
        if fast:
            metric = ("Mpoints/s through NARF keypoint + FPFH descriptor on 1M-pt cloud, opt-in MFMA-covariance "
                      "normals (not parity-exact)")
            workload = ("configs[2] scan with pfx_normals_fast_dev in place of the parity-exact normal estimation "
                        "(deviation from the parity path in `deviation_from_parity_path`)")
        if npts != N_POINTS:
            metric = "Mpoints/s through NARF keypoint + FPFH descriptor, configs[2] scene at 10x density"
            workload = (f"SURVEY 8(d) dense variant: configs[2]'s room scene (same scale) at {npts // 1_000_000}M "
                        f"points, NARF(support 0.2) + normals(r 0.05) + FPFH(r 0.08) at the keypoints")
            data = f"synthetic (synth_room at 10x density: {npts} points, k(0.05)~{int(nb / npts)}; see synth.py)"
    # the critical path: every stage's HIP-event time on its own stream inside the
    # timed region, per scan -- NARF on the main stream beside the normal estimation on the side
    # stream, then FPFH's SPFH and weighting on the main stream behind the normals
    stages = {}
    for nm, key in (("narf", "narf"), ("normals", "normals_fast" if fast else "normals"), ("fpfh_spfh", "fpfh_spfh"),
                    ("fpfh_weight", "fpfh_weight"), ("shot", "shot")):
        ms, calls = timers.get(key, (0.0, 0))
        if calls:
            stages[nm] = round(ms / max(per_scan_calls, 1), 4)
    stages_note = ("HIP events around each stage on its stream, inside the timed region, per scan; NARF (range image, "
                   "borders, interest, NMS + the host greedy selection, keypoint gather) runs on the main stream while "
                   "the normal estimation runs on the side stream, then SPFH and the weighting follow the normals")
    return {
        "metric": metric, "value": round(value, 4), "unit": "Mpoints/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": workload, "points_per_scan": npts, "scans_per_step": n_scans,
                   "image": "640x480", "parallelism": f"scan-per-gpu x{world}"},
        "stages_ms_per_scan": stages, "stages_note": stages_note,
        "roofline": roofline,
    }


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
        # MFMA work per step: one tile pass over the padded (ns x nt) grid, K = 3 x 352 (bf16 split);
        # the candidate test runs over the pruned pair list the pass emits (a second contraction only
        # when that list overflows: match_filter, counted if it ran)
        # plus the seeding pass over the cross of the first 4 row / column tiles (match_seed)
        pad = lambda v: (v + 127) // 128 * 128  # noqa: E731
        tb, nb = ctx.kernel_time("match_bound")
        tf, nf = ctx.kernel_time("match_filter")
        tsd, nsd = ctx.kernel_time("match_seed")
        gx, gy = pad(nt) // 128, pad(ns) // 128
        sr, sc = min(gy, max(4, (gy + 19) // 20)), min(gx, max(4, (gx + 19) // 20))
        seed_tiles = sr * gx + sc * (gy - sr) if (gx > 16 and gy > 16) else 0
        flops = ((1 + nf / max(nb, 1)) * pad(ns) * pad(nt) + (nsd / max(nb, 1)) * seed_tiles * 128 * 128) * 2.0 * 3 * 352
        tiles_s = (tb + tf + tsd) / max(nb, 1) / 1e3
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
        def stat(nm):
            try:
                return ctx.stat(nm)
            except Exception:  # a library build without that statistic
                return None

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
            "roofline": {"bound": "mfma", "kernel": ("k_match_tiles<0,seed> + " if nsd else "") + "k_match_tiles<0>"
                         + (" + k_match_tiles<1>" if nf else ""), "achieved": round(achieved, 2),
                         "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 5),
                         "traffic": None, "flops_per_step": flops, "avg_tiles_ms": round(tiles_s * 1e3, 4),
                         "candidates": {"pairs_emitted": stat("match_pairs_emitted"),
                                        "rows": stat("match_candidates_rows"),
                                        "cols": stat("match_candidates_cols")}},
            "cpu_baseline": cpu,
        }
        if os.environ.get("PFX_BENCH_VERBOSE"):
            rep = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4)
                   for nm in ("match", "match_seed", "match_bound", "match_filter", "match_exact")}
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


def bench_harris(args, torch, dev, world, rank, local, six=False):
    """Keypoints("Harris3D" / "Harris6D").compute over the 1M-point room scan (one
    per rank); Harris6D reads the scan's colours (synth.texture_rgb: a smooth procedural texture)."""
    import numpy as np

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import keypoints_harris3d, keypoints_harris6d
    from pcl_feature_extraction_amd.synth import synth_room, texture_rgb

    seed = 2 if world == 1 else 100 + rank
    x, y, z, _ = synth_room(N_POINTS, seed)
    rgb = texture_rgb(x, y, z, seed)
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    dx, dy, dz = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    drgb = torch.from_numpy(rgb.view(np.int32)).to(dev)
    idx = torch.empty(N_POINTS, dtype=torch.int32, device=dev)
    tag = "harris6d" if six else "harris3d"

    def step():
        if six:
            return keypoints_harris6d(ctx, dx, dy, dz, drgb, idx)
        return keypoints_harris3d(ctx, dx, dy, dz, idx)
    k = 0
    for _ in range(args.warmup):
        k = step()
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    ctx.reset_timing()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        nb = ctx.stat("normals_neighbors")
        if six:
            # gradient (two passes: list entry 4 B + xyz 12 B + rgb 4 B per neighbour, normal in and
            # gradient out 24 B per point) + response (entry 4 B + normal 12 B + gradient 12 B per
            # neighbour, 4 B out): sum_q |N_0.01(q)| x 68 B + N x 28 B
            tg, ng = ctx.kernel_time("harris6d_gradient")
            tr, nr = ctx.kernel_time("harris6d_response")
            resp_s = (tg / max(ng, 1) + tr / max(nr, 1)) / 1e3
            algo = nb * 68 + N_POINTS * 28
            kname = "k_intensity_gradient + k_harris6d_response"
        else:
            # the response kernel: every query's FLANN-ordered list (4 B entries) and its neighbours'
            # normals; algorithmic bytes per launch = sum_q |N_0.01(q)| x (4 + 12) B + N x 4 B
            tr, nr = ctx.kernel_time("harris3d_response")
            resp_s = tr / max(nr, 1) / 1e3
            algo = nb * 16 + N_POINTS * 4
            kname = "k_harris_response + k_harris_nms"
        achieved = algo / resp_s / 1e9 if resp_s > 0 else 0.0
        names = (tag, "normals_lists_phase", "grid_bbox", "grid_build", "normals_tiles", "normals_lists_small",
                 "normals_lists_sparse", "normals_lists_dense", "normals_lists_wide", "normals_lists_query", "normals_chain",
                 "normals_chain_big", "normals_long", tag + "_refine")
        names += ("harris6d_gradient", "harris6d_response") if six else ("harris3d_response",)
        stages = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4) for nm in names}
        corners = ctx.stat(tag + "_corners")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            runs = []
            for _ in range(2):  # 1 warm-up + 1 timed: the OpenMP restatement takes seconds per scan
                c0 = time.perf_counter()
                okp = (O.harris6d(x, y, z, rgb, 0.01, 1e-6, True, threads=threads)[0] if six
                       else O.harris3d(x, y, z, 0.01, 1e-6, True, threads=threads)[0])
                runs.append(time.perf_counter() - c0)
            csec = runs[-1]
            same = bool(np.array_equal(okp, idx[:k].cpu().numpy()))
            cpu = {"value": round(N_POINTS / csec / 1e6, 6), "unit": "Mpoints/s", "cores": threads, "kind": "port",
                   "sample": (f"the same 1M-point scan through the CPU restatement (oracle/or_keypoints.cpp "
                              f"orc_{tag}: OpenMP normals, {'gradients, ' if six else ''}responses, suppression, "
                              f"refinement), 1 warm-up + 1 timed run: {csec:.1f}s"),
                   "parity": {"keypoints": same}}
        label = "HARRIS_6D" if six else "HARRIS_3D"
        line = {
            "metric": f"Mpoints/s through {'Harris6D' if six else 'Harris3D'} keypoints (Keypoints::compute "
                      f"{label} branch) on 1M-pt cloud",
            "value": round(world * N_POINTS * args.steps / elapsed / 1e6, 4),
            "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic (synth_room: seeded pinhole room scan" +
                     (", colours from synth.texture_rgb" if six else "") + "; see synth.py)"),
            "config": {"workload": (f"SURVEY 8(f) F3: HarrisKeypoint{'6D' if six else '3D(HARRIS'}"
                                    f"{'(' if six else ', '}r 0.01, nms, threshold 1e-6, refine) + "
                                    "getKeypointsCloud on configs[2]'s 1M-pt room"), "points_per_scan": N_POINTS,
                       "corners": int(corners), "keypoints": int(k), "parallelism": f"scan-per-gpu x{world}"},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None, "algorithmic_bytes_per_launch": int(algo), "avg_ms": round(resp_s * 1e3, 4),
                         "neighbors_per_launch": int(nb), "stages_ms_per_step": stages},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()


def bench_config1(args, torch, dev, world, rank, local):
    """configs[1]: the 100k-point synthetic room (seed 1; replicas seed 1 + rank at N > 1),
    NormalEstimationOMP (r 0.05) + FPFHEstimation (r 0.05) at every point, input == surface
    (PCL's all-points SPFH branch, features.h:188-195 with the cloud as both).  One step =
    pfx_normals_dev + pfx_fpfh_dev(same_as_surface) on the device-resident cloud.  roofline: the
    dominant FPFH kernel of the step -- the all-points weighting over the FLANN
    lists (sum_q |N(q)| x 136 B: the 33-float SPFH row + the list entry per neighbour) or SPFH
    (sum_{p in S} |N(p)| x 24 B, S = every point), whichever took longer; both beside it.  The
    timed region carries the stage timers only; the per-kernel breakdown comes from extra steps."""
    import numpy as np

    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.pipeline import alloc
    from pcl_feature_extraction_amd.synth import synth_room

    n = 100_000
    x, y, z, _ = synth_room(n, 1 + rank)
    b = alloc(torch, n, dev, max_keypoints=n)
    for t, a in zip((b.x, b.y, b.z), (x, y, z)):
        t.copy_(torch.from_numpy(a))
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def step():
        ctx.normals_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
        ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.x, b.y, b.z, 0.05, b.desc, same_as_surface=True,
                     after_normals=True)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    ctx.set_timing(True, stages_only=True)
    ctx.reset_timing()
    elapsed = timed(torch, torch.distributed, dev, world, args.steps, step)
    live = {nm: round(ctx.kernel_time(nm)[0] / args.steps, 4) for nm in ("normals", "fpfh_spfh", "fpfh_weight")}
    detail_steps = max(3, args.steps // 4)
    ctx.set_timing(True)
    ctx.reset_timing()
    timed(torch, torch.distributed, dev, world, detail_steps, step)
    if rank != 0:
        ctx.close()
        return
    names = ("normals", "fpfh_mark", "fpfh_spfh", "fpfh_weight", "grid_build", "normals_lists_small",
             "normals_lists_sparse", "normals_lists_dense", "normals_lists_wide", "normals_lists_query", "normals_chain",
             "normals_chain_big", "normals_long")
    stages = {nm: round(ctx.kernel_time(nm)[0] / detail_steps, 4) for nm in names}
    ctx.set_timing(False)
    pairs = ctx.stat("fpfh_spfh_pairs")
    nb = ctx.stat("normals_neighbors")
    spfh_ms, weight_ms = live["fpfh_spfh"], live["fpfh_weight"]
    kern = {"fpfh_spfh": {"kernel": "k_fpfh_spfh + k_fpfh_exact + k_fpfh_finalize", "ms": spfh_ms,
                          "algorithmic_bytes_per_launch": int(pairs * 24),
                          "note": "sum_{p in S} |N(p)| x 24 B (xyz + normal per pair, SURVEY 8(d)); S = all 100k points"},
            "fpfh_weight": {"kernel": "k_fpfh_weight_lists / k_fpfh_weight_units (input == surface)", "ms": weight_ms,
                            "algorithmic_bytes_per_launch": int(nb * 136),
                            "note": "sum_q |N(q)| x 136 B (the neighbour's 33-float SPFH row + its list entry)"}}
    for v in kern.values():
        v["achieved"] = round(v["algorithmic_bytes_per_launch"] / (v["ms"] / 1e3) / 1e9, 2) if v["ms"] > 0 else None
        v["frac"] = round(v["achieved"] / HBM_PEAK_GBS, 5) if v["achieved"] else None
    dom = max(kern, key=lambda nm: kern[nm]["ms"])
    algo = kern[dom]["algorithmic_bytes_per_launch"]
    achieved = kern[dom]["achieved"] or 0.0
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)

        def once(cx, cy, cz):
            t0 = time.perf_counter()
            on = O.normals(cx, cy, cz, 0.05, threads=threads)
            t1 = time.perf_counter()
            od = O.fpfh(cx, cy, cz, on[0], on[1], on[2], cx, cy, cz, 0.05, same_as_surface=True, threads=1)
            return (t1 - t0, time.perf_counter() - t1), (on, od)
        once(x[::10], y[::10], z[::10])  # warm-up on a 1/10 subsample
        runs, out = [], None
        for _ in range(5):
            t, out = once(x, y, z)
            runs.append(t)
        tot = sorted(sum(t) for t in runs)
        med = tot[len(tot) // 2]
        st = [sorted(t[i] for t in runs)[len(runs) // 2] for i in range(2)]

        def same(a, c):  # raw bits, NaN rows included (PCL's quiet_NaN on both sides)
            a, c = np.ascontiguousarray(np.asarray(a, np.float32)), np.ascontiguousarray(np.asarray(c, np.float32))
            return bool(a.shape == c.shape and np.array_equal(a.view(np.uint32), c.view(np.uint32)))
        parity = {"normals": all(same(t.cpu().numpy(), o) for t, o in zip((b.nx, b.ny, b.nz, b.curv), out[0])),
                  "descriptors": same(b.desc[:n].cpu().numpy(), out[1])}
        cpu = {"value": round(n / med / 1e6, 6), "unit": "Mpoints/s", "cores": threads, "kind": "port",
               "sample": (f"the same 100k-point scan through the CPU restatement (oracle/), 1 warm-up (1/10 "
                          f"subsample) + median of 5 full runs: normals {threads} threads {st[0]:.2f}s, FPFH at every "
                          f"point 1 thread (PCL 1.7's non-OMP FPFHEstimation) {st[1]:.2f}s"),
               "runs_s": [round(v, 3) for v in tot], **host_info(), "parity": parity}
    line = {
        "metric": "Mpoints/s through NormalEstimation + FPFH (r 0.05) at every point of a 100k-pt cloud",
        "value": round(world * n * args.steps / elapsed / 1e6, 4), "unit": "Mpoints/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (synth_room(100000, seed 1): seeded pinhole room scan, k(0.05)~230; see synth.py)",
        "config": {"workload": "configs[1] 100k-pt synthetic room, NormalEstimation(r 0.05) + FPFH(r 0.05) at all "
                               "points (input == surface)", "points_per_scan": n,
                   "parallelism": f"scan-per-gpu x{world}"},
        "stages_ms_per_scan": live,
        "roofline": {"bound": "hbm", "kernel": kern[dom]["kernel"], "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "algorithmic_bytes_per_launch": int(algo), "avg_ms": kern[dom]["ms"], "pairs_per_launch": int(pairs),
                     "note": kern[dom]["note"] + "; the dominant FPFH kernel of the step (live stage timers)",
                     "kernels": kern, "normals_neighbors": int(nb), "stages_ms_per_step": stages,
                     "stages_basis": f"per-kernel HIP events over {detail_steps} extra steps after the timed region"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
