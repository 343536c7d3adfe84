"""Profiling aid: normal estimation alone (no concurrent NARF stream) on the bench scans, with
the per-kernel HIP-event times -- the chain-stage roofline without cross-stream interference."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc  # noqa: E402
from pcl_feature_extraction_amd.synth import ROOM_SCALE, synth_room, synth_seabed  # noqa: E402

SCENES = {
    "room": lambda: synth_room(1_000_000, 2),
    "seabed": lambda: synth_seabed(1_000_000, 3),
    # bench --workload dense: the room scene at 10x the density (same scale)
    "dense": lambda: synth_room(10_000_000, 2, scale=ROOM_SCALE * 0.1 ** 0.5),
}
for name in os.environ.get("PFX_NO_SCENES", "room,seabed").split(","):
    x, y, z, _ = SCENES[name]()
    dev = torch.device("cuda", 0)
    b = alloc(torch, len(x), dev)
    b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
    with Context(0) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        for _ in range(2):
            ctx.normals_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.reset_timing()
        steps = int(os.environ.get("PFX_NO_STEPS", "20"))
        for _ in range(steps):
            ctx.normals_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
        torch.cuda.synchronize()
        names = ["grid_build", "normals", "normals_lists_small", "normals_lists_sparse", "normals_lists_dense", "normals_lists_wide", "normals_lists_query",
                 "normals_chain", "normals_chain_big", "normals_long"]
        t = {n: round(ctx.kernel_time(n)[0] / steps, 4) for n in names}
        nb = ctx.stat("normals_neighbors")
        chain = t["normals_chain"] + t["normals_chain_big"]
        gbs = (nb * 12 + len(x) * 16) / (chain / 1e3) / 1e9
        def stat(k):
            try:
                return ctx.stat("normals_" + k)
            except Exception:  # (a library build without that statistic)
                return None
        st = {k: stat(k) for k in ("wide", "single", "mid", "huge", "long_lists", "queries", "tiles_sparse", "tiles_dense",
                                   "chain_wg_staged", "chain_wg_table", "chain_wg_lane", "chain_wg_deferred")}
        print(name, json.dumps(t), json.dumps(st), "chain GB/s %.0f frac %.3f" % (gbs, gbs / 8000.0), flush=True)
