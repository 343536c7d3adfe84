"""Profiling aid: the NARF + normals + FPFH pass run sequentially on ONE stream (no overlap), so
every stage's HIP-event time is its own (bench.py overlaps NARF with normal estimation)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc, narf_fpfh  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

NAMES = ["grid_build", "range_image", "narf_border", "narf_interest", "narf_nms", "normals_lists_sparse",
         "normals_lists_dense", "normals_lists_query", "normals_chain", "normals_chain_big", "normals_long",
         "fpfh_mark", "fpfh_spfh", "fpfh_weight"]
x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
with Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(2):
        narf_fpfh(ctx, b)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_timing()
    steps = 5
    t0 = time.perf_counter()
    for _ in range(steps):
        narf_fpfh(ctx, b)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    t = {n: round(ctx.kernel_time(n)[0] / steps, 4) for n in NAMES}
    print("sequential pass %.3f ms" % wall, json.dumps(t), "sum %.3f" % sum(t.values()), flush=True)
