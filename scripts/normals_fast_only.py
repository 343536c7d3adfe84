"""Profiling aid: the opt-in MFMA normal estimation (pfx_normals_fast_dev) alone on the bench scan,
5 launches, with HIP-event times per stage."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
with Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.normals_fast_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(5):
        ctx.normals_fast_dev(b.x, b.y, b.z, 0.05, b.nx, b.ny, b.nz, b.curv)
    torch.cuda.synchronize()
    print(json.dumps({n: round(ctx.kernel_time(n)[0] / 5, 4) for n in ("normals_fast", "normals_mfma", "grid_build")}))
