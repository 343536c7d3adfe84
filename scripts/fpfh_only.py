"""Profiling aid: FPFH at the NARF keypoints of the bench scan alone (normals precomputed), with
per-stage HIP-event times; PFX_LIB selects the library build (A/B of compile-time variants)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc, narf_fpfh  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
with Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    _, k = narf_fpfh(ctx, b)
    torch.cuda.synchronize()
    for _ in range(2):
        ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], 0.08, b.desc[:k])
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_timing()
    steps = 10
    for _ in range(steps):
        ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], 0.08, b.desc[:k])
    torch.cuda.synchronize()
    t = {n: round(ctx.kernel_time(n)[0] / steps, 4) for n in ("fpfh_mark", "fpfh_spfh", "fpfh_weight")}
    print(os.path.basename(os.environ.get("PFX_LIB", "libpfx.so")), json.dumps(t), flush=True)
