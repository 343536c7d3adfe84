"""Profiling aid: NARF keypoints alone on the bench scan, per-stage HIP-event times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context, camera, narf_params  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
b.x.copy_(torch.from_numpy(x)); b.y.copy_(torch.from_numpy(y)); b.z.copy_(torch.from_numpy(z))
with Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(2):
        kp = ctx.narf_keypoints_dev(b.x, b.y, b.z, narf_params(support_size=0.2), camera())
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_timing()
    steps = 10
    for _ in range(steps):
        kp = ctx.narf_keypoints_dev(b.x, b.y, b.z, narf_params(support_size=0.2), camera())
    torch.cuda.synchronize()
    t = {n: round(ctx.kernel_time(n)[0] / steps, 4) for n in ("range_image", "narf_border", "narf_interest", "narf_nms")}
    print(os.path.basename(os.environ.get("PFX_LIB", "libpfx.so")), len(kp), json.dumps(t), flush=True)
