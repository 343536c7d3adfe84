"""Diagnostic: run configs[3] (1M seabed, narf_shot) on the GPU and save the outputs to
gpurun_out/shot_full.npz for comparison with the oracle off the box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import alloc, alloc_shot, narf_shot  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_seabed  # noqa: E402

N = 1_000_000
x, y, z, _ = synth_seabed(N, 3)
dev = torch.device("cuda", 0)
b = alloc(torch, N, dev)
for t, a in ((b.x, x), (b.y, y), (b.z, z)):
    t.copy_(torch.from_numpy(a))
s = alloc_shot(torch, 1 << 16, dev)
sample_np = np.sort(np.random.default_rng(10).choice(N, 10_000, replace=False))
sample = torch.from_numpy(sample_np.astype(np.int64)).to(dev)
with Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    rows = narf_shot(ctx, b, s, sample)
    torch.cuda.synchronize(dev)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/shot_full.npz", desc=s.desc[:rows].cpu().numpy(), rf=s.rf[:rows].cpu().numpy(),
                    nx=b.nx.cpu().numpy(), ny=b.ny.cpu().numpy(), nz=b.nz.cpu().numpy(), rows=rows)
print("rows", rows)
