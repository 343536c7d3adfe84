import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import torch
from pcl_feature_extraction_amd import Context, camera, narf_params
from pcl_feature_extraction_amd.synth import synth_room
x, y, z, _ = synth_room(1_000_000, 2)
with Context(0) as ctx:
    kp = ctx.narf_keypoints(x, y, z, params=narf_params(support_size=0.2, calculate_sparse_interest_image=0))
    it = np.asarray(ctx.narf_debug_image("interest"), np.float32).ravel()
    scs = np.asarray(ctx.narf_debug_image("surface_change"), np.float32).ravel() if True else None
    print("kp", len(kp), "pixels", it.size, "interest>0", (it > 0).sum(), ">=0.2", (it >= 0.2).sum(), ">=0.3", (it >= 0.3).sum(), ">=0.45", (it >= 0.45).sum())
    for q in (0.5, 0.9, 0.99):
        print(q, np.quantile(it[it > 0], q))
    print("scs>=0.45", (scs >= 0.45).sum(), "scs>=0.2", (scs >= 0.2).sum(), "scs==1", (scs == 1).sum())
