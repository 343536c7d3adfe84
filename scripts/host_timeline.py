"""Host-side timeline of the overlapped (NARF, FPFH) step: entry/exit of every C-ABI call (per
thread) against the device time at which each step's work drained, on one time axis (us from a
synchronised reference event).  Shows whether the host issues step i+1 before step i drains."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import DeviceRows, OverlappedNarfFpfh, alloc  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
for t, a in zip((b.x, b.y, b.z), (x, y, z)):
    t.copy_(torch.from_numpy(a))
ctx, ctx_n = Context(0), Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
rows = DeviceRows(torch, dev)
log = []


def wrap(obj, name, tag):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            log.append((t0, time.perf_counter(), threading.current_thread().name[:6], tag))
    setattr(obj, name, g)


for nm in ("narf_keypoints_dev", "gather_points_dev", "fpfh_prepare_dev", "fpfh_prepare_queries_dev", "fpfh_dev"):
    wrap(ctx, nm, nm)
for nm in ("normals_launch_dev", "normals_finish_dev", "normals_dev"):
    wrap(ctx_n, nm, "side." + nm)
for _ in range(3):
    kp, k = run(b)
    rows(kp, len(x))
torch.cuda.synchronize()
ref = torch.cuda.Event(enable_timing=True)
ref.record()
torch.cuda.synchronize()
h0 = time.perf_counter()
log.clear()
ends, starts = [], []
for i in range(6):
    log.append((time.perf_counter(), time.perf_counter(), "Main", "---- step %d" % i))
    kp, k = run(b)
    rows(kp, len(x))
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    ends.append(e)
torch.cuda.synchronize()
for i, e in enumerate(ends):
    print("device drained step %d at %8.1f us" % (i, ref.elapsed_time(e) * 1e3))
for t0, t1, th, tag in sorted(log):
    print("%-7s %8.1f %8.1f  %s" % (th, (t0 - h0) * 1e6, (t1 - t0) * 1e6, tag))
