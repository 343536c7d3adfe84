"""Probe of the device idle time between consecutive overlapped (NARF, FPFH) steps: run under
`rocprofv3 --kernel-trace`, then `python scripts/gap_probe.py --report <kernel_trace.csv>` prints,
per step boundary, the time from the last FPFH weighting kernel's end to the next kernel's start.
Modes (argv[1]): base (the bench step), norows (no descriptor-row index copy), notimer (no stage
timers), sync (torch.cuda.synchronize after every step)."""
import csv
import os
import sys

if sys.argv[1] == "--report":
    rows = list(csv.DictReader(open(sys.argv[2])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gaps = []
    for i, r in enumerate(rows):
        if "k_fpfh_weight<true>" in r["Kernel_Name"] and i + 1 < len(rows):
            e = int(r["End_Timestamp"])
            nxt = [x for x in rows[i + 1:i + 40] if "copyBuffer" not in x["Kernel_Name"]]
            if nxt:
                n = nxt[0]
                gaps.append(((int(n["Start_Timestamp"]) - e) / 1e3, n["Kernel_Name"].split("(")[0][-30:]))
    print(" ".join("%.0f" % g for g, _ in gaps[3:]), "|", gaps[-1][1] if gaps else "")
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pcl_feature_extraction_amd import Context  # noqa: E402
from pcl_feature_extraction_amd.pipeline import DeviceRows, OverlappedNarfFpfh, alloc  # noqa: E402
from pcl_feature_extraction_amd.synth import synth_room  # noqa: E402

mode = sys.argv[1]
x, y, z, _ = synth_room(1_000_000, 2)
dev = torch.device("cuda", 0)
b = alloc(torch, len(x), dev)
for t, a in zip((b.x, b.y, b.z), (x, y, z)):
    t.copy_(torch.from_numpy(a))
ctx, ctx_n = Context(0), Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
run = OverlappedNarfFpfh(torch, ctx, ctx_n, dev)
rows = DeviceRows(torch, dev)
if mode != "notimer":
    for c in (ctx, ctx_n):
        c.set_timing(True, stages_only=True)
for i in range(12):
    kp, k = run(b)
    if mode != "norows":
        rows(kp, len(x))
    if mode == "sync":
        torch.cuda.synchronize()
torch.cuda.synchronize()
print(mode, "done")
