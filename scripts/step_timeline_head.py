"""First `window` us of one timed bench step: every kernel (any length) and every memory copy,
from a rocprofv3 --kernel-trace --memory-copy-trace CSV pair (usage: dir window_us)."""
import csv
import glob
import sys

d, win = sys.argv[1], float(sys.argv[2])
kr = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
kr.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(kr) if "k_fpfh_weight<true>" in r["Kernel_Name"] or "k_fpfh_weight<false>" in r["Kernel_Name"]]
t0 = int(kr[ends[-4]]["End_Timestamp"])
ev = []
for r in kr:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s <= t0 + win * 1e3:
        n = r["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]
        ev.append((s, e, "q" + r.get("Queue_Id", "?"), n))
mc = glob.glob(d + "/*memory_copy_trace.csv")
if mc:
    for r in csv.DictReader(open(mc[0])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s <= t0 + win * 1e3:
            ev.append((s, e, "copy", r.get("Direction", "?") + " " + r.get("Size", "?")))
for s, e, q, n in sorted(ev):
    print("%-5s %8.1f %8.1f  %s" % (q, (s - t0) / 1e3, (e - s) / 1e3, n))
