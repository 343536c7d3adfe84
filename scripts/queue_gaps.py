"""Per-queue view of one bench step from a rocprofv3 kernel trace: every dispatch on each queue
with the idle time before it (host launch latency or a cross-queue wait shows up there), and the
queue's busy / idle totals."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_ri_init" in r["Kernel_Name"]]
t0, t1 = starts[-3], starts[-2]
step = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
print("step %.3f ms" % ((t1 - t0) / 1e6))
for q in sorted({r["Queue_Id"] for r in step}):
    ks = [r for r in step if r["Queue_Id"] == q]
    prev_e, busy, idle = None, 0, 0
    print("queue", q, len(ks), "dispatches")
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = 0 if prev_e is None else max(0, s - prev_e)
        idle += gap
        busy += e - s
        n = r["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        n = n.replace("rocprim::ROCPRIM_400200_NS::detail::", "")[:50]
        print("  +%7.1f  gap %6.1f  dur %7.1f  %s" % ((s - t0) / 1e3, gap / 1e3, (e - s) / 1e3, n))
        prev_e = e if prev_e is None else max(prev_e, e)
    print("  busy %.1f us, gaps %.1f us" % (busy / 1e3, idle / 1e3))
