"""Per-kernel timeline of one timed bench step from a rocprofv3 kernel-trace CSV (queue, start
offset, duration in us; kernels >= 10 us), plus per-kernel durations across all launches."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_fpfh_weight<true>" in r["Kernel_Name"]]
k0, k1 = ends[-6], ends[-5]  # a step inside the timed region (bench: 5 timed steps, then 3 with per-kernel timers)
t0, t1 = int(rows[k0]["End_Timestamp"]), int(rows[k1]["End_Timestamp"])
print("step us %.1f" % ((t1 - t0) / 1e3))
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and e <= t1 and e - s >= 10000:
        n = r["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        print("q%s %8.1f %8.1f  %s" % (r.get("Queue_Id", "?"), (s - t0) / 1e3, (e - s) / 1e3, n))
