"""Every kernel/copy of one timed bench step's first N us (rocprofv3 kernel-trace CSV), queue and
offsets from the end of the previous step's last FPFH weighting kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 900.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_fpfh_weight<true>" in r["Kernel_Name"]]
k0, k1 = ends[-6], ends[-5]  # inside the timed region (5 timed steps, then 3 detail steps)
t0, t1 = int(rows[k0]["End_Timestamp"]), int(rows[k1]["End_Timestamp"])
for r in rows[k0 - 6:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t1 and (s - t0) < lim * 1e3:
        n = r["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        n = n.replace("rocprim::ROCPRIM_400200_NS::detail::", "")[:70]
        print("q%s %8.1f %8.1f  %s" % (r.get("Queue_Id", "?"), (s - t0) / 1e3, (e - s) / 1e3, n))
