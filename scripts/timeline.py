"""Per-stream timeline of the last bench step from a rocprofv3 kernel-trace CSV: kernels in
start order with queue id, start offset and duration (us), to see what overlaps what."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step: from the last k_bbox launch pair's first launch (each step builds grids)
starts = [i for i, r in enumerate(rows) if "k_bbox" in r["Kernel_Name"]]
first = starts[-3] if len(starts) >= 3 else 0
t0 = int(rows[first]["Start_Timestamp"])
end = 0
for r in rows[first:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    end = max(end, e)
    name = r["Kernel_Name"]
    name = name.replace("pfx::(anonymous namespace)::", "").replace("void ", "")
    name = name.replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim:").split("(")[0][:48]
    print(f"q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3} {s / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")
print("span us", end / 1e3)
