"""HIP API calls issued in the first `window` us of one timed bench step (rocprofv3
--kernel-trace --hip-runtime-trace CSVs): thread, start offset, duration, name -- what the host
does between the readbacks of the grid build and the next launches (usage: dir window_us [start_us])."""
import csv
import glob
import sys

d, win = sys.argv[1], float(sys.argv[2])
lo = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0  # window start (us, may be negative)
kr = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
kr.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(kr) if "k_fpfh_weight<false>" in r["Kernel_Name"]]
t0 = int(kr[ends[-4]]["End_Timestamp"])
api = list(csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0])))
rows = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 + lo * 1e3 <= s <= t0 + win * 1e3:
        rows.append((s, e, r.get("Thread_Id", "?"), r.get("Function", r.get("Operation", "?"))))
for s, e, t, n in sorted(rows):
    print("t%-8s %8.1f %7.1f  %s" % (t, (s - t0) / 1e3, (e - s) / 1e3, n))
