"""Idle-gap analysis of a bench step from a rocprofv3 kernel trace: per step, the time no queue
is busy and the largest gaps with their neighbouring dispatches (host round trips show up as
gaps next to copyBuffer)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_ri_init" in r["Kernel_Name"]]
for si in range(max(0, len(starts) - 3), len(starts) - 1):
    t0, t1 = starts[si], starts[si + 1]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
           r["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:36])
          for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    busy, cur_s, cur_e, gaps, prev = 0, None, None, [], None
    for s, e, q, n in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(((s - cur_e) / 1e3, (cur_e - t0) / 1e6, prev, "q%s %s" % (q, n)))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            prev = "q%s %s" % (q, n)
    busy += cur_e - cur_s
    print("step %.3f ms, idle %.3f ms" % ((t1 - t0) / 1e6, (t1 - t0 - busy) / 1e6))
    for g in sorted(gaps, reverse=True)[:8]:
        print("  gap %5.1f us at %.3f ms after %s before %s" % g)
