"""Summarise a rocprofv3 kernel_stats.csv: short kernel name, calls, avg/total us, share."""
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    m = re.search(r"rocprim::[A-Z0-9_]+::detail::(\w+)", name)
    return ("rocprim:" + m.group(1)) if m else name[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
agg = {}
for r in rows:
    k = short(r["Name"])
    c, t = agg.get(k, (0, 0.0))
    agg[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
tot = sum(t for _, t in agg.values())
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
print(f"{'kernel':48s} {'calls':>6s} {'avg_us':>9s} {'per_step_us':>11s} {'share':>6s}")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:48s} {c:6d} {t / c / 1e3:9.1f} {t / steps / 1e3:11.1f} {100 * t / tot:5.1f}%")
