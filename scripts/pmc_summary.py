#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (scripts/gpu_pmc.sh output directory).

FETCH_SIZE is reported doubled (x2, MI355X_MICROARCH.md: gfx950 tallies 128-B requests at 64 B)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].replace("pfx::(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][:60]
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        if row["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
            dur[name + row["Counter_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
rows = []
for k, d in vals.items():
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    t = dur.get(k + "SQ_WAVES") or [0]
    rows.append((sum(t) / len(t) / 1e3, k, avg))
rows.sort(key=lambda r: -r[0])
for us, k, a in rows[:20]:
    print(f"== {k}  ~{us:.1f} us/dispatch (profiled)")
    if "FETCH_SIZE" in a:
        a["FETCH_SIZE_x2_MB"] = a.pop("FETCH_SIZE") * 2 / 1024
    if "WRITE_SIZE" in a:
        a["WRITE_SIZE_MB"] = a.pop("WRITE_SIZE") / 1024
    w = a.get("SQ_WAVES", 0) or 1
    extra = {}
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
        if c in a:
            extra[c + "/wave"] = a[c] / w
    if "SQ_WAVE_CYCLES" in a and a["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in a:
                extra[c + "_frac"] = a[c] / a["SQ_WAVE_CYCLES"]
    if a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0):
        extra["L2_hit"] = a["TCC_HIT_sum"] / (a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted({**a, **extra}.items())))

# machine-readable HBM traffic of one stage for bench.py's roofline.traffic: the sum over the
# named kernels (comma-separated prefixes; every template instance of a prefix counts) of their
# per-dispatch averages
if len(sys.argv) > 3:
    import json
    kernels, dest = sys.argv[2].split(","), sys.argv[3]
    fetch = write = 0.0
    found, per = [], {}
    for us, k, a in rows:
        if any(k == p or k.startswith(p + "<") or k.startswith(p + "(") for p in kernels):
            f = a.get("FETCH_SIZE_x2_MB", 0.0) * 1024 * 1024
            w = a.get("WRITE_SIZE_MB", 0.0) * 1024 * 1024
            fetch += f
            write += w
            found.append(k)
            per[k] = {"hbm_bytes": int(f + w), "us_profiled": round(us, 1),
                      **{c: a[c] for c in ("SQ_WAIT_ANY_frac", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS")
                         if c in a}}
            if "SQ_WAVE_CYCLES" in a and a["SQ_WAVE_CYCLES"] and "SQ_WAIT_ANY" in a:
                per[k]["SQ_WAIT_ANY_frac"] = a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"]
            if a.get("SQ_ACTIVE_INST_LDS"):
                per[k]["lds_conflict_per_active"] = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_ACTIVE_INST_LDS"]
    # the build the counters describe: bench.py reports whether its own libpfx.so is that build
    import hashlib
    import os
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pcl_feature_extraction_amd",
                       "libpfx.so")
    lib_sha16 = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None
    with open(dest, "w") as f:
        json.dump({"kernel": " + ".join(found), "hbm_bytes_per_launch": int(fetch + write), "libpfx_sha16": lib_sha16,
                   "stage_hbm_bytes_per_launch": int(fetch + write),
                   "fetch_bytes_x2": int(fetch), "write_bytes": int(write), "kernels": per,
                   "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, FETCH x2 "
                             "(MI355X_MICROARCH.md gfx950 correction); sum of the kernels' per-dispatch "
                             "averages over bench.py warmup + timed steps"}, f, indent=1)
