#!/bin/bash
# rocprofv3 kernel-trace summary of the SHOT workload (configs[3])
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_shot -o run -- python3 $R/bench.py --workload shot --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_shot.log 2>&1 || { tail -20 $R/gpurun_out/prof_shot.log; exit 1; }
cd $R && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_shot/run_kernel_stats.csv")))
for r in rows[:14]:
    print("%9.3f ms  calls %5s  avg %8.3f  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], float(r["AverageNs"]) / 1e6, r["Name"][:70]))
PY
