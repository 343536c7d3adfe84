#!/bin/bash
# SHOT line A/B of the query order (PFX_SHOT_ORDER=0: caller order), two rounds each
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for o in 0 1; do
    PFX_SHOT_ORDER=$o timeout -k 10 300 python bench.py --workload shot --no-cpu-baseline --no-e2e > gpurun_out/sh.json 2> gpurun_out/sh.err || { tail -20 gpurun_out/sh.err; exit 1; }
    echo "shot order=$o $(python -c "import json; d=json.load(open('gpurun_out/sh.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'shot stage', r['avg_ms'])")"
  done
done
