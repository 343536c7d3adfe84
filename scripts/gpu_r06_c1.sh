#!/bin/bash
# configs[1] line A/B of library builds (two rounds each): value, step, weighting and SPFH stages
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    PFX_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -20 gpurun_out/c1.err; exit 1; }
    echo "config1 $(basename $L) $(python -c "import json; d=json.load(open('gpurun_out/c1.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('stages_ms_per_scan')), json.dumps(d['roofline']['stages_ms_per_step']))")"
  done
done
