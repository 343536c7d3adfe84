#!/bin/bash
# round 6: SPFH on surfaces of <= 256k points (configs[1]) with 1/2 / 1/4 of its waves
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" ss2 ss4; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/bench_c1_ab.json 2> gpurun_out/bench_c1_ab.err || { tail -20 gpurun_out/bench_c1_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c1_ab.json')); r=d['roofline']; print('c1 $L', d['value'], d['ms_per_step'], d.get('stages_ms_per_scan'))"
done
done
