#!/bin/bash
# round 6: the all-points FPFH weighting at 24 / 32 (shipped) / 40 / 48 workgroups per CU (configs[1])
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" w24 w40 w48; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/bench_c1_ab.json 2> gpurun_out/bench_c1_ab.err || { tail -20 gpurun_out/bench_c1_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c1_ab.json')); r=d['roofline']; print('c1 $L', d['value'], d['ms_per_step'], d.get('stages_ms_per_scan'))"
done
done
