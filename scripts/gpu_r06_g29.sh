#!/bin/bash
# round 6: the all-points FPFH weighting at 32 (shipped) / 64 / 128 workgroups per CU (configs[1])
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" g64 g128; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  if [ $r = 1 ] && [ "$L" = "" ]; then extra=""; else extra="--no-cpu-baseline"; fi
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload config1 $extra > gpurun_out/bench_c1_ab.json 2> gpurun_out/bench_c1_ab.err || { tail -20 gpurun_out/bench_c1_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c1_ab.json')); r=d['roofline']; print('c1 $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'), (d.get('cpu_baseline') or {}).get('parity'))"
done
done
