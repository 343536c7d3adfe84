#!/bin/bash
# round 6: SPFH on surfaces over 4M points with 4x / 16x its waves (sp4 / sp16) -- dense line
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" sp4 sp16; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 500 python bench.py --workload dense --steps 2 --warmup 1 > gpurun_out/bench_dense_ab.json 2> gpurun_out/bench_dense_ab.err || { tail -20 gpurun_out/bench_dense_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_dense_ab.json')); print('$L', d['value'], d['ms_per_step'], d.get('stages_ms_per_scan'))"
done
done
