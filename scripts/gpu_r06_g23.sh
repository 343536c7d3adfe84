#!/bin/bash
# round 6: the FPFH weighting's intermediate global-scratch pass -- bucketed sort on 128 workgroups
# (shipped) against the bitonic network on 128 and the bucketed sort on 16 (dense bench stages)
set -o pipefail
mkdir -p gpurun_out
for L in "" bit128 bkt16; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 500 python bench.py --workload dense --steps 2 --warmup 1 > gpurun_out/bench_dense_ab.json 2> gpurun_out/bench_dense_ab.err || { tail -20 gpurun_out/bench_dense_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_dense_ab.json')); print('$L', d['value'], d['ms_per_step'], d.get('stages_ms_per_scan'))"
done
