#!/bin/bash
# round 6: the FPFH weighting's global-scratch passes with the windowed bucket rank and double-
# buffered rows (shipped) against the bitonic sort; the FPFH GPU tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06v.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06v.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06v.log | head -30; exit 1; }
for r in 1 2; do
for L in "" bit128; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 500 python bench.py --workload dense --steps 2 --warmup 1 > gpurun_out/bench_dense_ab.json 2> gpurun_out/bench_dense_ab.err || { tail -20 gpurun_out/bench_dense_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_dense_ab.json')); print('$L', d['value'], d['ms_per_step'], d.get('stages_ms_per_scan'))"
done
done
