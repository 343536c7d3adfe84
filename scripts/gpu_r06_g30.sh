#!/bin/bash
# round 6: SHOT's split kernels with 2x / 4x their grids (s2 / s4) against the shipped grids
# (configs[3] line, alternating); SHOT GPU tests on s4 first
set -o pipefail
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_s4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_shot.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06y.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06y.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06y.log | head -30; exit 1; }
for r in 1 2; do
for L in "" s2 s4; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload shot --no-cpu-baseline > gpurun_out/bench_shot_ab.json 2> gpurun_out/bench_shot_ab.err || { tail -20 gpurun_out/bench_shot_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_shot_ab.json')); r=d['roofline']; print('shot $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'))"
done
done
# the keypoint weighting's grid: 512 (shipped) / 2048 (w2k) / 256 (w256) workgroups (headline)
for r in 1 2; do
for L in "" w2k w256; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_ab.json 2> gpurun_out/bench_head_ab.err || { tail -20 gpurun_out/bench_head_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_head_ab.json')); r=d['roofline']; print('head $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'))"
done
done
