#!/bin/bash
# round 6: the deferred workgroups' lists over 1024 entries chained by a second k_normals_long on
# the side stream beside k_normals_chain_big (shipped) against no split -- GPU tests, then room /
# dense normal estimation alone and the headline line, alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06z.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06z.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06z.log | head -30; exit 1; }
for r in 1 2; do
for L in "" nosplit; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  echo "== $L"
  PFX_LIB=$PWD/$lib PFX_NO_SCENES=room,dense PFX_NO_STEPS=3 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
  grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  PFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_ab.json 2> gpurun_out/bench_head_ab.err || { tail -20 gpurun_out/bench_head_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_head_ab.json')); r=d['roofline']; k=r['kernels_ms_per_scan']; print('head $L', d['value'], d['ms_per_step'], r['avg_ms'], r['chain']['frac'], k['normals_chain'], k['normals_chain_big'], k['normals_long'])"
done
done
