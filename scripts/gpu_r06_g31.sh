#!/bin/bash
# round 6: k_normals_chain_big over 256 (shipped) / 1024 / 4096 workgroups (static stride over
# the deferred groups) -- dense and room normal estimation alone, then the headline line each
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" b1k b4k; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  echo "== $L"
  PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
  grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
done
done
for L in "" b1k b4k; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_ab.json 2> gpurun_out/bench_head_ab.err || { tail -20 gpurun_out/bench_head_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_head_ab.json')); r=d['roofline']; print('head $L', d['value'], d['ms_per_step'], r['avg_ms'], r['chain']['frac'], d.get('stages_ms_per_scan'))"
done
