#!/bin/bash
# round 6: k_normals_long's queue split into per-XCD eighths (variant libpfx_xcd) against the
# shipped build -- dense / room normal
# estimation alone, the headline and the dense line, alternating
set -o pipefail
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_xcd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -x -q -m gpu -k normals --timeout 120 --timeout-method thread > gpurun_out/t_r06g38.log 2>&1 || { tail -30 gpurun_out/t_r06g38.log; exit 1; }
tail -1 gpurun_out/t_r06g38.log
for r in 1 2; do
for L in xcd ""; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  echo "== $L"
  PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=3 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
  grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  if [ $r -eq 1 ]; then
    PFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_ab.json 2> gpurun_out/bench_head_ab.err || { tail -20 gpurun_out/bench_head_ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_head_ab.json')); r=d['roofline']; print('head $L', d['value'], d['ms_per_step'], r['chain']['frac'])"
    PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload dense --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dense_ab.json 2> gpurun_out/bench_dense_ab.err || { tail -20 gpurun_out/bench_dense_ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_dense_ab.json')); print('dense $L', d['value'], d['ms_per_step'])"
  fi
done
done
