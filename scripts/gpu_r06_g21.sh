#!/bin/bash
# round 6: 4-wide bucket rank reads in the per-query tiers + the FPFH weighting's two global-scratch
# passes (bucketed sort) -- GPU tests, dense normals A/B against the previous commit, then the
# dense and headline bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06u.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06u.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06u.log | head -30; exit 1; }
for r in 1 2; do
  for L in base ""; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  done
done
timeout -k 10 500 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/bench_dense_r06u.json 2> gpurun_out/bench_dense_r06u.err || { tail -20 gpurun_out/bench_dense_r06u.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_dense_r06u.json')); r=d['roofline']; print('dense', d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], d.get('stages_ms_per_scan'))"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_r06u.json 2> gpurun_out/bench_head_r06u.err || { tail -20 gpurun_out/bench_head_r06u.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_head_r06u.json')); r=d['roofline']; print('head', d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], r['chain']['frac'], d.get('stages_ms_per_scan'))"
