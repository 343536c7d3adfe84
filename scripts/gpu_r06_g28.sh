#!/bin/bash
# round 6: more workgroups than resident for the statically strided kernels (finer load balance)
# -- the all-points FPFH weighting at 8 (shipped) / 16 / 32 workgroups per CU (configs[1]) and
# k_normals_long at 1 / 4 / 8x its resident grid (dense normal estimation alone)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for L in "" g16 g32; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/bench_c1_ab.json 2> gpurun_out/bench_c1_ab.err || { tail -20 gpurun_out/bench_c1_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c1_ab.json')); r=d['roofline']; print('c1 $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'))"
  PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
  grep -E "^dense" gpurun_out/ab_d.log | cut -c1-330
done
done
