#!/bin/bash
# round 6: grids of resident workgroups for the statically strided kernels -- the all-points FPFH
# weighting (configs[1] line against the previous commit, libpfx_base) and the SHOT split kernels
# (configs[3] line against libpfx_shot0); FPFH / SHOT GPU tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_shot.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06x.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06x.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06x.log | head -30; exit 1; }
for r in 1 2; do
for L in "" base; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  if [ $r = 1 ] && [ "$L" = "" ]; then extra=""; else extra="--no-cpu-baseline"; fi
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload config1 $extra > gpurun_out/bench_c1_ab.json 2> gpurun_out/bench_c1_ab.err || { tail -20 gpurun_out/bench_c1_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c1_ab.json')); r=d['roofline']; print('c1 $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'), (d.get('cpu_baseline') or {}).get('parity'))"
done
for L in "" shot0; do
  lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
  PFX_LIB=$PWD/$lib timeout -k 10 400 python bench.py --workload shot --no-cpu-baseline > gpurun_out/bench_shot_ab.json 2> gpurun_out/bench_shot_ab.err || { tail -20 gpurun_out/bench_shot_ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_shot_ab.json')); r=d['roofline']; print('shot $L', d['value'], d['ms_per_step'], r['avg_ms'], d.get('stages_ms_per_scan'))"
done
done
