#!/bin/bash
# A/B of the matching workload (bench.py --workload match): libpfx_base.so (a build of the previous
# commit) vs libpfx.so (the working tree), after the matching GPU tests on the working tree; two
# pairs, alternating, with the per-kernel HIP-event times (PFX_BENCH_VERBOSE).
set -o pipefail
mkdir -p gpurun_out
BASE=$PWD/pcl_feature_extraction_amd/libpfx_base.so
NEW=$PWD/pcl_feature_extraction_amd/libpfx.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py > gpurun_out/t_match.log 2>&1 || { tail -30 gpurun_out/t_match.log; exit 1; }
tail -1 gpurun_out/t_match.log
for i in 1 2; do
for v in base new; do
  if [ $v = base ]; then L=$BASE; else L=$NEW; fi
  PFX_BENCH_VERBOSE=1 PFX_LIB=$L timeout -k 10 300 python bench.py --workload match --no-cpu-baseline > gpurun_out/b_m.json 2> gpurun_out/b_m.err || { tail -20 gpurun_out/b_m.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/b_m.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_tiles_ms'])") $(grep 'per-step' gpurun_out/b_m.err)"
done
done
