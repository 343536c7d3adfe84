#!/bin/bash
# A/B of the dense 10M-point variant (bench.py --workload dense): libpfx_base.so vs libpfx.so,
# one run each, per-kernel times of the normal-estimation stage.   usage: bash scripts/gpu_ab_dense.sh
set -o pipefail
mkdir -p gpurun_out
for v in base new; do
  if [ $v = base ]; then L=$PWD/pcl_feature_extraction_amd/libpfx_base.so; else L=$PWD/pcl_feature_extraction_amd/libpfx.so; fi
  PFX_LIB=$L timeout -k 10 400 python bench.py --workload dense --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/d_ab.json 2> gpurun_out/d_ab.err || { tail -20 gpurun_out/d_ab.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/d_ab.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], json.dumps(r['kernels_ms_per_scan']))")"
done
