#!/bin/bash
# A/B of the FPFH stage (fpfh_only.py): base vs current library, twice; FPFH parity tests first.
mkdir -p gpurun_out
K=${1:-fpfh or pipeline or fullsize or determinism or golden}
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 200 python scripts/fpfh_only.py > gpurun_out/ab_f.log 2>&1 || { tail -30 gpurun_out/ab_f.log; exit 1; }
  grep libpfx gpurun_out/ab_f.log
done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
cut -c1-220 gpurun_out/b_ab.json
timeout -k 10 300 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/b_ab1.json 2> gpurun_out/b_ab1.err || { tail -30 gpurun_out/b_ab1.err; exit 1; }
cut -c1-220 gpurun_out/b_ab1.json
