#!/bin/bash
# A/B of the NARF stage: parity tests of the current build, then narf_only.py with the base and the
# current library alternately.   usage: bash scripts/gpu_ab_narf.sh [pytest -k expr]
mkdir -p gpurun_out
K=${1:-narf or pipeline or fullsize}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 120 python scripts/narf_only.py > gpurun_out/ab_n.log 2>&1 || { tail -30 gpurun_out/ab_n.log; exit 1; }
  grep libpfx gpurun_out/ab_n.log
done
done
timeout -k 10 120 python scripts/narf_stats.py > gpurun_out/narf_stats.log 2>&1 || { tail -30 gpurun_out/narf_stats.log; exit 1; }
grep sparse gpurun_out/narf_stats.log
