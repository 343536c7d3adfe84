#!/bin/bash
# A/B of the NARF stage only (no tests): base vs current library, twice; then the default bench line.
mkdir -p gpurun_out
for i in 1 2; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 120 python scripts/narf_only.py > gpurun_out/ab_n.log 2>&1 || { tail -30 gpurun_out/ab_n.log; exit 1; }
  grep libpfx gpurun_out/ab_n.log
done
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
cut -c1-220 gpurun_out/b_ab.json
