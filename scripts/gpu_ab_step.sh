#!/bin/bash
# step-level A/B: NARF/pipeline parity tests, then the default bench line (no CPU leg) with the base
# and the current library, alternately, twice each
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "narf or pipeline or fullsize" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
  echo "$L $(cut -c80-150 gpurun_out/b_ab.json)"
done
done
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx.so timeout -k 10 120 python scripts/narf_only.py 2>&1 | grep libpfx
