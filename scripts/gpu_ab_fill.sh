#!/bin/bash
# A/B: base vs current library on the headline step (three pairs), after the grid/list tests
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "normals or pipeline or determinism or radius or iss or harris or grid or fpfh" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2 3; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
  echo "$L $(cut -c80-150 gpurun_out/b_ab.json)"
done
done
