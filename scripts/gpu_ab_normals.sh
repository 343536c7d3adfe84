#!/bin/bash
# A/B of normal estimation alone (normals_only.py): base vs current library, twice; parity tests of
# the normals/lists paths; the default bench line.   usage: bash scripts/gpu_ab_normals.sh [-k expr]
mkdir -p gpurun_out
K=${1:-normals or search or fpfh or determinism or fullsize or pipeline}
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2; do
for L in libpfx_base.so libpfx.so; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/$L timeout -k 10 200 python scripts/normals_only.py > gpurun_out/ab_no.log 2>&1 || { tail -30 gpurun_out/ab_no.log; exit 1; }
  echo $L; grep -E "^(room|seabed)" gpurun_out/ab_no.log | cut -c1-330
done
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
cut -c1-220 gpurun_out/b_ab.json
