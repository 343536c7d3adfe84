#!/bin/bash
# round 6: per-query list tiers (wider workgroups, records prefetched, direct tier routing, the
# global tier's windowed rank) -- GPU tests on the new build, then normal estimation alone on the
# dense and room scenes: previous build / new / new at 256 threads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06m.log 2>&1; rc=$?
tail -2 gpurun_out/t_r06m.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06m.log | head -30; exit 1; }
for r in 1 2; do
  for L in base "" nt256; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-460
  done
done
