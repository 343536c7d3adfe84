#!/bin/bash
# round 6: 64-step long-list batches (shipped) against 32 (lb32); GPU tests first (with the new
# list-buffer edge test), then dense + room normal estimation alone
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06r.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06r.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06r.log | head -30; exit 1; }
for r in 1 2; do
  for L in "" lb32; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  done
done
