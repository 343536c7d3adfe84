#!/bin/bash
# round 6: the > 16k list tier (one bucket array, 4096-entry rank windows, eight entries per thread
# in flight), the 8k tier at 1024 threads, chunk prefetch in the wide tiles -- GPU tests, then dense
# + room normal estimation against the previous commit's build, then the phase counters of the
# profiling build on the dense scene
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06o.log 2>&1; rc=$?
tail -1 gpurun_out/t_r06o.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06o.log | head -30; exit 1; }
for r in 1 2; do
  for L in base ""; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  done
done
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so PFX_NO_SCENES=dense PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/dense_prof2.log 2>&1 || { tail -30 gpurun_out/dense_prof2.log; exit 1; }
grep -E "cycles|phases" gpurun_out/dense_prof2.log | tail -8
