#!/bin/bash
# round 6: two variants -- list-to-wave assignment by descending k (PFX_SORT_LPT) and packed-float4
# staging in the small chain kernel only (PFX_CHAIN_F4, the big kernel keeps 12288 SoA slots) --
# GPU tests on each, then normals-only + headline A/B against the default build
set -o pipefail
mkdir -p gpurun_out
for V in lpt f4; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_$V.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06l_$V.log 2>&1; rc=$?
  echo "tests $V rc=$rc"; tail -2 gpurun_out/t_r06l_$V.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06l_$V.log | head -30; exit 1; }
done
bash scripts/gpu_ab_n.sh pcl_feature_extraction_amd/libpfx.so pcl_feature_extraction_amd/libpfx_lpt.so pcl_feature_extraction_amd/libpfx_f4.so
