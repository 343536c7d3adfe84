#!/bin/bash
# round-6 A/B: GPU tests on the new library, then normals-only + headline bench for each library
# given (gpu_ab_n.sh), then the phase profile of the instrumented build.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_$TAG.log | head -30; exit 1; }
bash scripts/gpu_ab_n.sh "$@" || exit 1
if [ -f pcl_feature_extraction_amd/libpfx_prof.so ]; then
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so PFX_NO_STEPS=1 timeout -k 10 200 python scripts/normals_only.py > gpurun_out/noprof_$TAG.log 2>&1 && grep -E "tile cycles|query cycles|wave cycles" gpurun_out/noprof_$TAG.log | head -6
fi
