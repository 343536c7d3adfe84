#!/bin/bash
# A variant library's GPU tests, then the normals-only + headline A/B against the default build
# usage: bash scripts/gpu_r06_variant.sh <variant.so> [tag]
set -o pipefail
mkdir -p gpurun_out
V=$1; TAG=${2:-var}
PFX_LIB=$PWD/$V timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_$TAG.log | head -30; exit 1; }
bash scripts/gpu_ab_n.sh pcl_feature_extraction_amd/libpfx.so $V
