#!/bin/bash
# round 6: the FPFH 11-lane-unit weighting (config1 A/B + GPU tests on that build) and the chain
# kernels' 32-bit list index (normals-only + headline A/B)
set -o pipefail
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_units.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06h.log 2>&1; rc=$?; tail -1 gpurun_out/t_r06h.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06h.log | head -20; exit 1; }
bash scripts/gpu_r06_c1.sh pcl_feature_extraction_amd/libpfx.so pcl_feature_extraction_amd/libpfx_units.so || exit 1
bash scripts/gpu_ab_n.sh pcl_feature_extraction_amd/libpfx.so pcl_feature_extraction_amd/libpfx_idx32.so
