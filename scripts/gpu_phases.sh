#!/bin/bash
# GPU-box profiling aid: normal estimation alone with the instrumented build (tile phase cycles)
# and with the product build (per-kernel HIP-event times).   usage: bash scripts/gpu_phases.sh
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python scripts/normals_only.py > gpurun_out/phases_prof.log 2>&1 || { tail -30 gpurun_out/phases_prof.log; exit 1; }
grep -E "cycles|^(room|seabed)" gpurun_out/phases_prof.log
timeout -k 10 300 python scripts/normals_only.py > gpurun_out/normals_only.log 2>&1 || { tail -30 gpurun_out/normals_only.log; exit 1; }
grep -E "^(room|seabed)" gpurun_out/normals_only.log
