#!/bin/bash
# phase cycles (stage / test / sort / write) of the list-builder tile kernels, instrumented build
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python scripts/normals_only.py > gpurun_out/tileprof.log 2>&1 || { tail -30 gpurun_out/tileprof.log; exit 1; }
grep -E "cycles|^room|^seabed" gpurun_out/tileprof.log | tail -12
