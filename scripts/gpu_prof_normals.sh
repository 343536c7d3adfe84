#!/bin/bash
# normals alone with the instrumented build (phase cycles of the chain kernel on stderr)
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python scripts/normals_only.py > gpurun_out/normals_prof.log 2>&1 || { tail -30 gpurun_out/normals_prof.log; exit 1; }
grep -E "^(room|seabed|chain)" gpurun_out/normals_prof.log
