#!/bin/bash
# round 6: where the dense variant's normal estimation spends its time -- per-kernel HIP events
# and list-tier counts (normals_only.py, dense scene), the phase counters of the profiling build,
# and a rocprofv3 kernel trace of the same run
set -o pipefail
mkdir -p gpurun_out
export PFX_NO_SCENES=dense PFX_NO_STEPS=3
timeout -k 10 300 python scripts/normals_only.py > gpurun_out/dense_no.log 2>&1 || { tail -30 gpurun_out/dense_no.log; exit 1; }
cat gpurun_out/dense_no.log
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python scripts/normals_only.py > gpurun_out/dense_prof.log 2>&1 || { tail -30 gpurun_out/dense_prof.log; exit 1; }
grep -E "cycles|^dense" gpurun_out/dense_prof.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PFX_NO_STEPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dense -o run -- python scripts/normals_only.py > gpurun_out/dense_rocprof.log 2>&1 || { tail -30 gpurun_out/dense_rocprof.log; exit 1; }
f=$(ls gpurun_out/prof_dense/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find gpurun_out/prof_dense -name "*kernel_stats.csv" | head -1)
cut -c1-220 "$f" | head -25
