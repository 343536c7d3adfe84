#!/bin/bash
# GPU-box kernel-trace profile of one bench workload: rocprofv3 kernel stats + the trace.
# usage: bash scripts/gpu_prof.sh <tag> [workload]
TAG=${1:-dev}; W=${2:-fpfh}
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -40
