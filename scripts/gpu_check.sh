#!/bin/bash
# GPU-box check: parity tests, a verbose bench line, a rocprofv3 kernel-trace summary.
# usage (from the repo root, via gpurun): bash scripts/gpu_check.sh [profile-tag]
TAG=${1:-dev}
R=$PWD; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
PFX_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
cat gpurun_out/b.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1
