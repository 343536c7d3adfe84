#!/bin/bash
# GPU-box: HIP API trace of a short bench run; the host calls of one step's first 0.9 ms
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/trace_api -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/trace_api.log 2>&1 || { tail -20 $R/gpurun_out/trace_api.log; exit 1; }
cd $R && ls gpurun_out/trace_api && python3 scripts/api_gap.py gpurun_out/trace_api ${1:-900} ${2:-0}
