#!/bin/bash
# GPU-box: kernel trace of a short bench run and the timeline of one timed step
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/trace.log 2>&1 || { tail -20 $R/gpurun_out/trace.log; exit 1; }
cd $R && python3 scripts/step_timeline.py gpurun_out/trace/run_kernel_trace.csv
