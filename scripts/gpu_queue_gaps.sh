#!/bin/bash
# GPU-box: kernel trace of a short headline bench run, per-queue dispatch sequence of one step
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/qtrace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/qtrace.log 2>&1 || { tail -20 $R/gpurun_out/qtrace.log; exit 1; }
cd $R && python3 scripts/queue_gaps.py gpurun_out/qtrace/run_kernel_trace.csv > gpurun_out/queue_gaps.txt && head -5 gpurun_out/queue_gaps.txt
