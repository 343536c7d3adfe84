#!/bin/bash
# GPU-box: kernel + memory-copy trace of a short bench run; the first 1.2 ms of one timed step
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/trace_h -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/trace_h.log 2>&1 || { tail -20 $R/gpurun_out/trace_h.log; exit 1; }
cd $R && python3 scripts/step_timeline_head.py gpurun_out/trace_h 1200
