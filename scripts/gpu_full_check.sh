#!/bin/bash
# full GPU parity suite, the default bench line twice (no CPU leg), one step's kernel timeline
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1 || { tail -30 gpurun_out/t_full.log; exit 1; }
tail -1 gpurun_out/t_full.log
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }; cut -c80-150 gpurun_out/b_ab.json; done
bash scripts/gpu_step_trace.sh
