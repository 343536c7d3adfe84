#!/bin/bash
# GPU-box iteration: full parity suite, then normal estimation alone (instrumented phases + timings).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash scripts/gpu_phases.sh
