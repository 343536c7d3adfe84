#!/bin/bash
# GPU-box iteration: parity suite, FPFH alone (per-stage times), headline line.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python scripts/fpfh_only.py > gpurun_out/fpfh_only.log 2>&1 || { tail -30 gpurun_out/fpfh_only.log; exit 1; }
cat gpurun_out/fpfh_only.log | grep libpfx
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_head.json 2> gpurun_out/b_head.err || { tail -30 gpurun_out/b_head.err; exit 1; }
cut -c1-300 gpurun_out/b_head.json
