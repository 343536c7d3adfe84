#!/bin/bash
# GPU-box: parity suite, then the configs[1] and dense-variant bench lines.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
PFX_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --workload config1 > gpurun_out/b_config1.json 2> gpurun_out/b_config1.err || { tail -30 gpurun_out/b_config1.err; exit 1; }
cut -c1-1500 gpurun_out/b_config1.json
PFX_BENCH_VERBOSE=1 timeout -k 10 400 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/b_dense.json 2> gpurun_out/b_dense.err || { tail -30 gpurun_out/b_dense.err; exit 1; }
cut -c1-2500 gpurun_out/b_dense.json
grep -E "per-step|stats" gpurun_out/b_dense.err | cut -c1-1500
