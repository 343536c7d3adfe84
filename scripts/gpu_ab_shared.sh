#!/bin/bash
# A/B of the headline step: NARF flood fill at 20 waves per CU (PFX_FF_WAVES=20, the pre-hint
# shape) vs the default (4 when the context is marked shared), three times each, after the
# NARF/pipeline parity tests
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "narf or pipeline or determinism or fullsize" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2 3; do
  PFX_FF_WAVES=20 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
  echo "ff20 $(cut -c80-150 gpurun_out/b_ab.json)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -30 gpurun_out/b_ab.err; exit 1; }
  echo "default $(cut -c80-150 gpurun_out/b_ab.json)"
done
