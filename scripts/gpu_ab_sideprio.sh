#!/bin/bash
# A/B: the normals' forked long-list stream at the caller stream's priority vs default priority
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "normals or pipeline or determinism" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2 3; do
  PFX_SIDE_NOPRIO=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_sp.json 2> gpurun_out/b_sp.err || { tail -30 gpurun_out/b_sp.err; exit 1; }
  echo "noprio $(cut -c80-150 gpurun_out/b_sp.json)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_sp.json 2> gpurun_out/b_sp.err || { tail -30 gpurun_out/b_sp.err; exit 1; }
  echo "inherit $(cut -c80-150 gpurun_out/b_sp.json)"
done
