#!/bin/bash
# A/B: blocking hipStreamSynchronize (PFX_SYNC_BLOCK=1) vs polled event for the grid-bbox and
# list-builder readbacks; parity tests first, then the headline and the ISS / Harris lines
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "normals or pipeline or determinism or radius or fpfh" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2 3; do
  PFX_SYNC_BLOCK=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_sy.json 2> gpurun_out/b_sy.err || { tail -30 gpurun_out/b_sy.err; exit 1; }
  echo "block $(cut -c80-150 gpurun_out/b_sy.json)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_sy.json 2> gpurun_out/b_sy.err || { tail -30 gpurun_out/b_sy.err; exit 1; }
  echo "spin $(cut -c80-150 gpurun_out/b_sy.json)"
done
for w in config1 harris iss; do
for m in block spin; do
  if [ $m = block ]; then export PFX_SYNC_BLOCK=1; else unset PFX_SYNC_BLOCK; fi
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_sy.json 2> gpurun_out/b_sy.err || { tail -30 gpurun_out/b_sy.err; exit 1; }
  echo "$w $m $(python3 -c "import json;d=json.load(open('gpurun_out/b_sy.json'));print(d['value'],d['ms_per_step'])")"
done
done
