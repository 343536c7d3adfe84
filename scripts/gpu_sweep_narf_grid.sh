#!/bin/bash
# Sweep of the NARF flood-fill grid (PFX_FF_WAVES waves per CU for k_interest_ff) on the headline
# step: NARF shares the device with
# the critical normal-estimation stream, so the step time, not the NARF stage time, decides.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "narf" > gpurun_out/sw_t.log 2>&1 || { tail -30 gpurun_out/sw_t.log; exit 1; }
tail -1 gpurun_out/sw_t.log
for i in 1 2; do
for cfg in "4 512" "3 512" "6 512"; do
  set -- $cfg
  PFX_FF_WAVES=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -30 gpurun_out/sw.err; exit 1; }
  echo "ff=$1 $(cut -c80-150 gpurun_out/sw.json)"
done
done
