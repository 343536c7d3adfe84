#!/bin/bash
# The normal-estimation stream at high priority (default now) against the flood-fill width
mkdir -p gpurun_out
for i in 1 2; do
for ff in 4 8 20; do
  PFX_FF_WAVES=$ff timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_pr.json 2> gpurun_out/b_pr.err || { tail -30 gpurun_out/b_pr.err; exit 1; }
  echo "ff=$ff $(cut -c80-150 gpurun_out/b_pr.json)"
done
done
