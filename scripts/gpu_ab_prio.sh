#!/bin/bash
# A/B of the normals-stream priority in the overlapped step (bench line, twice each)
mkdir -p gpurun_out
for i in 1 2; do
for P in 0 -1; do
  PFX_NORMALS_PRIORITY=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_prio.json 2> gpurun_out/b_prio.err || { tail -30 gpurun_out/b_prio.err; exit 1; }
  echo "prio $P $(cut -c1-160 gpurun_out/b_prio.json)"
done
done
