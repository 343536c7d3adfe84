#!/bin/bash
# Sweep of the list builder's tiles per queue fetch per tile class (PFX_TILE_CHUNK_S / _P / _D:
# small / sparse / dense tiles) on the headline step and the other list-building lines
mkdir -p gpurun_out
for cfg in "4 4 4" "4 2 2" "4 2 1" "4 1 2" "2 2 2" "8 2 2" "2 4 4"; do
  set -- $cfg
  for w in fpfh harris config1; do
    PFX_TILE_CHUNK_S=$1 PFX_TILE_CHUNK_P=$2 PFX_TILE_CHUNK_D=$3 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_sw.json 2> gpurun_out/b_sw.err || { tail -30 gpurun_out/b_sw.err; exit 1; }
    echo "$cfg $w $(python3 -c "import json;d=json.load(open('gpurun_out/b_sw.json'));print(d['value'],d['ms_per_step'])")"
  done
done
