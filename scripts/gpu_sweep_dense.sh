#!/bin/bash
# Dense-variant line (10M points) against the dense / sparse tile chunk
mkdir -p gpurun_out
for cfg in "2 1" "2 2" "2 4" "4 4"; do
  set -- $cfg
  PFX_TILE_CHUNK_P=$1 PFX_TILE_CHUNK_D=$2 timeout -k 10 400 python bench.py --workload dense --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_sd.json 2> gpurun_out/b_sd.err || { tail -30 gpurun_out/b_sd.err; exit 1; }
  echo "P=$1 D=$2 dense $(python3 -c "import json;d=json.load(open('gpurun_out/b_sd.json'));print(d['value'],d['ms_per_step'])")"
done
