#!/bin/bash
# round 6: packed-float4 chain staging (ds_read_b128 vs b64 + b32) -- tests on that
# build, normals-only + headline A/B -- and the dense line of the default build
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_r06_variant.sh pcl_feature_extraction_amd/libpfx_f4.so r06k || exit 1
timeout -k 10 500 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/bench_dense_r06k.json 2> gpurun_out/bench_dense_r06k.err || { tail -20 gpurun_out/bench_dense_r06k.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_dense_r06k.json')); r=d['roofline']; print('dense', d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], d.get('stages_ms_per_scan'))"
