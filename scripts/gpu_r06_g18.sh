#!/bin/bash
# round 6: the dense variant's bench line and the headline line on the current build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/bench_dense_r06q.json 2> gpurun_out/bench_dense_r06q.err || { tail -20 gpurun_out/bench_dense_r06q.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_dense_r06q.json')); r=d['roofline']; print('dense', d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], d.get('stages_ms_per_scan')); print(r.get('kernels_ms_per_scan'))"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_head_r06q.json 2> gpurun_out/bench_head_r06q.err || { tail -20 gpurun_out/bench_head_r06q.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_head_r06q.json')); r=d['roofline']; print('head', d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], r['chain']['frac'], d.get('stages_ms_per_scan')); print(r.get('kernels_ms_per_scan'))"
