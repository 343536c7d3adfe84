#!/bin/bash
# round 6: GPU tests, the headline line (CPU baseline included) and the configs[1] / SHOT lines
# usage: bash scripts/gpu_r06_lines.sh <tag>
set -o pipefail
TAG=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -1 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_$TAG.log | head -20; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); r=d['roofline']; c=d['cpu_baseline']; print('headline', d['value'], d['ms_per_step'], 'stage', r['avg_ms'], r['frac'], 'chain', r['chain']['frac'], 'stages', d.get('stages_ms_per_scan'), 'parity', d.get('parity_all_scans'), 'cpu', c['value'], c.get('all_single_threaded'))"
for w in config1 shot; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_${w}_$TAG.json 2> gpurun_out/bench_${w}_$TAG.err || { tail -20 gpurun_out/bench_${w}_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${w}_$TAG.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['kernel'][:40], r['avg_ms'], r['frac'], d.get('stages_ms_per_scan'), (d.get('cpu_baseline') or {}).get('parity'))"
done
