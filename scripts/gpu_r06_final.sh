#!/bin/bash
# round 6: the driver's round-end sequence on the committed tree -- smoke(), then the default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_final.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['chain']['frac'], (r.get('traffic_source') or {}).get('same_build_as_this_run'), d['cpu_baseline'].get('parity'))"
