#!/bin/bash
# Full GPU parity suite, then the list-building bench lines (no CPU legs)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cl_t.log 2>&1 || { tail -30 gpurun_out/cl_t.log; exit 1; }
tail -1 gpurun_out/cl_t.log
for w in fpfh config1 harris harris6d iss shot; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/b_cl.json 2> gpurun_out/b_cl.err || { tail -30 gpurun_out/b_cl.err; exit 1; }
  echo "$w $(python3 -c "import json;d=json.load(open('gpurun_out/b_cl.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 400 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/b_cl.json 2> gpurun_out/b_cl.err || { tail -30 gpurun_out/b_cl.err; exit 1; }
echo "dense $(python3 -c "import json;d=json.load(open('gpurun_out/b_cl.json'));print(d['value'],d['ms_per_step'])")"
