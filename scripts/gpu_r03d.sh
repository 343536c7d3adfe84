set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_r03d.log 2>&1 || { tail -30 gpurun_out/t_r03d.log; exit 1; }
tail -1 gpurun_out/t_r03d.log
for w in fpfh fastnormals shot; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || { tail -30 gpurun_out/b_$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['frac'], r.get('avg_ms'), json.dumps(r.get('kernels_ms_per_scan')), d.get('end_to_end_h2d_d2h',{}) and d['end_to_end_h2d_d2h']['value'])"
done
timeout -k 10 300 python bench.py --scans 8 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/b_s8.json 2> gpurun_out/b_s8.err || { tail -30 gpurun_out/b_s8.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_s8.json')); print('scans8', d['value'], d['ms_per_step'], json.dumps(d.get('batch_pipeline')))"
