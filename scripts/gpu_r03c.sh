set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -k "normals_fast" > gpurun_out/t_r03c.log 2>&1; rc=$?
tail -25 gpurun_out/t_r03c.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload fastnormals --no-e2e --steps 10 > gpurun_out/bench_fast.json 2> gpurun_out/bench_fast.err || { tail -30 gpurun_out/bench_fast.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_fast.json'))
print(d['value'], d['ms_per_step']); r=d['roofline']; print(json.dumps({k:r[k] for k in ('avg_ms','frac','kernels_ms_per_scan','mfma_kernel','isolated')}))
print(json.dumps(d['deviation_from_parity_path']))"
