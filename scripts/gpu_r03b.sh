set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "batch or fpfh or harris6d or pipeline or determinism or abi" > gpurun_out/t_r03b.log 2>&1 || { tail -40 gpurun_out/t_r03b.log; exit 1; }
tail -3 gpurun_out/t_r03b.log
timeout -k 10 400 python bench.py --no-cpu-baseline --scans 8 --steps 5 --warmup 2 --no-e2e > gpurun_out/bench_r03b_scans8.json 2> gpurun_out/bench_r03b_scans8.err || { tail -30 gpurun_out/bench_r03b_scans8.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03b_scans8.json')); print(d['value'], d['ms_per_step'], d.get('batch_pipeline'))"
