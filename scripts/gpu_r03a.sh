set -o pipefail
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r03a.log 2>&1 || { tail -30 gpurun_out/t_r03a.log; exit 1; }
tail -1 gpurun_out/t_r03a.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || { tail -30 gpurun_out/bench_r03a.err; exit 1; }
cut -c1-600 gpurun_out/bench_r03a.json
