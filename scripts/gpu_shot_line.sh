set -o pipefail
# configs[3] line after a parity pass over the SHOT / pipeline tests
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "shot or pipeline" --timeout 300 --timeout-method thread > gpurun_out/t_shot.log 2>&1 || { tail -30 gpurun_out/t_shot.log; exit 1; }
tail -1 gpurun_out/t_shot.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload shot --no-cpu-baseline --no-e2e > gpurun_out/b_sh.json 2> gpurun_out/b_sh.err || { tail -20 gpurun_out/b_sh.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_sh.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_ms'])"
done
