set -o pipefail
# headline A/B over an environment switch: bash scripts/gpu_ab_env.sh VAR "v1 v2" [pytest -k expr]
VAR=$1; VALS=$2; K=$3
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 200 --timeout-method thread > gpurun_out/t_env.log 2>&1 || { tail -30 gpurun_out/t_env.log; exit 1; }
  tail -1 gpurun_out/t_env.log
fi
for i in 1 2 3; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_e.json 2> gpurun_out/b_e.err || { tail -20 gpurun_out/b_e.err; exit 1; }
  echo "$VAR=$v $(python -c "import json; d=json.load(open('gpurun_out/b_e.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_ms'])")"
done
done
