set -o pipefail
# headline A/B over environment settings, 3 rounds: bash scripts/gpu_ab_env.sh "A=0 B=1" "A=1 B=1" ...
# (each argument: one configuration, space-separated VAR=value pairs)
mkdir -p gpurun_out
for i in 1 2 3; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_env.json 2> gpurun_out/b_env.err || { tail -20 gpurun_out/b_env.err; exit 1; }
    echo "[$cfg] $(python -c "import json; d=json.load(open('gpurun_out/b_env.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'])")"
  done
done
