# headline step with and without the live per-kernel HIP-event timers (twice each)
for i in 1 2; do
for v in "" 1; do
  PFX_BENCH_NO_TIMING=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_t.json 2> gpurun_out/b_t.err || { tail -20 gpurun_out/b_t.err; exit 1; }
  echo "no_timing=$v $(python -c "import json; d=json.load(open('gpurun_out/b_t.json')); print(d['value'], d['ms_per_step'])")"
done
done
