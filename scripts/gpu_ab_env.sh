#!/bin/bash
# A/B of an environment switch VAR (0 vs 1): parity tests (-k $3) under VAR=1, then fpfh_only.py
# and the headline bench line under both settings.  usage: gpu_ab_env.sh VAR "test filter"
V=$1; K=${2:-fpfh or pipeline or fullsize or determinism or golden}
mkdir -p gpurun_out
export $V=1
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for i in 1 2; do
for s in 0 1; do
  export $V=$s
  timeout -k 10 200 python scripts/fpfh_only.py > gpurun_out/ab_f.log 2>&1 || { tail -30 gpurun_out/ab_f.log; exit 1; }
  echo "$V=$s $(grep libpfx gpurun_out/ab_f.log)"
done
done
for s in 0 1; do
  export $V=$s
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab$s.json 2> gpurun_out/b_ab$s.err || { tail -30 gpurun_out/b_ab$s.err; exit 1; }
  echo "$V=$s $(cut -c1-200 gpurun_out/b_ab$s.json)"
  timeout -k 10 300 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/b_ab1$s.json 2> gpurun_out/b_ab1$s.err || { tail -30 gpurun_out/b_ab1$s.err; exit 1; }
  echo "$V=$s config1 $(cut -c1-200 gpurun_out/b_ab1$s.json)"
done
