#!/bin/bash
# Partial round evidence after a matching-only library change: GPU tests, the matching line, its
# kernel profile, and the PMC passes (re-tagged with the new library hash).  usage: <tag>
TAG=${1:-dev}
R=$PWD; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 400 python bench.py --workload match > gpurun_out/bench_match_$TAG.json 2> gpurun_out/bench_match_$TAG.err || { tail -30 gpurun_out/bench_match_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_match_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_match_$TAG -o run -- python3 $R/bench.py --workload match --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_match_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_match_$TAG.log; exit 1; }
cd $R && bash scripts/gpu_pmc.sh $TAG
