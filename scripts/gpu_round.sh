#!/bin/bash
# Round evidence on the GPU box: parity tests, the default bench line (with the CPU baseline),
# the secondary lines, a rocprofv3 kernel-trace summary and the PMC HBM-traffic passes.
# usage: bash scripts/gpu_round.sh <tag>
TAG=${1:-r01}
R=$PWD; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
for w in shot match iss harris harris6d config1 fastnormals demand; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_${w}_$TAG.json 2> gpurun_out/bench_${w}_$TAG.err || { tail -30 gpurun_out/bench_${w}_$TAG.err; exit 1; }
done
timeout -k 10 400 python bench.py --scans 8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_scans8_$TAG.json 2> gpurun_out/bench_scans8_$TAG.err || { tail -30 gpurun_out/bench_scans8_$TAG.err; exit 1; }
timeout -k 10 400 python bench.py --workload dense --steps 3 --warmup 1 > gpurun_out/bench_dense_$TAG.json 2> gpurun_out/bench_dense_$TAG.err || { tail -30 gpurun_out/bench_dense_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_iss_$TAG -o run -- python3 $R/bench.py --workload iss --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_iss_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_iss_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_match_$TAG -o run -- python3 $R/bench.py --workload match --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_match_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_match_$TAG.log; exit 1; }
cd $R && bash scripts/gpu_pmc.sh $TAG || exit 1
# the dense variant's normal estimation alone, per kernel (round 6)
cd /tmp && PFX_NO_SCENES=dense PFX_NO_STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dense_$TAG -o run -- python3 $R/scripts/normals_only.py > $R/gpurun_out/prof_dense_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_dense_$TAG.log; exit 1; }
echo round evidence done
