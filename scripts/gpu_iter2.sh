#!/bin/bash
# GPU-box iteration: parity tests, verbose bench lines (fpfh, shot, match), normals alone.
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for w in fpfh shot match; do
  PFX_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.log 2>&1 || { tail -30 gpurun_out/b_$w.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/b_$w.log | cut -c1-300
done
timeout -k 10 300 python scripts/normals_only.py > gpurun_out/normals_only.log 2>&1 || { tail -30 gpurun_out/normals_only.log; exit 1; }
cat gpurun_out/normals_only.log
