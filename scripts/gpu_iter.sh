#!/bin/bash
# GPU-box iteration: all parity tests, the instrumented build's phase cycles, both bench lines.
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for w in fpfh shot; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/bp_$w.log 2>&1 || { tail -30 gpurun_out/bp_$w.log; exit 1; }
  grep cycles gpurun_out/bp_$w.log
  PFX_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.log 2>&1 || { tail -30 gpurun_out/b_$w.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/b_$w.log | cut -c1-250
done
