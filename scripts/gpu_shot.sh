#!/bin/bash
# GPU-box SHOT iteration: parity tests, the instrumented build's phase cycles, the shot bench line.
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_shot.py tests/test_gpu_fullsize.py tests/test_facade.py -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python bench.py --workload shot --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/bp.log 2>&1 || { tail -30 gpurun_out/bp.log; exit 1; }
grep phase gpurun_out/bp.log
PFX_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --workload shot --no-cpu-baseline > gpurun_out/bs.log 2>&1 || { tail -30 gpurun_out/bs.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bs.log | cut -c1-330
