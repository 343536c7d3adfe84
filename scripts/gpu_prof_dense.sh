#!/bin/bash
# rocprofv3 kernel-trace summary of the dense (10M) workload: which list tier costs what
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dense -o run -- python3 $R/bench.py --workload dense --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_dense.log 2>&1 || { tail -20 $R/gpurun_out/prof_dense.log; exit 1; }
head -14 $R/gpurun_out/prof_dense/run_kernel_stats.csv | cut -d, -f1-8
