#!/bin/bash
# round 6: kernel trace of the dense step (FPFH weighting passes)
set -o pipefail
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_densestep2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_densestep2 -o run -- python3 $R/bench.py --workload dense --steps 2 --warmup 1 > $R/gpurun_out/prof_densestep2.log 2>&1 || { tail -20 $R/gpurun_out/prof_densestep2.log; exit 1; }
echo trace done
