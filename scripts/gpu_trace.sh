#!/bin/bash
# kernel-trace timeline of the bench step (for stream-overlap analysis with scripts/timeline.py)
TAG=${1:-trace}; W=${2:-fpfh}
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.log 2>&1 || { tail -20 $R/gpurun_out/$TAG.log; exit 1; }
python3 $R/scripts/timeline.py $(find $R/gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
