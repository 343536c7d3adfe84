#!/bin/bash
# GPU-box: device idle time at the step boundary of the overlapped pass, per host-side variant
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-base norows notimer sync}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gap_$m -o run -- python3 $R/scripts/gap_probe.py $m > $R/gpurun_out/gap_$m.log 2>&1 || { tail -5 $R/gpurun_out/gap_$m.log; exit 1; }
  echo "$m: $(python3 $R/scripts/gap_probe.py --report $R/gpurun_out/gap_$m/run_kernel_trace.csv)"
done
