#!/bin/bash
# PMC passes over the SHOT workload (configs[3]); summary of the SHOT kernels
R=$PWD; mkdir -p gpurun_out/pmc_shot
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_shot/p$i -o run -- \
    python3 $R/bench.py --workload shot --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_shot/p$i.log 2>&1 || exit 1
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_shot > gpurun_out/pmc_shot/summary.txt && grep -A1 "k_shot" gpurun_out/pmc_shot/summary.txt
