#!/bin/bash
# PMC passes (separate runs, kernel-trace only) over one step of a secondary workload, summarised
# per kernel: e.g. the SHOT stage's VALU issue and HBM traffic.  usage: <tag> <workload>
TAG=${1:-dev}; W=${2:-shot}
R=$PWD; mkdir -p gpurun_out/pmc_${W}_$TAG
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_${W}_$TAG/p$i -o run -- \
    python3 $R/bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_${W}_$TAG/p$i.log 2>&1 || exit 1
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_${W}_$TAG > $R/gpurun_out/pmc_${W}_$TAG/summary.txt
grep -A1 "k_shot\|k_match" $R/gpurun_out/pmc_${W}_$TAG/summary.txt | cut -c1-400
