#!/bin/bash
# Instruction-cache and issue-stall counters of the normal estimation (scripts/normals_only.py,
# one pass per counter set; kernel-trace only).  usage: bash scripts/gpu_pmc_icache.sh <tag> [lib]
TAG=${1:-dev}; LIB=${2:-}
R=$PWD; mkdir -p gpurun_out/pmc_ic_$TAG
cd /tmp && export TMPDIR=/tmp
P1="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_IFETCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  PFX_LIB=$LIB PFX_NO_STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_ic_$TAG/p$i -o run -- \
    python3 $R/scripts/normals_only.py > $R/gpurun_out/pmc_ic_$TAG/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_ic_$TAG/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_ic_$TAG > $R/gpurun_out/pmc_ic_$TAG/summary.txt
grep -A1 "k_nb_tile\|k_nb_query\|k_normals_chain" $R/gpurun_out/pmc_ic_$TAG/summary.txt | cut -c1-700
