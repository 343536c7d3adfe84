#!/bin/bash
# PMC passes over the opt-in MFMA normal estimation alone (scripts/normals_fast_only.py)
R=$PWD; mkdir -p gpurun_out/pmcf
timeout -k 10 120 python3 scripts/normals_fast_only.py || exit 1
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
P3="FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmcf/p$i -o run -- \
    python3 $R/scripts/normals_fast_only.py > $R/gpurun_out/pmcf/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmcf/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcf k_normals_mfma $R/gpurun_out/pmcf/pmc_fast.json > $R/gpurun_out/pmcf/summary.txt
head -12 $R/gpurun_out/pmcf/summary.txt
