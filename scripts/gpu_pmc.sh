#!/bin/bash
# GPU-box PMC collection (separate --pmc passes, kernel-trace only; MI355X_MICROARCH.md "rocprofv3
# PMC slots") over one bench step.  usage: bash scripts/gpu_pmc.sh <tag>
TAG=${1:-dev}
R=$PWD; mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $R/gpurun_out/pmc_$TAG/p$i -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_$TAG/p$i.log 2>&1 || exit 1
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_$TAG k_normals_chain,k_normals_chain_big $R/gpurun_out/pmc_$TAG/pmc_normals_chain.json > $R/gpurun_out/pmc_$TAG/summary.txt
# the whole neighbour-gather stage (grid kernels excluded: shared with the FPFH grid in the step)
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_$TAG k_tile_class,k_nb_tile,k_nb_wide,k_nb_query,k_normals_chain,k_normals_chain_big,k_normals_long $R/gpurun_out/pmc_$TAG/pmc_normals_stage.json > /dev/null
cat $R/gpurun_out/pmc_$TAG/summary.txt
