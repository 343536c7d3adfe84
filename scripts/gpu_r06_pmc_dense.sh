#!/bin/bash
# round 6: L1 -> L2 request and L2 hit counters of the dense normal estimation (k_normals_long's
# per-neighbour gathers), one --pmc pass, kernel trace only
set -o pipefail
R=$PWD; mkdir -p gpurun_out/pmc_dense
cd /tmp && export TMPDIR=/tmp
PFX_NO_SCENES=dense PFX_NO_STEPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum --output-format csv -d $R/gpurun_out/pmc_dense/p1 -o run -- python3 $R/scripts/normals_only.py > $R/gpurun_out/pmc_dense/p1.log 2>&1 || { tail -20 $R/gpurun_out/pmc_dense/p1.log; exit 1; }
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_dense > $R/gpurun_out/pmc_dense/summary.txt
grep -A1 "k_normals_long\|k_normals_chain_big\|k_nb_query<4096" $R/gpurun_out/pmc_dense/summary.txt | cut -c1-700
