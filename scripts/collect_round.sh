#!/bin/bash
# Copy a round's GPU evidence (scripts/gpu_round.sh <tag>) from gpurun_out/ into profiles/.
# (referenced from DESIGN.md section 9: the evidence files each round commits)
T=$1
cp gpurun_out/bench_$T.json profiles/${T}_bench_fpfh_line.json
for w in shot match iss harris harris6d config1 fastnormals demand scans8 dense; do cp gpurun_out/bench_${w}_$T.json profiles/${T}_bench_${w}_line.json; done
cp gpurun_out/prof_$T/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
cp gpurun_out/prof_iss_$T/run_kernel_stats.csv profiles/${T}_iss_kernel_stats.csv
cp gpurun_out/prof_match_$T/run_kernel_stats.csv profiles/${T}_match_kernel_stats.csv
cp gpurun_out/pmc_$T/summary.txt profiles/${T}_pmc_summary.txt
cp gpurun_out/pmc_$T/pmc_normals_stage.json profiles/pmc_normals_stage.json
cp gpurun_out/pmc_$T/pmc_normals_chain.json profiles/pmc_normals_chain.json
cp gpurun_out/t_$T.log profiles/${T}_pytest_gpu.log
[ -f gpurun_out/prof_dense_$T/run_kernel_stats.csv ] && cp gpurun_out/prof_dense_$T/run_kernel_stats.csv profiles/${T}_dense_normals_kernel_stats.csv
[ -f gpurun_out/prof_dense_$T.log ] && grep -E "^(dense)" gpurun_out/prof_dense_$T.log > profiles/${T}_dense_normals_only.txt
