mkdir -p gpurun_out
timeout -k 10 300 python scripts/narf_stats.py > gpurun_out/narf_stats.log 2>&1 || { tail -30 gpurun_out/narf_stats.log; exit 1; }
grep sparse gpurun_out/narf_stats.log
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python scripts/narf_only.py > gpurun_out/narf_prof.log 2>&1 || { tail -30 gpurun_out/narf_prof.log; exit 1; }
grep -E "cycles" gpurun_out/narf_prof.log | tail -2
