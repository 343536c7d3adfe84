set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06a.log 2>&1; rc=$?; tail -3 gpurun_out/t_r06a.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06a.log | head -30; exit 1; }
timeout -k 10 200 python scripts/normals_only.py > gpurun_out/no_r06a.log 2>&1 && grep -E "^(room|seabed)" gpurun_out/no_r06a.log
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so PFX_NO_STEPS=5 timeout -k 10 200 python scripts/normals_only.py > gpurun_out/noprof_r06a.log 2>&1 && grep -E "cycles|chain" gpurun_out/noprof_r06a.log | head -20
