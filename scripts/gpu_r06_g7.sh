set -o pipefail
mkdir -p gpurun_out
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_s5.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06g.log 2>&1; rc=$?; tail -1 gpurun_out/t_r06g.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06g.log | head -20; exit 1; }
bash scripts/gpu_ab_n.sh pcl_feature_extraction_amd/libpfx.so pcl_feature_extraction_amd/libpfx_s5.so pcl_feature_extraction_amd/libpfx_e3.so || exit 1
timeout -k 10 200 python bench.py --workload config1 --no-cpu-baseline > gpurun_out/c1.json 2> gpurun_out/c1.err && python -c "import json; d=json.load(open('gpurun_out/c1.json')); print('config1', d['value'], d['ms_per_step'], d['roofline']['stages_ms_per_step']['fpfh_weight'])"
bash scripts/gpu_pmc_workload.sh r06g shot
