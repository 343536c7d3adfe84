set -o pipefail
bash scripts/gpu_ab_env.sh PFX_NORMALS_SPLIT "0 1" "pipeline" || exit 1
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_prof.so timeout -k 10 300 python bench.py --workload shot --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/shotprof.json 2> gpurun_out/shotprof.err || { tail -5 gpurun_out/shotprof.err; exit 1; }
grep "shot phase" gpurun_out/shotprof.err | tail -2
