set -o pipefail
# k_shot_hist occupancy variants (PFX_SHOT_HIST_WG builds): SHOT stage time on the configs[3] line
mkdir -p gpurun_out
B=$PWD/pcl_feature_extraction_amd
for i in 1 2; do
for L in libpfx.so libpfx_s3.so libpfx_s4.so; do
  PFX_LIB=$B/$L timeout -k 10 300 python bench.py --workload shot --no-cpu-baseline --no-e2e > gpurun_out/b_sw.json 2> gpurun_out/b_sw.err || { tail -20 gpurun_out/b_sw.err; exit 1; }
  echo "$L $(python -c "import json; d=json.load(open('gpurun_out/b_sw.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_ms'])")"
done
done
