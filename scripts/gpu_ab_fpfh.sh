set -o pipefail
# FPFH stage A/B: libpfx_base.so (previous commit) vs libpfx.so (working tree) and any extra
# variants given as library paths; FPFH parity tests on the working tree first
mkdir -p gpurun_out
B=$PWD/pcl_feature_extraction_amd
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "fpfh or config1" --timeout 200 --timeout-method thread > gpurun_out/t_fpfh.log 2>&1 || { tail -30 gpurun_out/t_fpfh.log; exit 1; }
tail -1 gpurun_out/t_fpfh.log
for i in 1 2; do
for L in $B/libpfx_base.so $B/libpfx.so "$@"; do
  PFX_LIB=$L timeout -k 10 200 python scripts/fpfh_only.py || exit 1
done
done
for L in $B/libpfx_base.so $B/libpfx.so; do
  PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_f.json 2> gpurun_out/b_f.err || { tail -20 gpurun_out/b_f.err; exit 1; }
  echo "$(basename $L) $(python -c "import json; d=json.load(open('gpurun_out/b_f.json')); print(d['value'], d['ms_per_step'])")"
done
