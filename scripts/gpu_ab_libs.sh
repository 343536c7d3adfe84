set -o pipefail
# A/B/... of library builds: bash scripts/gpu_ab_libs.sh <helper.py or -> <lib.so> <lib.so> ...
# (the helper, e.g. scripts/fpfh_only.py, runs twice per library; then the headline bench, 3 rounds)
mkdir -p gpurun_out
H=$1; shift
if [ "$H" != "-" ]; then
  for i in 1 2; do for L in "$@"; do
    PFX_LIB=$L timeout -k 10 200 python $H 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
  done; done
fi
for i in 1 2 3; do
  for L in "$@"; do
    PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_l.json 2> gpurun_out/b_l.err || { tail -20 gpurun_out/b_l.err; exit 1; }
    echo "$(basename $L) $(python -c "import json; d=json.load(open('gpurun_out/b_l.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_ms'])")"
  done
done
