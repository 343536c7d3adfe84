set -o pipefail
# A/B of two library builds: gpurun_tmp/libpfx_base.so (the previous build, copied there before
# rebuilding) vs pcl_feature_extraction_amd/libpfx.so (the working tree).  Optional first argument:
# a helper script run under both (e.g. scripts/fpfh_only.py); then the headline bench, 3 pairs.
mkdir -p gpurun_out
BASE=$PWD/gpurun_tmp/libpfx_base.so
NEW=$PWD/pcl_feature_extraction_amd/libpfx.so
if [ -n "$1" ]; then
  for L in $BASE $NEW $BASE $NEW; do
    PFX_LIB=$L timeout -k 10 200 python $1 2>&1 | tail -2 || exit 1
  done
fi
for i in 1 2 3; do
for v in base new; do
  if [ $v = base ]; then L=$BASE; else L=$NEW; fi
  PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_l.json 2> gpurun_out/b_l.err || { tail -20 gpurun_out/b_l.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/b_l.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_ms'])")"
done
done
