set -o pipefail
# A/B of two library builds on the headline bench and the normals-only stage timing:
# libpfx_base.so (the previous commit) vs libpfx.so (the working tree)
mkdir -p gpurun_out
B=$PWD/pcl_feature_extraction_amd
for i in 1 2 3; do
for v in base new; do
  if [ $v = base ]; then L=$B/libpfx_base.so; else L=$B/libpfx.so; fi
  PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_l.json 2> gpurun_out/b_l.err || { tail -20 gpurun_out/b_l.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/b_l.json')); r=d['roofline']; k=r['isolated']['kernels_ms']; print(d['value'], d['ms_per_step'], r['avg_ms'], {a: b for a, b in k.items() if 'lists' in a})")"
done
done
