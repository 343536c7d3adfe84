set -o pipefail
# dense (10M) and headline A/B: libpfx_base.so (previous commit) vs libpfx.so (working tree);
# the every-list-path parity test on the working tree first
mkdir -p gpurun_out
B=$PWD/pcl_feature_extraction_amd
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "every_list or speculative or radius" --timeout 200 --timeout-method thread > gpurun_out/t_dense.log 2>&1 || { tail -30 gpurun_out/t_dense.log; exit 1; }
tail -1 gpurun_out/t_dense.log
for L in $B/libpfx_base.so $B/libpfx.so; do
  PFX_LIB=$L timeout -k 10 400 python bench.py --workload dense --steps 2 --warmup 1 > gpurun_out/b_d.json 2> gpurun_out/b_d.err || { tail -20 gpurun_out/b_d.err; exit 1; }
  echo "$(basename $L) dense $(python -c "import json; d=json.load(open('gpurun_out/b_d.json')); r=d['roofline']; k=r['isolated']['kernels_ms']; print(d['value'], d['ms_per_step'], {a: b for a, b in k.items() if 'lists' in a or 'long' in a})")"
  PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_l.json 2> gpurun_out/b_l.err || { tail -20 gpurun_out/b_l.err; exit 1; }
  echo "$(basename $L) head $(python -c "import json; d=json.load(open('gpurun_out/b_l.json')); r=d['roofline']; k=r['isolated']['kernels_ms']; print(d['value'], d['ms_per_step'], {a: b for a, b in k.items() if 'lists' in a})")"
done
