set -o pipefail
# A/B of the normals stage's host round trips: PFX_NORMALS_SYNC=1 (grid bounds readback + list
# readback before the chains) vs the default (speculative grid + deferred list check), and the
# deferred check on exact bounds (PFX_GRID_NOHINT=1)
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
fi
for i in 1 2 3; do
for v in sync spec defer; do
  case $v in
    sync) e="PFX_NORMALS_SYNC=1";;
    spec) e="PFX_AB_DUMMY=1";;
    defer) e="PFX_NORMALS_DEFER=1";;
  esac
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_s.json 2> gpurun_out/b_s.err || { tail -20 gpurun_out/b_s.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/b_s.json')); r=d['roofline']; k=r['kernels_ms_per_scan']; print(d['value'], d['ms_per_step'], r['frac'], r['avg_ms'], k.get('grid_bbox'), k.get('grid_build'))")"
done
done
