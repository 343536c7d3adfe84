#!/bin/bash
# A/B of two library builds on one box: pcl_feature_extraction_amd/libpfx_base.so (a build of the
# previous commit) vs pcl_feature_extraction_amd/libpfx.so (the working tree): the normal
# estimation alone (scripts/normals_only.py: per-kernel HIP-event times) and the headline bench,
# two pairs each, alternating.  usage: bash scripts/gpu_ab2.sh [extra helper script]
set -o pipefail
mkdir -p gpurun_out
BASE=$PWD/pcl_feature_extraction_amd/libpfx_base.so
NEW=$PWD/pcl_feature_extraction_amd/libpfx.so
for L in $BASE $NEW $BASE $NEW; do
  echo "== $(basename $L)"
  PFX_LIB=$L timeout -k 10 200 python scripts/normals_only.py 2>&1 | tail -2 || exit 1
  if [ -n "$1" ]; then PFX_LIB=$L timeout -k 10 200 python $1 2>&1 | tail -3 || exit 1; fi
done
for i in 1 2; do
for v in base new; do
  if [ $v = base ]; then L=$BASE; else L=$NEW; fi
  PFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -20 gpurun_out/b_ab.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/b_ab.json')); r=d['roofline']; k=r['kernels_ms_per_scan']; print(d['value'], d['ms_per_step'], r['avg_ms'], json.dumps(k))")"
done
done
