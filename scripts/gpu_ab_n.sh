#!/bin/bash
# A/B of N library builds on one box: the normal estimation alone (scripts/normals_only.py:
# per-kernel HIP-event times) and the headline bench (value, stage, chain kernels), two rounds,
# alternating.   usage: bash scripts/gpu_ab_n.sh <lib.so> [<lib.so> ...]   (paths relative to the
# repo root; a *_prof.so build prints its phase counters instead of taking part in the bench)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    echo "== $(basename $L) normals_only"
    PFX_LIB=$PWD/$L timeout -k 10 200 python scripts/normals_only.py > gpurun_out/ab_n.log 2>&1 || { tail -30 gpurun_out/ab_n.log; exit 1; }
    grep -E "^(room|seabed)|chain" gpurun_out/ab_n.log
  done
done
for r in 1 2; do
  for L in "$@"; do
    case $L in *_prof.so) continue;; esac
    PFX_LIB=$PWD/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab_n.json 2> gpurun_out/ab_n.err || { tail -30 gpurun_out/ab_n.err; exit 1; }
    echo "bench $(basename $L) $(python -c "import json; d=json.load(open('gpurun_out/ab_n.json')); r=d['roofline']; c=r['chain']; k=r['kernels_ms_per_scan']; print(d['value'], d['ms_per_step'], 'stage', r['avg_ms'], 'chain', c['ms'], c['frac'], 'lists', round(k['normals_lists_small']+k['normals_lists_sparse']+k['normals_lists_dense']+k['normals_lists_query'],4), 'grid', k['grid_build'])")"
  done
done
