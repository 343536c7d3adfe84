#!/bin/bash
# round 6: the 4k list tier -- held to 8 waves per SIMD (shipped) against 6, and without the
# record prefetch; dense + room normal estimation alone (tests on each variant first)
set -o pipefail
mkdir -p gpurun_out
for V in q6 nopf; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_$V.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06p_$V.log 2>&1; rc=$?
  echo "tests $V rc=$rc"; tail -1 gpurun_out/t_r06p_$V.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06p_$V.log | head -30; exit 1; }
done
for r in 1 2; do
  for L in "" q6 nopf; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  done
done
