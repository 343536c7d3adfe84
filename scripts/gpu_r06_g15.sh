#!/bin/bash
# round 6: dense normal estimation -- the shipped build (chunk prefetch in the wide tiles) against
# the lane-cap x4, the 1024-thread 8k-tier and the dense-tile chunk prefetch variants (tests on both variants first), then a rocprofv3 kernel trace of the
# shipped build on the dense scene
set -o pipefail
mkdir -p gpurun_out
for V in "" ld4 m8w dpf; do
  PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx${V:+_$V}.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r06n_$V.log 2>&1; rc=$?
  echo "tests $V rc=$rc"; tail -1 gpurun_out/t_r06n_$V.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_r06n_$V.log | head -30; exit 1; }
done
for r in 1 2; do
  for L in "" ld4 m8w dpf; do
    lib=pcl_feature_extraction_amd/libpfx${L:+_$L}.so
    echo "== $(basename $lib)"
    PFX_LIB=$PWD/$lib PFX_NO_SCENES=dense,room PFX_NO_STEPS=2 timeout -k 10 300 python scripts/normals_only.py > gpurun_out/ab_d.log 2>&1 || { tail -30 gpurun_out/ab_d.log; exit 1; }
    grep -E "^(dense|room)" gpurun_out/ab_d.log | cut -c1-330
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_dense2
PFX_NO_SCENES=dense PFX_NO_STEPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dense2 -o run -- python scripts/normals_only.py > gpurun_out/dense_rocprof2.log 2>&1 || { tail -30 gpurun_out/dense_rocprof2.log; exit 1; }
echo rocprof done
