#!/bin/bash
# Build a library variant for on-box A/B: every source recompiled with extra defines into its own
# object directory.   usage: bash scripts/build_variant.sh <out-name> <-Ddefines...>
# -> pcl_feature_extraction_amd/<out-name>.so (load it with PFX_LIB=...)
set -e
OUT=$1; shift
cd "$(dirname "$0")/../pcl_feature_extraction_amd/csrc"
D=build_var/$OUT
mkdir -p $D
for f in *.hip; do
  EXTRA=""
  # (the Makefile's per-file flags: pfx_nblist.hip without the atomic optimizer)
  [ "$f" = pfx_nblist.hip ] && EXTRA="-mllvm -amdgpu-atomic-optimizer-strategy=None"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-function \
    -Wno-unused-result -munsafe-fp-atomics $EXTRA "$@" -c $f -o $D/${f%.hip}.o &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 0.2; done
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../$OUT.so $D/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built pcl_feature_extraction_amd/$OUT.so"
