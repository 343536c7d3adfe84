#!/bin/bash
# A/B helper: build the committed HEAD's library into pcl_feature_extraction_amd/libpfx_base.so
# (a temporary git worktree; the working tree is untouched).   usage: bash scripts/build_base.sh [rev]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/pfx_base.XXXXXX)
git -C "$ROOT" worktree add -q "$WT" "$REV"
make -C "$WT/pcl_feature_extraction_amd/csrc" -j8 > /dev/null 2>&1
cp "$WT/pcl_feature_extraction_amd/libpfx.so" "$ROOT/pcl_feature_extraction_amd/libpfx_base.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built pcl_feature_extraction_amd/libpfx_base.so from $(git -C "$ROOT" rev-parse --short "$REV")"
