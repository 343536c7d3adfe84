#!/bin/bash
# GPU-box quick iteration: the full parity suite (or a -k selection), then normal estimation
# alone with per-kernel HIP-event times.   usage: bash scripts/gpu_quick.sh [pytest -k expr]
mkdir -p gpurun_out
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread "${K[@]}" > gpurun_out/tq.log 2>&1 || { tail -40 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
timeout -k 10 300 python scripts/normals_only.py > gpurun_out/normals_only.log 2>&1 || { tail -30 gpurun_out/normals_only.log; exit 1; }
grep -E "^(room|seabed)" gpurun_out/normals_only.log
