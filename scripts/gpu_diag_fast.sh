# timing of the opt-in MFMA normal estimation alone (2 runs), then its GPU tests
for i in 1 2; do timeout -k 10 120 python scripts/normals_fast_only.py || exit 1; done
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "normals_fast" 2>&1 | tail -3
