mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_s4.log 2>&1 || { tail -30 gpurun_out/t_s4.log; exit 1; }
tail -1 gpurun_out/t_s4.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_s4.json 2> gpurun_out/b_s4.err || { tail -30 gpurun_out/b_s4.err; exit 1; }
cut -c1-200 gpurun_out/b_s4.json
timeout -k 10 300 python scripts/normals_only.py > gpurun_out/normals_only_s4.log 2>&1 || { tail -30 gpurun_out/normals_only_s4.log; exit 1; }
grep -E "^(room|seabed)" gpurun_out/normals_only_s4.log
timeout -k 10 300 python scripts/narf_only.py > gpurun_out/narf_only_s4.log 2>&1 || { tail -30 gpurun_out/narf_only_s4.log; exit 1; }
tail -5 gpurun_out/narf_only_s4.log
timeout -k 10 300 python scripts/fpfh_only.py > gpurun_out/fpfh_only_s4.log 2>&1 || { tail -30 gpurun_out/fpfh_only_s4.log; exit 1; }
tail -5 gpurun_out/fpfh_only_s4.log
