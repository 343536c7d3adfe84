mkdir -p gpurun_out
for i in 1 2; do for W in 12 16 20; do
PFX_LIB=$PWD/pcl_feature_extraction_amd/libpfx_w$W.so timeout -k 10 200 python scripts/fpfh_only.py > gpurun_out/ab_f.log 2>&1 || { tail -30 gpurun_out/ab_f.log; exit 1; }
echo "w$W $(grep libpfx gpurun_out/ab_f.log)"
done; done
