# A/B of the in-tree kernel library against ab_libs/libthk_base.so (same box, alternating processes):
# flash tests on the new library first, then FA backward timings.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
out=gpurun_out/${AB_TAG:-ab}
timeout -k 10 300 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread > ${out}_tests.log 2>&1 || { tail -20 ${out}_tests.log; exit 1; }
tail -1 ${out}_tests.log
for i in 1 2 3; do
  TH_KERNEL_LIB=$PWD/ab_libs/libthk_base.so FA_B=8 FA_FLAGS=0 timeout -k 10 120 python scripts/fa_bwd_ab.py | sed 's/^/base /' >> ${out}.log || exit 1
  FA_B=8 FA_FLAGS=0 timeout -k 10 120 python scripts/fa_bwd_ab.py | sed 's/^/new  /' >> ${out}.log || exit 1
done
cat ${out}.log
