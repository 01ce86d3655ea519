# A/B of the in-tree kernel library against ab_libs/libthk_base.so: flash GPU tests on the new
# library, then scripts/lib_ab.py (both libraries in one process, interleaved rounds).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
out=gpurun_out/${AB_TAG:-ab}
timeout -k 10 300 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread > ${out}_tests.log 2>&1 || { tail -20 ${out}_tests.log; exit 1; }
tail -1 ${out}_tests.log
AB_BASE_LIB=$PWD/ab_libs/libthk_base.so timeout -k 10 300 python scripts/lib_ab.py > ${out}.log 2>&1
rc=$?; cat ${out}.log; exit $rc
