# two in-process library A/Bs, 40 rounds each: (1) in-tree (fwd softmax split) vs HEAD; (2) HEAD vs pre-interleave kh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1 || { tail -20 gpurun_out/ab2_tests.log; exit 1; }
tail -1 gpurun_out/ab2_tests.log
AB_ROUNDS=40 AB_BASE_LIB=$PWD/ab_libs/libthk_head.so timeout -k 10 400 python scripts/lib_ab.py > gpurun_out/ab2_fwdsplit.log 2>&1 || exit 1
cat gpurun_out/ab2_fwdsplit.log
AB_ROUNDS=40 TH_KERNEL_LIB=$PWD/ab_libs/libthk_head.so AB_BASE_LIB=$PWD/ab_libs/libthk_preint.so timeout -k 10 400 python scripts/lib_ab.py > gpurun_out/ab2_khint.log 2>&1 || exit 1
cat gpurun_out/ab2_khint.log
