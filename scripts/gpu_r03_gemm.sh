# round 3: NT GEMM variants vs hipBLASLt; HBM counter GPU tests again (ready handshake)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/gemm_variants 600 python -u scripts/bench_gemm_nt_variants.py
run_step r03/hbm_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/gpu/test_hbm_counter_gpu.py
run_step r03/native_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/gpu/test_native_gpu.py
grep -h '"gemm"' gpurun_out/r03/gemm_variants.log; tail -5 gpurun_out/r03/gemm_variants.log; tail -n 12 gpurun_out/r03/hbm_tests.log gpurun_out/r03/native_tests.log
