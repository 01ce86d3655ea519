# round 4: new NT GEMM (tests + bench vs hipBLASLt), MFMA metrics vs PMC (+ coexistence), partial-HBM test
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r04c
run_step r04c/gemm_test 300 python -u -m pytest tests/gpu/test_gemm_nt_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
tail -n 3 gpurun_out/r04c/gemm_test.log
grep -q " passed" gpurun_out/r04c/gemm_test.log && ! grep -q "failed" gpurun_out/r04c/gemm_test.log && run_step r04c/gemm_bench 300 python -u scripts/bench_gemm_nt.py
cat gpurun_out/r04c/gemm_bench.log | grep gemm | cut -c1-220
run_step r04c/probe_vs_pmc 900 python -u scripts/probe_vs_pmc.py gpurun_out/r04c/probe_vs_pmc
tail -n 6 gpurun_out/r04c/probe_vs_pmc.log
run_step r04c/pytest_new 900 python -u -m pytest tests/gpu/test_remote_telemetry_gpu.py tests/gpu/test_mfma_metrics_gpu.py tests/gpu/test_probe_gpu.py tests/gpu/test_native_gpu.py -v -m gpu --timeout 300 --timeout-method thread
tail -n 12 gpurun_out/r04c/pytest_new.log
