# round 5: TN GEMM on 32x32x16 MFMAs (modes 11/12) -- fp32 tests, then timing against hb (9/10) and hipBLASLt
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-h32}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/tests 300 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 3 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
TN_MODES=${MODES:-9,10,11,12} run_step r05/$T/bench 400 python -u scripts/bench_gemm_tn_hb.py
grep gemm gpurun_out/r05/$T/bench.log
