# TN GEMM mode 9 (LDS-staged epilogue): TN GPU tests, per-shape A/B against mode 6, step A/B
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_tn
run_step r03_tn/tests 600 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 1 gpurun_out/r03_tn/tests.log
grep -q " passed" gpurun_out/r03_tn/tests.log && ! grep -q failed gpurun_out/r03_tn/tests.log || exit 1
TN_PP=6,9,6,9 TN_ALL_SPLITK=0 run_step r03_tn/bench 300 python scripts/bench_gemm_tn.py
cat gpurun_out/r03_tn/bench.log | grep gemm
ROUNDS=2 CONFIGS="TH_GEMM_TN_PP=6;TH_GEMM_TN_PP=9" bash scripts/gpu_env_matrix.sh
