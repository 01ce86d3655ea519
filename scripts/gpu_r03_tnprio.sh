# TN GEMM pp2 with s_setprio over the compute slot: TN GPU tests on the new library, per-shape A/B (two processes
# per library, alternating), then the step A/B through TH_KERNEL_LIB
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_tn
run_step r03_tn/tests_prio 600 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 1 gpurun_out/r03_tn/tests_prio.log
grep -q " passed" gpurun_out/r03_tn/tests_prio.log && ! grep -q failed gpurun_out/r03_tn/tests_prio.log || exit 1
for i in 1 2; do
  for lib in base tnprio; do
    TH_KERNEL_LIB=$PWD/ab_libs/libthk_$lib.so TN_PP=6 TN_ALL_SPLITK=0 timeout -k 10 200 python scripts/bench_gemm_tn.py > gpurun_out/r03_tn/bench_${lib}_$i.log 2>&1 || exit 1
    echo "$lib $i $(python scripts/tn_bench_summary.py gpurun_out/r03_tn/bench_${lib}_$i.log)"
  done
done
ROUNDS=2 CONFIGS="TH_KERNEL_LIB=$PWD/ab_libs/libthk_base.so;TH_KERNEL_LIB=$PWD/ab_libs/libthk_tnprio.so" bash scripts/gpu_env_matrix.sh
