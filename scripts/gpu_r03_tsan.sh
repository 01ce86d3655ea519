cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh; mkdir -p gpurun_out/r03/tsan
run_step r03/tsan_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/gpu/test_native_gpu.py -k tsan
TSAN_OPTIONS="log_path=$PWD/gpurun_out/r03/tsan/tsan:halt_on_error=0:second_deadlock_stack=1" timeout -k 10 120 setarch x86_64 -R tensorhive_fixed_amd/native/bin/thsmi-stress-tsan --iters 20 > gpurun_out/r03/tsan/stress.out 2>&1
echo "stress rc=$?"; ls gpurun_out/r03/tsan; head -c 4000 gpurun_out/r03/tsan/tsan* 2>/dev/null
