# round 3: TSan sweep (all reports), TSan GPU test, real-node multi-tenant test + harness (device-freed wake)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/tsan_sweep 400 python scripts/tsan_sweep.py
cat gpurun_out/r03/tsan_sweep.log | tail -8
run_step r03/tsan 400 python -u -m pytest tests/gpu/test_native_gpu.py -x -q --timeout 300 --timeout-method thread -k tsan --basetemp gpurun_out/r03/tsan_tmp2
tail -n 2 gpurun_out/r03/tsan.log
run_step r03/mt_test 300 python -u -m pytest tests/gpu/test_multitenant_node_gpu.py -x -q --timeout 200 --timeout-method thread
tail -n 3 gpurun_out/r03/mt_test.log
run_step r03/mt_bench 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
tail -n 1 gpurun_out/r03/mt_bench.log
