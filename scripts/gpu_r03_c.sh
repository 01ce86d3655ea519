# round 3: HBM counter GPU tests, rccl-bench both modes, TSan on the GPU; training step with and
# without the in-task counter tool (its overhead), 10 steps each
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/c_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/gpu/test_hbm_counter_gpu.py tests/gpu/test_native_gpu.py
run_step r03/c_bench_tool 600 env ROCP_TOOL_LIBRARIES=$PWD/tensorhive_fixed_amd/native/lib/libthhbm.so \
  TH_HBM_OUT=$PWD/gpurun_out/r03/c_bench_tool_hbm.json python bench.py --steps 10 --warmup 3 --daemon-bench 0
run_step r03/c_bench_plain 600 python bench.py --steps 10 --warmup 3 --daemon-bench 0
tail -n 25 gpurun_out/r03/c_tests.log; grep -h metric gpurun_out/r03/c_bench_*.log | cut -c1-300; cat gpurun_out/r03/c_bench_tool_hbm.json | cut -c1-400
