cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
run_step r02b_newtests 400 python -u -m pytest tests/gpu/test_fullwidth_gpu.py tests/gpu/test_hbm_counter_gpu.py tests/gpu/test_native_gpu.py tests/gpu/test_telemetry_calibration_gpu.py -v -s --timeout 300 --timeout-method thread
run_step r02b_bench_default 300 python bench.py --daemon-bench 0
TH_GRAD_FP32=1 run_step r02b_bench_gradfp32 300 python bench.py --daemon-bench 0
tail -n 3 gpurun_out/r02b_bench_default.log gpurun_out/r02b_bench_gradfp32.log
