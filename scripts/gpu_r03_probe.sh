# round 3: per-GPU th-probe agent + self-pid exclusion (verdict item 1), native/protection GPU
# tests, and the device-counting experiment with tenant queue profiling on (verdict item 3)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/probe_tests 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/gpu/test_probe_gpu.py tests/gpu/test_native_gpu.py tests/gpu/test_protection_gpu.py
run_step r03/counters_env 300 bash scripts/counters_env_probe.sh
tail -n 15 gpurun_out/r03/probe_tests.log; grep -c . gpurun_out/r03/counters_env/avail.txt
