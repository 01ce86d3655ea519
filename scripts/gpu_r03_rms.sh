# wave-per-row RMSNorm forward: kernel GPU tests, isolated A/B (two processes each way), step A/B
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_rms
run_step r03_rms/tests 300 python -u -m pytest tests/gpu/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k rmsnorm
tail -n 1 gpurun_out/r03_rms/tests.log
grep -q " passed" gpurun_out/r03_rms/tests.log && ! grep -q failed gpurun_out/r03_rms/tests.log || exit 1
for i in 1 2; do for v in 0 1; do TH_RMS_WAVE=$v timeout -k 10 120 python scripts/bench_rmsnorm_fwd.py || exit 1; done; done
ROUNDS=2 CONFIGS="TH_RMS_WAVE=0;TH_RMS_WAVE=1" bash scripts/gpu_env_matrix.sh
