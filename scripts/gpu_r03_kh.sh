# half-width paired dK|dV kernel (flag 256): flash GPU tests, then interleaved A/B against the default at B8 S4096
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_kh
run_step r03_kh/flash_tests 600 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 300 --timeout-method thread
tail -n 3 gpurun_out/r03_kh/flash_tests.log
grep -q " passed" gpurun_out/r03_kh/flash_tests.log && ! grep -q "failed" gpurun_out/r03_kh/flash_tests.log || exit 1
FA_B=8 FA_FLAGS=0,256 run_step r03_kh/ab 300 python scripts/fa_bwd_ab.py
cat gpurun_out/r03_kh/ab.log
