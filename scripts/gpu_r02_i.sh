# one-barrier paired dK|dV kernel (flags 128): numerics first, then interleaved timing A/B
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02i_flash_tests 500 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/r02i_flash_tests.log
grep -q " passed" gpurun_out/r02i_flash_tests.log && ! grep -q "failed" gpurun_out/r02i_flash_tests.log || exit 1
FA_FLAGS=${AB_FLAGS:-0,128} run_step r02i_ab 300 python scripts/fa_bwd_ab.py
cat gpurun_out/r02i_ab.log | grep flags
