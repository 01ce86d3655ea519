# rotary of Q folded into the flash forward: flash GPU tests (incl. fused-vs-separate forward), the
# attention/training tests, in-process kernel A/B (plain forward: must be unchanged), and the step A/B via
# TH_FA_ROPE_FWD (the backward fusion stays on in both arms)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_ropefwd
run_step r03_ropefwd/tests 600 python -u -m pytest tests/gpu/test_flash_attn_gpu.py tests/gpu/test_train_gpu.py -x -q --timeout 200 --timeout-method thread
tail -n 2 gpurun_out/r03_ropefwd/tests.log
grep -q " passed" gpurun_out/r03_ropefwd/tests.log && ! grep -q failed gpurun_out/r03_ropefwd/tests.log || exit 1
AB_ROUNDS=24 AB_BASE_LIB=$PWD/ab_libs/libthk_base.so run_step r03_ropefwd/ab 300 python scripts/lib_ab.py
grep op gpurun_out/r03_ropefwd/ab.log
ROUNDS=3 CONFIGS="TH_FA_ROPE_FWD=0;TH_FA_ROPE_FWD=1" bash scripts/gpu_env_matrix.sh
