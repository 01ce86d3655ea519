# rotary backward folded into the dQ / dK epilogues: flash GPU tests (incl. fused-vs-separate), the attention+rope
# test, in-process kernel A/B (plain backward: must be unchanged), and the step A/B via TH_FA_ROPE_FUSED
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_rope
run_step r03_rope/tests 600 python -u -m pytest tests/gpu/test_flash_attn_gpu.py -x -q --timeout 200 --timeout-method thread
tail -n 2 gpurun_out/r03_rope/tests.log
grep -q " passed" gpurun_out/r03_rope/tests.log && ! grep -q failed gpurun_out/r03_rope/tests.log || exit 1
AB_ROUNDS=24 AB_BASE_LIB=$PWD/ab_libs/libthk_base.so run_step r03_rope/ab 300 python scripts/lib_ab.py
cat gpurun_out/r03_rope/ab.log | grep op
ROUNDS=3 CONFIGS="TH_FA_ROPE_FUSED=0;TH_FA_ROPE_FUSED=1" bash scripts/gpu_env_matrix.sh
