# round 3: the one-wave-per-SIMD NT GEMM (w1) against the ping-pong kernel and hipBLASLt
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/gemm_w1 600 python -u scripts/bench_gemm_nt_variants.py
grep -h '"gemm"\|Error\|assert' gpurun_out/r03/gemm_w1.log; tail -3 gpurun_out/r03/gemm_w1.log
