# half-width paired dK|dV kernel: step-level A/B (TH_FA_BWD_FLAGS 0 vs 256), PMC of the flash kernels with it, step profile
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_kh
AB_VAR=TH_FA_BWD_FLAGS AB_A=0 AB_B=256 bash scripts/gpu_ab_env_step.sh || exit 1
FA_BWD_FLAGS=256 timeout -k 10 400 bash scripts/pmc_session.sh scripts/flash_pmc.py > gpurun_out/r03_kh/pmc_kh.txt 2>&1 || { tail gpurun_out/r03_kh/pmc_kh.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
TH_FA_BWD_FLAGS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03_kh/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $GRAFT_REPO_ROOT/gpurun_out/r03_kh/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/step_summary.py $(ls gpurun_out/r03_kh/prof/*/run_kernel_stats.csv gpurun_out/r03_kh/prof/run_kernel_stats.csv 2>/dev/null | head -1) --steps 3 > gpurun_out/r03_kh/step_summary.txt; head -20 gpurun_out/r03_kh/step_summary.txt
