# step profile of the current tree (rocprofv3 kernel trace + stats of bench.py --steps 2 --warmup 1)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03p
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03p/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $GRAFT_REPO_ROOT/gpurun_out/r03p/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/step_summary.py gpurun_out/r03p/prof/run_kernel_stats.csv --steps 3 > gpurun_out/r03p/step_summary.txt; head -18 gpurun_out/r03p/step_summary.txt
