# rocprof kernel-trace of the default training step (2 timed + 1 warmup step)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r02v8_prof
export TMPDIR=/tmp
run_step r02v8_prof 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02v8_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --daemon-bench 0
find gpurun_out/r02v8_prof -name "*kernel_stats.csv" | head -3
python3 scripts/step_summary.py $(find gpurun_out/r02v8_prof -name "*kernel_stats.csv" | head -1) 3 > gpurun_out/r02v8_summary.txt 2>&1; tail -40 gpurun_out/r02v8_summary.txt
