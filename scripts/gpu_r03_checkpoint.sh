# round 3 checkpoint on the current tree: whole GPU suite, smoke, the driver's bench line (20 steps), a step profile
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03c
run_step r03c/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 3 gpurun_out/r03c/pytest.log
run_step r03c/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -n 1 gpurun_out/r03c/smoke.log
run_step r03c/bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r03c/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03c/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $GRAFT_REPO_ROOT/gpurun_out/r03c/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/step_summary.py gpurun_out/r03c/prof/run_kernel_stats.csv --steps 3 > gpurun_out/r03c/step_summary.txt; head -18 gpurun_out/r03c/step_summary.txt
