cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02c_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run_step r02c_bench 300 python bench.py --daemon-bench 0
cd /tmp && export TMPDIR=/tmp
run_step r02c_prof 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02c_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --daemon-bench 0
cd $GRAFT_REPO_ROOT
tail -n 3 gpurun_out/r02c_pytest_gpu.log gpurun_out/r02c_bench.log
