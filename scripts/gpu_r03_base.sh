# round-3 baseline on the round-2 HEAD: GPU tests, smoke, bench with the driver's command line
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
run_step r03/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run_step r03/bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
tail -n 3 gpurun_out/r03/pytest_gpu.log gpurun_out/r03/smoke.log; grep metric gpurun_out/r03/bench.log | tail -1
