# round 3 checkpoint: the whole GPU suite, smoke, the driver's bench line, on the current tree
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/full_pytest 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
run_step r03/full_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run_step r03/full_bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
tail -n 5 gpurun_out/r03/full_pytest.log; tail -1 gpurun_out/r03/full_smoke.log; grep metric gpurun_out/r03/full_bench.log | cut -c1-600
