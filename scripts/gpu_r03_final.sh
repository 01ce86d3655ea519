# round-3 final tree: the driver's three GPU tiers as it runs them (pytest -m gpu, smoke, bench), then a step profile
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03f
run_step r03f/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 3 gpurun_out/r03f/pytest.log
run_step r03f/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -n 1 gpurun_out/r03f/smoke.log
run_step r03f/bench_default 600 python bench.py
grep metric gpurun_out/r03f/bench_default.log | cut -c1-300
run_step r03f/bench_20 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r03f/bench_20.log | cut -c1-300
