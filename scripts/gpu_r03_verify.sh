# round-3 last code change: GPU suite + smoke on the final tree
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03v
run_step r03v/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 3 gpurun_out/r03v/pytest.log
run_step r03v/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -n 1 gpurun_out/r03v/smoke.log
run_step r03v/bench_20 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r03v/bench_20.log | cut -c1-300
