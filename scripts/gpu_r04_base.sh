# round-4 start: GPU suite after the trust fixes + a 20-step bench
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r04a
run_step r04a/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 5 gpurun_out/r04a/pytest.log
run_step r04a/bench_20 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r04a/bench_20.log | cut -c1-300
