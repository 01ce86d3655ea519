# round-end rehearsal with the driver's own command lines: GPU tests, smoke, bench --steps 20 --warmup 5
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02y_pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu
run_step r02y_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run_step r02y_bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
tail -n 2 gpurun_out/r02y_pytest_gpu.log gpurun_out/r02y_smoke.log; grep metric gpurun_out/r02y_bench.log | tail -1
