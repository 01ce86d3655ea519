# round-end rehearsal: GPU tests, smoke, default bench (with the daemon bench), as the driver runs them
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02z_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run_step r02z_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run_step r02z_bench 600 python bench.py
tail -n 2 gpurun_out/r02z_pytest_gpu.log gpurun_out/r02z_smoke.log; grep metric gpurun_out/r02z_bench.log | tail -1
