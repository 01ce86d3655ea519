cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
run_step r02_probe 120 python -u -m pytest tests/gpu/test_telemetry_calibration_gpu.py -x -v -s --timeout 100 --timeout-method thread
run_step r02_hbmcal 120 python -u scripts/hbm_calibrate.py
run_step r02_smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run_step r02_bench 400 python bench.py
tail -1 gpurun_out/r02_bench.log
