# round 5: hb-only TN file -- full GPU suite, then a 20-step bench
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tnfinal}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 2 gpurun_out/r05/$T/pytest.log
grep -q " passed" gpurun_out/r05/$T/pytest.log && ! grep -q "failed" gpurun_out/r05/$T/pytest.log || exit 1
run_step r05/$T/bench_20 500 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r05/$T/bench_20.log | cut -c1-200
