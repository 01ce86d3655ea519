# round-3 last tree: the driver's three GPU tiers (pytest -m gpu, smoke, bench) plus bench.py launched the way the
# driver launches N > 1 (torch.distributed.run, one rank per GPU) with every RCCL collective forced on one GPU
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03g
run_step r03g/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
tail -n 3 gpurun_out/r03g/pytest.log
run_step r03g/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -n 1 gpurun_out/r03g/smoke.log
run_step r03g/bench_default 600 python bench.py
grep metric gpurun_out/r03g/bench_default.log | cut -c1-300
run_step r03g/bench_20 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r03g/bench_20.log | cut -c1-300
run_step r03g/bench_torchrun_rccl 600 env TH_DIST_BACKEND=nccl TH_FORCE_COLLECTIVES=1 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --steps 8 --warmup 3
grep metric gpurun_out/r03g/bench_torchrun_rccl.log | cut -c1-400
