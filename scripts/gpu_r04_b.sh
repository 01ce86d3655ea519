# round 4: new GPU tests (remote agent, partial HBM, profile task), probe vs PMC, forced-RCCL bench
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r04b
run_step r04b/pytest_new 600 python -u -m pytest tests/gpu/test_remote_telemetry_gpu.py tests/gpu/test_hbm_counter_gpu.py -v -m gpu --timeout 300 --timeout-method thread
tail -n 8 gpurun_out/r04b/pytest_new.log
run_step r04b/probe_vs_pmc 900 python -u scripts/probe_vs_pmc.py gpurun_out/r04b/probe_vs_pmc
tail -n 6 gpurun_out/r04b/probe_vs_pmc.log
TH_FORCE_COLLECTIVES=1 run_step r04b/bench_rccl 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --daemon-bench 0
grep metric gpurun_out/r04b/bench_rccl.log | cut -c1-600
cp /tmp/th-rccl-init-*.log gpurun_out/r04b/ 2>/dev/null; true
