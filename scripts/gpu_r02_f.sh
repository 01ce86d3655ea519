# RCCL one-rank collective path: the DDP check (pytest) and the full 8B step under torchrun with ZeRO-1
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02f_ddp 400 python -u -m pytest tests/gpu/test_ddp_gpu.py -v -s --timeout 300 --timeout-method thread
TH_FORCE_COLLECTIVES=1 run_step r02f_bench_rccl_zero1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 5 --warmup 2 --daemon-bench 0 --zero 1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r02f_ddp.log | tail -4
grep metric gpurun_out/r02f_bench_rccl_zero1.log | tail -1
