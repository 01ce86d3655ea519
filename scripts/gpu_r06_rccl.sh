# round 6: the multi-rank code path on real RCCL with every round-6 change -- a one-rank process group that still
# issues every reduce-scatter / all-gather (TH_FORCE_COLLECTIVES=1, ZeRO-1), launched by torchrun like the driver
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-rccl}; O=gpurun_out/r06/$T; mkdir -p $O
TH_FORCE_COLLECTIVES=1 run_step r06/$T/bench_torchrun 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 8 --warmup 3 --daemon-bench 0
grep '^{' $O/bench_torchrun.log | python3 -c '
import sys, json
d = json.loads(sys.stdin.readline())
print(d["value"], d["ms_per_step"], d["config"]["zero"], d["config"]["optimizer"], d["exposed_comm_ms_per_step"], d["dist"]["backend"], d["dist"]["comm"].get("rccl"), d["dist"]["comm_env"].get("TENSILE_STREAMK_DATA_PARALLEL"))'
