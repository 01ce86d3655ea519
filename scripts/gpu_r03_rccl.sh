# round 3: the collective path on one GPU (one-rank RCCL group issuing every collective, ZeRO-1 and ZeRO-0) against
# the plain step, alternating; then a kernel trace of the ZeRO-1 run to see what the collectives cost in the step
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03_rccl
for i in 1 2; do
  run_step r03_rccl/plain_$i 300 python bench.py --gpus 1 --steps 10 --warmup 3 --daemon-bench 0
  TH_FORCE_COLLECTIVES=1 run_step r03_rccl/zero1_$i 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2961$i bench.py --gpus 1 --steps 10 --warmup 3 --daemon-bench 0 --zero 1
  TH_FORCE_COLLECTIVES=1 run_step r03_rccl/zero0_$i 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2962$i bench.py --gpus 1 --steps 10 --warmup 3 --daemon-bench 0 --zero 0
done
for f in gpurun_out/r03_rccl/*.log; do echo "$f $(grep -h '"metric"' $f | python -c 'import sys,json; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["zero"])')"; done
cd /tmp && export TMPDIR=/tmp
TH_FORCE_COLLECTIVES=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03_rccl/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 2 --warmup 1 --daemon-bench 0 --zero 1 > $GRAFT_REPO_ROOT/gpurun_out/r03_rccl/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03_rccl/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/step_summary.py gpurun_out/r03_rccl/prof/run_kernel_stats.csv --steps 3 | head -20
