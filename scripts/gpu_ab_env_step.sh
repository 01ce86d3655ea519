# same-box A/B of one environment variable on the full training step: runs alternate A, B, A, B
# usage: AB_VAR=NAME AB_A=value AB_B=value bash scripts/gpu_ab_env_step.sh
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$AB_A" "$AB_B"; do
    run_step ab_step_${AB_VAR}_${v}_$i 400 env $AB_VAR=$v python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "$AB_VAR=$v $(grep -h metric gpurun_out/ab_step_${AB_VAR}_${v}_$i.log | python -c 'import sys,json; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
