# same-box step A/B over environment settings: CONFIGS="A=1 B=2;A=3;..." (one bench.py run each, in order, ROUNDS times)
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/envm
IFS=';' read -ra CFG <<< "$CONFIGS"
for r in $(seq 1 ${ROUNDS:-1}); do
  i=0
  for c in "${CFG[@]}"; do
    i=$((i+1))
    run_step envm/r${r}_c$i ${STEP_LIMIT:-300} env $c python bench.py --steps ${STEPS:-8} --warmup 3 --daemon-bench 0
    echo "[$c] $(grep -h metric gpurun_out/envm/r${r}_c$i.log | python -c 'import sys,json; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
