# round 5: input-gradient GEMM form with the measured GEMM table loaded -- transpose W then NT (TH_DGRAD_NT=1,
# default) against hipBLASLt's NN form on the untransposed weight (TH_DGRAD_NT=0); interleaved step A/B
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-dgrad}; mkdir -p gpurun_out/r05/$T
for i in 1 2; do
  for d in 1 0; do
    TH_DGRAD_NT=$d run_step r05/$T/bench_d${d}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "dgrad_nt=$d run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_d${d}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_d${d}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_d${d}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
