# round 5: finish the TunableOp table (shapes the first pass did not reach), survey with it, then an interleaved
# step A/B of the trainer with the table (TH_GEMM_TUNED=1) against the library defaults
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tune2}; mkdir -p gpurun_out/r05/$T
( while true; do date >> gpurun_out/r05/$T/heartbeat.txt; sleep 30; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TH_TUNE_KINDS=fwd,dgrad TH_TUNED_FILE=$R/tensorhive_fixed_amd/ops/tuned/gemm_gfx950_t32768.csv
run_step r05/$T/resume 900 python -u scripts/gemm_tune.py resume
cp $TH_TUNED_FILE gpurun_out/r05/$T/
run_step r05/$T/check 300 python -u scripts/gemm_tune.py check
grep gemm_ms_per_step gpurun_out/r05/$T/check.log
for i in 1 2; do
  for tu in 0 1; do
    TH_GEMM_TUNED=$tu run_step r05/$T/bench_tuned${tu}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "gemm_tuned=$tu run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_tuned${tu}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_tuned${tu}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_tuned${tu}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
