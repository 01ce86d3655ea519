# round 5: gradient-norm sums of squares per bucket during backward (TH_OPT_SUMSQ_EARLY=1) -- training and
# DDP GPU tests (the forced-collectives one-rank RCCL path waits on each bucket's collective from the side
# stream), then an interleaved step A/B against the one pass after backward
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-sumsq}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/tests 600 python -u -m pytest tests/gpu/test_train_gpu.py tests/gpu/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread
tail -n 2 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
for i in 1 2; do
  for e in 1 0; do
    TH_OPT_SUMSQ_EARLY=$e run_step r05/$T/bench_e${e}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "sumsq_early=$e run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_e${e}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_e${e}_$i.log) $(grep -o '"opt_wait_ms": [0-9.]*' gpurun_out/r05/$T/bench_e${e}_$i.log | head -n 1) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_e${e}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
