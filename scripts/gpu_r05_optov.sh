# round 5: overlapped optimizer (side stream, default) vs in-line, interleaved A/B on one box
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-optov}; mkdir -p gpurun_out/r05/$T
for i in 1 2; do
  for ov in 1 0; do
    TH_OPT_OVERLAP=$ov run_step r05/$T/bench_ov${ov}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "opt_overlap=$ov run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_ov${ov}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_ov${ov}_$i.log) $(grep -o '"opt_wait_ms": [0-9.]*' gpurun_out/r05/$T/bench_ov${ov}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
