# round 5: step A/B of the edited TunableOp table (w13 input-gradient entry back to Default), interleaved, one box
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tune4}; mkdir -p gpurun_out/r05/$T
for i in 1 2 3; do
  for tu in 0 1; do
    TH_GEMM_TUNED=$tu run_step r05/$T/bench_tuned${tu}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "gemm_tuned=$tu run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_tuned${tu}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_tuned${tu}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
