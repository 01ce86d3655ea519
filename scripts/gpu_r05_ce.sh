# round 5: LM-head chunk A/B (TH_CE_CHUNK 4096 vs 8192 vs 16384 tokens per logits chunk), interleaved, one box
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-ce}; mkdir -p gpurun_out/r05/$T
for i in 1 2; do
  for ch in 4096 8192 16384; do
    TH_CE_CHUNK=$ch run_step r05/$T/bench_ce${ch}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "chunk=$ch run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_ce${ch}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_ce${ch}_$i.log) $(grep -o '"peak_mem_gib": [0-9.]*' gpurun_out/r05/$T/bench_ce${ch}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
