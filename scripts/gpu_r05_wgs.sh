# round 5: weight-gradient GEMMs on a side stream (TH_WGRAD_STREAM=1) -- training / DDP GPU tests with it on,
# then an interleaved step A/B against the default
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-wgs}; mkdir -p gpurun_out/r05/$T
TH_WGRAD_STREAM=1 run_step r05/$T/tests 600 python -u -m pytest tests/gpu/test_train_gpu.py tests/gpu/test_fullwidth_gpu.py tests/gpu/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread
tail -n 2 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
for i in 1 2; do
  for ws in 0 1; do
    TH_WGRAD_STREAM=$ws run_step r05/$T/bench_ws${ws}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "wgrad_stream=$ws run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_ws${ws}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_ws${ws}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_ws${ws}_$i.log) $(grep -o '"peak_mem_gib": [0-9.]*' gpurun_out/r05/$T/bench_ws${ws}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
