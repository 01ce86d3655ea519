# round 5: gate|up weight gradient on the TN kernel (TH_W13_WGRAD_TN=1, default) -- kernel + training GPU tests,
# the per-layer path timing, then an interleaved step A/B against the hipBLASLt path
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-w13}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/tests 600 python -u -m pytest tests/gpu/test_kernels_gpu.py tests/gpu/test_train_gpu.py tests/gpu/test_fullwidth_gpu.py -x -q --timeout 300 --timeout-method thread
tail -n 2 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
run_step r05/$T/paths 200 python -u scripts/bench_w13_wgrad_paths.py
grep '^{' gpurun_out/r05/$T/paths.log
for i in 1 2; do
  for tn in 1 0; do
    TH_W13_WGRAD_TN=$tn run_step r05/$T/bench_tn${tn}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "w13_tn=$tn run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_tn${tn}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_tn${tn}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_tn${tn}_$i.log) $(grep -o '"peak_mem_gib": [0-9.]*' gpurun_out/r05/$T/bench_tn${tn}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
