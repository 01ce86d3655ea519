# round 5: per-shape XCD band heights for the TN kernel (TH_GEMM_TN_BAND_POLICY=1, default) -- TN + training GPU
# tests, the band sweep on the final kernel, then an interleaved step A/B against the compiled default band
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-band}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/tests 600 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py tests/gpu/test_train_gpu.py -x -q --timeout 300 --timeout-method thread
tail -n 2 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
run_step r05/$T/sweep 300 python -u scripts/tn_band_sweep.py
grep '^{' gpurun_out/r05/$T/sweep.log
for i in 1 2; do
  for p in 1 0; do
    TH_GEMM_TN_BAND_POLICY=$p run_step r05/$T/bench_p${p}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "band_policy=$p run=$i $(grep -o '"value": [0-9.]*' gpurun_out/r05/$T/bench_p${p}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_p${p}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r05/$T/bench_p${p}_$i.log)"
  done
done | tee gpurun_out/r05/$T/ab.txt
