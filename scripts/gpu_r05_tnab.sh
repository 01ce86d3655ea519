# round 5: TN hb (mode 9) -- GPU tests, then an interleaved step A/B against mode 6 on one box
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; mkdir -p gpurun_out/r05/tnab
run_step r05/tnab/pytest 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_gemm_tn_gpu.py
tail -n 2 gpurun_out/r05/tnab/pytest.log
for i in 1 2; do
  for pp in 6 9; do
    TH_GEMM_TN_PP=$pp run_step r05/tnab/bench_pp${pp}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "pp=$pp run=$i $(grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/r05/tnab/bench_pp${pp}_$i.log)"
  done
done
