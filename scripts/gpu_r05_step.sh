# round 5: step A/B of the TN default (mode 10) against round 4's (mode 6), then a step kernel profile
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-step1}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/head_wgrad 200 python -u scripts/bench_head_wgrad.py
cat gpurun_out/r05/$T/head_wgrad.log | grep chunk
for i in 1 2; do
  for pp in 6 10 10h; do
    HT=0; [ "$pp" = "10h" ] && HT=1
    TH_HEAD_WGRAD_TN=$HT TH_GEMM_TN_PP=${pp%h} run_step r05/$T/bench_pp${pp}_$i 300 python bench.py --steps 10 --warmup 3 --daemon-bench 0
    echo "pp=$pp run=$i $(grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/r05/$T/bench_pp${pp}_$i.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05/$T/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --daemon-bench 0 > $R/gpurun_out/r05/$T/prof.log 2>&1 || exit 1
cd $R && python3 scripts/step_summary.py $(ls gpurun_out/r05/$T/prof/*kernel_stats.csv | head -1) --steps 4 > gpurun_out/r05/$T/step_summary.txt 2>&1; head -16 gpurun_out/r05/$T/step_summary.txt
