# round 5 baseline on a fresh box: 20-step bench + step kernel profile of the r04 final tree
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-base}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/bench_20 600 python bench.py --gpus 1 --steps 20 --warmup 5
grep metric gpurun_out/r05/$T/bench_20.log | cut -c1-260
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05/$T/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --daemon-bench 0 > $R/gpurun_out/r05/$T/prof.log 2>&1 || exit 1
cd $R && python3 scripts/step_summary.py $(ls gpurun_out/r05/$T/prof/*kernel_stats.csv | head -1) --steps 4 > gpurun_out/r05/$T/step_summary.txt 2>&1; head -24 gpurun_out/r05/$T/step_summary.txt
