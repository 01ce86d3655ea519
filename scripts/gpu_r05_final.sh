# round 5: final tree -- full GPU suite, smoke, 20-step bench (PART=1); step kernel profile + MFMA-busy PMC (PART=2)
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-final}; mkdir -p gpurun_out/r05/$T
if [ "${PART:-1}" = "1" ]; then
  run_step r05/$T/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
  tail -n 4 gpurun_out/r05/$T/pytest.log
  run_step r05/$T/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -n 1 gpurun_out/r05/$T/smoke.log
  run_step r05/$T/bench_20 500 python bench.py --gpus 1 --steps 20 --warmup 5
  grep metric gpurun_out/r05/$T/bench_20.log | cut -c1-300
else
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05/$T/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --daemon-bench 0 > $R/gpurun_out/r05/$T/prof.log 2>&1 || exit 1
  cd $R && python3 scripts/step_summary.py $(ls gpurun_out/r05/$T/prof/*kernel_stats.csv | head -1) --steps 4 > gpurun_out/r05/$T/step_summary.txt 2>&1; head -16 gpurun_out/r05/$T/step_summary.txt
  cd /tmp
  timeout -s KILL 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/r05/$T/pmc -o run -- python3 $R/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $R/gpurun_out/r05/$T/pmc.log 2>&1 || exit 1
  cd $R && python3 scripts/step_pmc_summary.py gpurun_out/r05/$T/pmc > gpurun_out/r05/$T/mfma_busy_by_category.txt && cat gpurun_out/r05/$T/mfma_busy_by_category.txt
fi
