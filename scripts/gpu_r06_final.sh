# round 6: full GPU suite, smoke, 20-step bench on the final tree (PART=1); step kernel profile + MFMA busy (PART=2)
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-final}; O=gpurun_out/r06/$T; mkdir -p $O
if [ "${PART:-1}" = "1" ]; then
  run_step r06/$T/pytest 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
  tail -n 4 $O/pytest.log
  run_step r06/$T/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -n 1 $O/smoke.log
  run_step r06/$T/bench_20 500 python bench.py --gpus 1 --steps 20 --warmup 5
  grep metric $O/bench_20.log | cut -c1-300
else
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --daemon-bench 0 > $R/$O/prof.log 2>&1 || exit 1
  cd $R && python3 scripts/step_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) --steps 4 > $O/step_summary.txt 2>&1; head -16 $O/step_summary.txt
  cd /tmp
  timeout -s KILL 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/$O/pmc -o run -- python3 $R/bench.py --steps 2 --warmup 1 --daemon-bench 0 > $R/$O/pmc.log 2>&1 || exit 1
  cd $R && python3 scripts/step_pmc_summary.py $O/pmc > $O/mfma_busy_by_category.txt && cat $O/mfma_busy_by_category.txt
fi
