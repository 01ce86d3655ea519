# round 6: RCCL channel-footprint rehearsal on one GPU (parallel/comm_emu.py).
# PART=1: GPU tests of the emulator + CU-aware TN; step time vs emulated channel CUs, without (TH_COMM_CUS=0)
# and with the CU-aware TN geometry.  PART=2: kernel stats at one k, without and with the fix.
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-sweep}; O=gpurun_out/r06/$T; mkdir -p $O
B="python bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARM:-3} --daemon-bench 0"
if [ "${PART:-1}" = "1" ]; then
  if [ "${TESTS:-1}" = "1" ]; then
    run_step r06/$T/pytest 600 python -u -m pytest tests/gpu/test_comm_emu_gpu.py tests/gpu/test_gemm_tn_gpu.py -x -v --timeout 120 --timeout-method thread
    tail -n 3 $O/pytest.log
    grep -q " passed" $O/pytest.log || exit 3
  fi
  run_step r06/$T/base 300 $B; grep metric $O/base.log | cut -c1-200
  for k in ${KS:-8 16 32 64}; do
    TH_COMM_EMU="cus=$k${EMU_EXTRA}" TH_COMM_CUS=0 run_step r06/$T/k${k}_nofix 300 $B
    grep -o '"value": [0-9.]*' $O/k${k}_nofix.log
    TH_COMM_EMU="cus=$k${EMU_EXTRA}" run_step r06/$T/k${k}_fix 300 $B
    grep -o '"value": [0-9.]*' $O/k${k}_fix.log
  done
else
  # VARIANTS: "name|TH_COMM_EMU spec|VAR=val;VAR=val" (spec empty = no emulation; names ending in _nofix plan
  # TN for 256 CUs)
  cd /tmp && export TMPDIR=/tmp
  for v in ${VARIANTS:-"base||" "k8_nofix|cus=8|"}; do
    IFS='|' read -r name spec envs <<< "$v"
    case $name in *_nofix) export TH_COMM_CUS=0;; *) unset TH_COMM_CUS;; esac
    ( IFS=';'; for e in $envs; do [ -n "$e" ] && export "$e"; done
      TH_COMM_EMU="$spec" timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$name -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --daemon-bench 0 > $R/$O/prof_$name.log 2>&1 ) || exit 1
    python3 $R/scripts/step_summary.py $(ls $R/$O/prof_$name/*kernel_stats.csv | head -1) --steps 4 > $R/$O/step_summary_$name.txt 2>&1; head -18 $R/$O/step_summary_$name.txt
  done
fi
