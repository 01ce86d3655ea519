# round 6: hipBLASLt / rocBLAS choices for a multi-rank step, whose GEMMs share the chip with RCCL's channel
# kernels: default heuristics idle and with K emulated channel CUs held, then TunableOp tuning under that
# contention (scripts/gemm_tune.py, TH_TUNE_EMU), then the tuned table idle and contended.
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tune}; O=gpurun_out/r06/$T; mkdir -p $O
K=${K:-16}
( while true; do sleep 30; echo "[hb] $(date +%T)"; done ) & HB=$!  # a tuning pass prints per shape only
trap "kill $HB 2>/dev/null" EXIT
export TH_TUNE_KINDS=${KINDS:-fwd,dgrad} TH_TUNED_FILE=${TABLE:-$R/$O/gemm_gfx950_t32768_dp.csv}
if [ "${PART:-1}" = "1" ]; then
  [ "${SURVEY:-1}" = "1" ] && run_step r06/$T/survey_idle 300 python -u scripts/gemm_tune.py survey; grep gemm_ms_per_step $O/survey_idle.log
  [ "${SURVEY:-1}" = "1" ] && TH_TUNE_EMU=cus=$K run_step r06/$T/survey_k$K 300 python -u scripts/gemm_tune.py survey; grep gemm_ms_per_step $O/survey_k$K.log
  if [ "${TUNE_MODE:-tune}" = "resume" ] && [ -n "${SEED:-}" ]; then
    # resume from the round-5 table without its "Default" rows: only those shapes are tuned (under contention)
    grep -v ',Default,' "$SEED" > "$TH_TUNED_FILE"
  fi
  TH_TUNE_EMU=cus=$K TH_TUNE_MS=${TUNE_MS:-250} run_step r06/$T/tune_k$K 780 python -u scripts/gemm_tune.py ${TUNE_MODE:-tune}
  tail -n 2 $O/tune_k$K.log
else
  run_step r06/$T/check_idle 300 python -u scripts/gemm_tune.py check; grep gemm_ms_per_step $O/check_idle.log
  TH_TUNE_EMU=cus=$K run_step r06/$T/check_k$K 300 python -u scripts/gemm_tune.py check; grep gemm_ms_per_step $O/check_k$K.log
fi
