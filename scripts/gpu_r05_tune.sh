# round 5: TunableOp over the step's hipBLASLt GEMMs at 32768 tokens (forward + input gradients; the weight
# gradients run on the TN kernel): default survey, tuning pass, survey with the tuned table
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tune}; mkdir -p gpurun_out/r05/$T
export TH_TUNE_KINDS=fwd,dgrad TH_TUNED_FILE=$R/gpurun_out/r05/$T/gemm_gfx950_t32768.csv
run_step r05/$T/survey_default 300 python -u scripts/gemm_tune.py survey
grep gemm_ms_per_step gpurun_out/r05/$T/survey_default.log
run_step r05/$T/tune 900 python -u scripts/gemm_tune.py tune
tail -n 2 gpurun_out/r05/$T/tune.log
run_step r05/$T/check 300 python -u scripts/gemm_tune.py check
grep gemm_ms_per_step gpurun_out/r05/$T/check.log
