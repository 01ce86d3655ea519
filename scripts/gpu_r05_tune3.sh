# round 5: per-shape effect of the TunableOp table on one box -- default survey and table survey, interleaved twice
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tune3}; mkdir -p gpurun_out/r05/$T
export TH_TUNE_KINDS=fwd,dgrad TH_TUNED_FILE=$R/tensorhive_fixed_amd/ops/tuned/gemm_gfx950_t32768.csv
for i in 1 2; do
  run_step r05/$T/default_$i 300 python -u scripts/gemm_tune.py survey
  run_step r05/$T/table_$i 300 python -u scripts/gemm_tune.py check
done
for f in default_1 table_1 default_2 table_2; do echo "== $f"; grep '"gemm"\|gemm_ms_per_step' gpurun_out/r05/$T/$f.log; done | tee gpurun_out/r05/$T/summary.txt
