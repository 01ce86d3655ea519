# round 6: TENSILE_STREAMK_DATA_PARALLEL=1 (hipBLASLt's stream-K kernels tile data-parallel instead of a one-
# workgroup-per-CU grid): per-shape GEMM survey with the step's table, interleaved step A/B idle, and the
# emulated comm schedules (profiles/r06_comm/)
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-skdp}; O=gpurun_out/r06/$T; mkdir -p $O
export TH_TUNE_KINDS=fwd,dgrad TH_TUNED_FILE=$R/tensorhive_fixed_amd/ops/tuned/gemm_gfx950_t32768.csv
E=${SKENV:-TENSILE_STREAMK_DATA_PARALLEL=1}
run_step r06/$T/check_def 300 python -u scripts/gemm_tune.py check; grep gemm_ms_per_step $O/check_def.log
( export $E; run_step r06/$T/check_dp 300 python -u scripts/gemm_tune.py check ); grep gemm_ms_per_step $O/check_dp.log
B="python bench.py --gpus 1 --steps ${STEPS:-8} --warmup ${WARM:-3} --daemon-bench 0"
for i in 1 2; do
  run_step r06/$T/base_def_$i 300 $B; echo "def $i $(grep -o '"value": [0-9.]*' $O/base_def_$i.log)"
  ( export $E; run_step r06/$T/base_dp_$i 300 $B ); echo "dp $i $(grep -o '"value": [0-9.]*' $O/base_dp_$i.log)"
done
for spec in cus=16 cus=32,mode=bucket; do
  n=$(echo $spec | tr ',=' '__')
  TH_COMM_EMU="$spec" TH_COMM_CUS=0 run_step r06/$T/${n}_def 300 $B; echo "$n def $(grep -o '"value": [0-9.]*' $O/${n}_def.log)"
  ( export $E; TH_COMM_EMU="$spec" TH_COMM_CUS=0 run_step r06/$T/${n}_dp 300 $B ); echo "$n dp $(grep -o '"value": [0-9.]*' $O/${n}_dp.log)"
done
