# round 6: the emulated RCCL footprint on the Llama-3-8B step (parallel/comm_emu.py) -- round-5 behaviour
# ("nofix": single-GPU GEMM table, TN planned for 256 CUs) against the round-6 multi-rank settings ("fix":
# the multi-rank GEMM table without stream-K defaults, TN planned for the CUs left) for
#   persist mode: k channel workgroups held from the first bucket-ready point to the end of backward;
#   bucket mode: one channel launch per bucket lasting its modelled ring reduce-scatter (8 ranks, busbw GB/s).
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-sweep2}; O=gpurun_out/r06/$T; mkdir -p $O
B="python bench.py --gpus 1 --steps ${STEPS:-6} --warmup ${WARM:-2} --daemon-bench 0"
SINGLE=$R/tensorhive_fixed_amd/ops/tuned/gemm_gfx950_t32768.csv
run_step r06/$T/base 300 $B; grep -o '"value": [0-9.]*' $O/base.log
for spec in ${SPECS:-cus=8 cus=16 cus=32 cus=64 cus=16,mode=bucket cus=32,mode=bucket}; do
  n=$(echo $spec | tr ',=' '__')
  if [ "${ONLY_DEFAULT:-0}" = "1" ]; then
    TH_COMM_EMU="$spec" TH_COMM_CUS=0 run_step r06/$T/${n}_default 300 $B
    echo "$n default $(grep -o '"value": [0-9.]*' $O/${n}_default.log)"
    continue
  fi
  # nofix: round-5 behaviour (stream-K grids as hipBLASLt picks them, TN planned for 256 CUs)
  TENSILE_STREAMK_DATA_PARALLEL=0 TH_COMM_EMU="$spec" TH_COMM_CUS=0 TH_GEMM_TUNED_FILE=$SINGLE run_step r06/$T/${n}_nofix 300 $B
  echo "$n nofix $(grep -o '"value": [0-9.]*' $O/${n}_nofix.log)"
  # default: the shipped multi-rank settings (stream-K kernels tiled data-parallel, TN planned for 256 CUs)
  TH_COMM_EMU="$spec" TH_COMM_CUS=0 run_step r06/$T/${n}_default 300 $B
  echo "$n default $(grep -o '"value": [0-9.]*' $O/${n}_default.log)"
  # fix: + the TN launch planned for the CUs the channels leave (TH_COMM_CUS, automatic under the rehearsal)
  TH_COMM_EMU="$spec" run_step r06/$T/${n}_fix 300 $B
  echo "$n fix $(grep -o '"value": [0-9.]*' $O/${n}_fix.log)"
done
