# round 4: the one-wave-per-SIMD NT GEMM vs hipBLASLt (w13 fwd), PMC passes + clock
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p $R/gpurun_out/r04/nt_pmc
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/r04/nt_pmc/p$i -o run -- python3 $R/scripts/nt_pmc.py \
    > $R/gpurun_out/r04/nt_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/r04/nt_pmc/p$i.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/r04/nt_pmc/p*/ > gpurun_out/r04/nt_pmc/summary.txt 2>&1; cat gpurun_out/r04/nt_pmc/summary.txt
