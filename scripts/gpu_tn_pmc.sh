# PMC passes over the TN kernel, modes 2 and 6 (one rocprofv3 run per counter set and mode; no tracing)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/tn_pmc; cd /tmp && export TMPDIR=/tmp
for pp in 2 6; do
  i=0
  for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
    i=$((i+1))
    TN_PP=$pp timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/tn_pmc/pp${pp}_$i -o run -- python3 $R/scripts/tn_pmc.py \
      > $R/gpurun_out/tn_pmc/pp${pp}_$i.log 2>&1 || { echo "pass pp$pp/$i failed"; tail -3 $R/gpurun_out/tn_pmc/pp${pp}_$i.log; }
  done
done
cd $R && for pp in 2 6; do echo "== mode $pp"; python3 scripts/pmc_summary.py gpurun_out/tn_pmc/pp${pp}_*/ 2>&1 | grep -A20 gemm_tn | head -20; done
