R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/mem_pmc; cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/mem_pmc/p$i -o run -- python3 $R/scripts/mem_pmc.py > $R/gpurun_out/mem_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/mem_pmc/p$i.log; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/mem_pmc/p*/
