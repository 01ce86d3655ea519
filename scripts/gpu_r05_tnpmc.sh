# round 5: PMC passes over the TN hb kernel vs hipBLASLt (NT and TN) on the wo wgrad FLOPs
R=$GRAFT_REPO_ROOT; cd $R; T=${TAG:-tnpmc}; mkdir -p gpurun_out/r05/$T
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
         "TCP_TCC_READ_REQ_sum TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/r05/$T/p$i -o run -- python3 $R/scripts/tn_pmc.py > $R/gpurun_out/r05/$T/p$i.log 2>&1 || exit 1
done
cd $R; for i in 1 2 3; do python3 scripts/tn_pmc.py --summary gpurun_out/r05/$T/p$i; done > gpurun_out/r05/$T/summary.txt; cat gpurun_out/r05/$T/summary.txt
