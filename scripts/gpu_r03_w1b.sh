# round 3: w1 schedule variants + PMC of w1 (sched 1) vs the ping-pong kernel vs hipBLASLt
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; mkdir -p $R/gpurun_out/r03/w1_pmc
run_step r03/gemm_w1b 600 python -u scripts/bench_gemm_nt_variants.py
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/r03/w1_pmc/p$i -o run -- python3 $R/scripts/nt_pmc.py \
    > $R/gpurun_out/r03/w1_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/r03/w1_pmc/p$i.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/r03/w1_pmc/p*/ > gpurun_out/r03/w1_pmc/summary.txt 2>&1; cat gpurun_out/r03/w1_pmc/summary.txt
grep -h '"gemm"' gpurun_out/r03/gemm_w1b.log | head -6
