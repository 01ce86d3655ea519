# round 3: where the NT kernel's time goes vs hipBLASLt's (w13 fwd), PMC passes (no tracing);
# plus the rccl-bench per-rank mode and the rest of the native GPU tests
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; mkdir -p $R/gpurun_out/r03/nt_pmc
run_step r03/native_tests2 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/gpu/test_native_gpu.py
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/r03/nt_pmc/p$i -o run -- python3 $R/scripts/nt_pmc.py \
    > $R/gpurun_out/r03/nt_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/r03/nt_pmc/p$i.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py gpurun_out/r03/nt_pmc/p*/ > gpurun_out/r03/nt_pmc/summary.txt 2>&1; cat gpurun_out/r03/nt_pmc/summary.txt
tail -n 15 gpurun_out/r03/native_tests2.log
