# round 5: TN hb DMA placement variants -- TN GPU tests with each variant, then the timing sweep
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tnpv}; mkdir -p gpurun_out/r05/$T
for pv in ${PVS:-1 2 3}; do
  TH_GEMM_TN_PV=$pv run_step r05/$T/tests_pv$pv 200 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread
  tail -n 1 gpurun_out/r05/$T/tests_pv$pv.log
  grep -q " passed" gpurun_out/r05/$T/tests_pv$pv.log && ! grep -q "failed" gpurun_out/r05/$T/tests_pv$pv.log || exit 1
done
run_step r05/$T/sweep 400 python -u scripts/tn_pv_sweep.py
cat gpurun_out/r05/$T/sweep.log
