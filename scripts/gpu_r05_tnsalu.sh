# round 5: TN hb with incremental DMA base pointers (fewer SALU per k-tile) vs the previous build, interleaved
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${TAG:-tnsalu}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/tests 300 python -u -m pytest tests/gpu/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread
tail -n 1 gpurun_out/r05/$T/tests.log
grep -q " passed" gpurun_out/r05/$T/tests.log && ! grep -q "failed" gpurun_out/r05/$T/tests.log || exit 1
for i in 1 2; do
  for v in old new; do
    TH_KERNEL_LIB=$R/ab_libs/tn_$v.so TN_MODES=10 run_step r05/$T/bench_${v}_$i 300 python -u scripts/bench_gemm_tn_hb.py
    echo "== $v run $i"; grep '"gemm"' gpurun_out/r05/$T/bench_${v}_$i.log | python3 -c "import sys,json; [print(d['gemm'], d['m10_ms']) for d in map(json.loads, sys.stdin)]"
  done
done | tee gpurun_out/r05/$T/ab.txt
