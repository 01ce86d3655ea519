# round 4: NT GEMM iteration: fp32 tests, bench vs hipBLASLt on a few shapes, one PMC pass on w13 fwd
R=$GRAFT_REPO_ROOT; cd $R; source scripts/gpu_step.sh; T=${GEMM_TAG:-g}; mkdir -p gpurun_out/r04/$T
run_step r04/$T/test 300 python -u -m pytest tests/gpu/test_gemm_nt_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
tail -n 2 gpurun_out/r04/$T/test.log
grep -q " passed" gpurun_out/r04/$T/test.log && ! grep -q "failed" gpurun_out/r04/$T/test.log || exit 1
GEMM_VARIANTS=${GEMM_VARIANTS:-0} run_step r04/$T/bench 300 python -u scripts/bench_gemm_nt.py ${GEMM_SHAPES:-w13.fwd wo.fwd w2.fwd w13.dgrad}
grep gemm gpurun_out/r04/$T/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $R/gpurun_out/r04/$T/pmc -o run -- python3 $R/scripts/nt_pmc.py > $R/gpurun_out/r04/$T/pmc.log 2>&1 || exit 1
cd $R && python3 scripts/pmc_summary.py gpurun_out/r04/$T/pmc/ | tee gpurun_out/r04/$T/pmc_summary.txt
