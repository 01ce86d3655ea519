#!/bin/bash
# Round 6: TN loop unrolled per stage (production) vs the previous tree (diag_libs/tn_prev.so).
set -o pipefail
OUT=gpurun_out/r06/tnun${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_gemm_tn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/tn_time.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/tn_prev.so python -u scripts/tn_time.py > $OUT/prev_$i.log 2>&1 || exit 1
done
cat $OUT/prod_*.log $OUT/prev_*.log | grep shape
