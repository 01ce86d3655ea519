#!/bin/bash
# Round 6: TN main-loop DMA pieces with M0 written before the gap's MFMA (diag_libs/tn_m0.so) vs production.
set -o pipefail
OUT=gpurun_out/r06/tnm0
mkdir -p $OUT
timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/tn_m0.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_gemm_tn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/tn_time.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/tn_m0.so python -u scripts/tn_time.py > $OUT/m0_$i.log 2>&1 || exit 1
done
cat $OUT/prod_*.log $OUT/m0_*.log | grep shape
