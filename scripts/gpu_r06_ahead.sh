#!/bin/bash
# Round 6: operand look-ahead of two steps in the forward S chain and the dQ kernel's K^T chain
# (diag_libs/fa_ahead_fq.so) against the production library, alternating processes.
set -o pipefail
OUT=gpurun_out/r06/ahead
mkdir -p $OUT
export B=8 VARIANTS=15,15 BWD_FLAGS=1006544,1006544
for i in 1 2; do
  timeout -k 10 200 python -u scripts/flash_variants.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/fa_ahead_fq.so python -u scripts/flash_variants.py > $OUT/ahead_$i.log 2>&1 || exit 1
done
for f in $OUT/*.log; do echo "== $f"; grep -E '"variant"|flash_bwd' $f | cut -c1-160; done
timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/fa_ahead_fq.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py > $OUT/pytest_ahead.log 2>&1; echo "pytest rc=$?"; tail -2 $OUT/pytest_ahead.log
