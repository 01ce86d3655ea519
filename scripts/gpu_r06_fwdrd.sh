#!/bin/bash
# Round 6: forward kernel change (production) vs diag_libs/fwd_rd0.so (the previous form), alternating processes.
set -o pipefail
OUT=gpurun_out/r06/fwdrd${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
export B=8 NO_BWD=1 VARIANTS=15,15
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/flash_variants.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/fwd_rd0.so python -u scripts/flash_variants.py > $OUT/rd0_$i.log 2>&1 || exit 1
done
for f in $OUT/prod_*.log $OUT/rd0_*.log; do echo "$f $(grep -o '"ms": [0-9.]*' $f | head -1)"; done
