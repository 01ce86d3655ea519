#!/bin/bash
# Round 6: backward A/B, production vs diag_libs/dq_nopre.so (here: kf without the paired lgkmcnt waits).
set -o pipefail
OUT=gpurun_out/r06/kfm0
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
export B=8 VARIANTS=15 BWD_FLAGS=1006544,1006544,1006544
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/flash_variants.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/dq_nopre.so python -u scripts/flash_variants.py > $OUT/nopre_$i.log 2>&1 || exit 1
done
for f in $OUT/prod_*.log $OUT/nopre_*.log; do echo "$f $(grep flash_bwd $f | grep -o '"ms": [0-9.]*' | tr '\n' ' ')"; done
