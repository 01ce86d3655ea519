#!/bin/bash
# Round 6: step A/B of the kf M0 split (production) against diag_libs/dq_nopre.so (TH_KF_M0SPLIT=0), alternating.
set -o pipefail
OUT=gpurun_out/r06/kfm0_step
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --daemon-bench 0 > $OUT/kfm0on_$i.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $OUT/kfm0on_$i.log
  timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/dq_nopre.so python -u bench.py --steps 8 --warmup 3 --daemon-bench 0 > $OUT/kfm0off_$i.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $OUT/kfm0off_$i.log
done
