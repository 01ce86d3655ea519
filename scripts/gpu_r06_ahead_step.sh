#!/bin/bash
# Round 6: step A/B of the forward S-chain look-ahead (production: 2; diag_libs/fwd_ahead1.so: 1), alternating.
set -o pipefail
OUT=gpurun_out/r06/ahead_step
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --daemon-bench 0 > $OUT/ahead2_$i.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $OUT/ahead2_$i.log
  timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/fwd_ahead1.so python -u bench.py --steps 8 --warmup 3 --daemon-bench 0 > $OUT/ahead1_$i.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $OUT/ahead1_$i.log
done
