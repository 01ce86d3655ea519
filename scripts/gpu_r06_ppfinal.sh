#!/bin/bash
# Round 6: production flash suite (ping-pong refused) + the ping-pong numerics against the diagnostic library.
set -o pipefail
OUT=gpurun_out/r06/ppfinal
mkdir -p $OUT
step() { local name=$1; shift; echo "[step] $name"; timeout -k 10 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[step] $name rc=$rc"; tail -3 $OUT/$name.log; return $rc; }
step prod 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py &&
step diag 300 env TH_KERNEL_LIB=diag_libs/fa_diag.so python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py -k pingpong &&
step diag_time 200 env TH_KERNEL_LIB=diag_libs/fa_diag.so B=8 NO_BWD=1 VARIANTS=15,64,15,64 python -u scripts/flash_variants.py
