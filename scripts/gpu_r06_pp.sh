#!/bin/bash
# Round 6: ping-pong flash forward -- numerics, then interleaved timing against the default kernel.
set -o pipefail
OUT=gpurun_out/r06/pp${TAG:+_$TAG}
mkdir -p $OUT
step() { local name=$1; shift; echo "[step] $name"; timeout -k 10 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[step] $name rc=$rc"; tail -3 $OUT/$name.log; return $rc; }
step pytest 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_flash_attn_gpu.py -k "pingpong or matches_reference" &&
step time_b8 200 env B=8 NO_BWD=1 VARIANTS=15,64,15,64 python -u scripts/flash_variants.py &&
if [ -n "$PROF" ]; then export B=8 NO_BWD=1 VARIANTS=15,64; step prof 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u scripts/flash_variants.py; fi &&
if [ -f diag_libs/pp_noprio.so ]; then step time_noprio 200 env TH_KERNEL_LIB=diag_libs/pp_noprio.so B=8 NO_BWD=1 VARIANTS=15,64,15,64 python -u scripts/flash_variants.py; fi &&
if [ -f diag_libs/pp_shift.so ]; then step time_shift 200 env TH_KERNEL_LIB=diag_libs/pp_shift.so B=8 NO_BWD=1 VARIANTS=15,64,15,64 python -u scripts/flash_variants.py; fi &&
if [ -f diag_libs/pp_stamp.so ]; then step stamps 120 env TH_KERNEL_LIB=diag_libs/pp_stamp.so python -u scripts/pp_stamps.py; fi
