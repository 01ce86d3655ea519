#!/bin/bash
# Round 6: gradient-bucket size under the modelled 8-rank ZeRO-1 step (TH_COMM_EMU bucket mode with the
# collective dependencies, deps=1): reduce-scatters beside backward, the optimizer waiting for them, the
# all-gathers beside the next forward and each layer waiting for its bucket.
set -o pipefail
OUT=gpurun_out/r06/bucket${TAG:+_$TAG}
mkdir -p $OUT
step() { local name=$1; shift; echo "[step] $name"; timeout -k 10 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[step] $name rc=$rc"; grep -o '"value": [0-9.]*' $OUT/$name.log | head -1; return $rc; }
S=${STEPS:-6}; W=${WARMUP:-3}
step none_256 300 python -u bench.py --steps $S --warmup $W --bucket-mb 256 || exit 1
for mb in ${BUCKETS:-64 128 256 512 1024}; do
  step emu${CUS:-32}_$mb 300 env TH_COMM_EMU="cus=${CUS:-32},mode=bucket,world=8,busbw=${BUSBW:-300},deps=1" \
    python -u bench.py --steps $S --warmup $W --bucket-mb $mb || exit 1
done
step none_256b 300 python -u bench.py --steps $S --warmup $W --bucket-mb 256
