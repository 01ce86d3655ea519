#!/usr/bin/env bash
# Does device-counting mode see a tenant's TCC/SQ/TCP events once the tenant's queues have
# profiling enabled (GPU_FORCE_QUEUE_PROFILING=1)?  Round 2 saw TCC_EA0_RDREQ ~64/s and SQ/TCP 0
# for a plain tenant (profiles/r02_counters/counters_hbm.log) while GRBM/TA counters were valid.
set -u
OUT=${OUT:-gpurun_out/r03/counters_env}
mkdir -p "$OUT"
TH=tensorhive_fixed_amd/native/bin/th-counters
timeout -k 5 60 $TH --list > "$OUT/avail.txt" 2>&1 || echo "list rc=$?"
SETS=("TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum" "SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
      "TCP_TCC_READ_REQ_sum,TCP_TCC_WRITE_REQ_sum" "TCC_READ_sum,TCC_WRITE_sum")
for envv in "TH_NONE=1" "GPU_FORCE_QUEUE_PROFILING=1"; do
  for set in "${SETS[@]}"; do
    env $envv timeout -k 5 60 python3 scripts/hbm_stream.py 4 add > "$OUT/stream.json" 2>/dev/null &
    pid=$!
    sleep 2.0
    echo "== $envv $set"
    timeout -k 5 30 $TH --count 2 --period 1100 --window 1000 --counters "$set" 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}
    wait $pid
    cat "$OUT/stream.json"
    if [ "$rc" -ne 0 ]; then echo "th-counters rc=$rc -- stopping"; exit 1; fi
  done
done
