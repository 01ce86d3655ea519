#!/usr/bin/env bash
# Which counters measure HBM traffic in rocprofiler-sdk DEVICE-counting mode on gfx950?
# Each set is sampled by th-counters (its own process) for 1 s while scripts/hbm_stream.py moves a
# known number of bytes in another process.  Round 1 saw TCC_EA0_*_sum read ~0 this way
# (profiles/r01_counters/); this run widens the search (raw vs derived TCC, TCP, SQ memory
# instruction counts) and cross-checks the same counters in DISPATCH mode with rocprofv3.
set -u
OUT=${OUT:-gpurun_out/counters_hbm}
mkdir -p "$OUT"
TH=tensorhive_fixed_amd/native/bin/th-counters
timeout -k 5 60 $TH --list > "$OUT/avail.txt" 2>&1 || echo "list rc=$?"
if [ "$#" -gt 0 ]; then SETS=("$@"); else SETS=(
  "GRBM_GUI_ACTIVE,GRBM_COUNT"
  "TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum"
  "TCC_EA0_RDREQ,TCC_EA0_WRREQ"
  "TCC_REQ_sum,TCC_HIT_sum,TCC_MISS_sum"
  "TCC_READ_sum,TCC_WRITE_sum"
  "TCC_EA0_RDREQ_64B_sum,TCC_EA0_WRREQ_64B_sum"
  "TCP_TCC_READ_REQ_sum,TCP_TCC_WRITE_REQ_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum"
  "SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
  "SQ_INSTS_VALU,SQ_WAVE_CYCLES"
  "TA_BUSY_avr,TA_TA_BUSY_sum"
  "GRBM_TC_BUSY,GRBM_EA_BUSY"
); fi
for kind in add copy; do
  for set in "${SETS[@]}"; do
    timeout -k 5 60 python3 scripts/hbm_stream.py 4 $kind > "$OUT/stream_${kind}.json" 2>/dev/null &
    pid=$!
    sleep 2.0
    echo "== $kind $set"
    timeout -k 5 30 $TH --count 2 --period 1100 --window 1000 --counters "$set" 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}
    wait $pid
    cat "$OUT/stream_${kind}.json"
    if [ "$rc" -ne 0 ]; then echo "th-counters rc=$rc -- stopping"; exit 1; fi
  done
done
[ -n "${SKIP_DISPATCH:-}" ] && exit 0
# dispatch-mode cross-check: the same TCC counters per kernel (rocprofv3 collects them per dispatch)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d "$OUT/pmc_dispatch" -o run \
  --output-format csv -- python3 scripts/hbm_stream.py 1 add > "$OUT/pmc_dispatch.log" 2>&1
echo "rocprofv3 rc=$?"
find "$OUT/pmc_dispatch" -name '*counter_collection*' | head -3
