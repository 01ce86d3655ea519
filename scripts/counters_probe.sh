#!/usr/bin/env bash
# Which memory counters does the device counting service deliver on gfx950? (one copy loop per set)
set -u
TH=tensorhive_fixed_amd/native/bin/th-counters
for set in "FETCH_SIZE,WRITE_SIZE" "TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_DRAM_sum,TCC_EA0_WRREQ_DRAM_sum" "SQ_WAVES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE" "BANDWIDTH_EA"; do
  python3 - "$set" <<'PY' &
import sys, time, torch
x = torch.empty(1 << 30, device="cuda", dtype=torch.uint8); y = torch.empty_like(x)
t0 = time.time()
while time.time() - t0 < 3:
    for _ in range(10): y.copy_(x)
    torch.cuda.synchronize()
PY
  pid=$!
  sleep 1.5
  echo "== $set"
  timeout -k 5 60 $TH --count 1 --window 500 --counters "$set" || echo "rc=$?"
  wait $pid
done
