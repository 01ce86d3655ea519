#!/bin/bash
# Round 6: TN DMA-slot placements (diag_libs/tn_v1..3.so) against production, alternating processes.
set -o pipefail
OUT=gpurun_out/r06/tnslots
mkdir -p $OUT
for v in v1 v2 v3; do
  timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/tn_$v.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_gemm_tn_gpu.py -k "matches_fp32 or llama" > $OUT/pytest_$v.log 2>&1 || { tail -3 $OUT/pytest_$v.log; exit 1; }
done
for i in 1 2; do
  timeout -k 10 200 python -u scripts/tn_time.py > $OUT/prod_$i.log 2>&1 || exit 1
  for v in v1 v2 v3; do
    timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/tn_$v.so python -u scripts/tn_time.py > $OUT/${v}_$i.log 2>&1 || exit 1
  done
done
python3 - $OUT <<'PY'
import json, sys, glob, collections
for kind in ("prod", "v1", "v2", "v3"):
    tot = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{sys.argv[1]}/{kind}_*.log")):
        for l in open(f):
            if l.startswith("{"):
                d = json.loads(l); tot[d["shape"]].append(d["ms"])
    print(kind, {k: round(min(v), 4) for k, v in tot.items()}, "sum_of_mins", round(sum(min(v) for v in tot.values()), 4))
PY
