#!/bin/bash
# Round 6: a TN schedule variant (diag_libs/tn_var.so) against production: TN GPU tests on the variant, then
# alternating-process timing of both.
set -o pipefail
OUT=gpurun_out/r06/tnvar${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 300 env TH_KERNEL_LIB=diag_libs/tn_var.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_gemm_tn_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/tn_time.py > $OUT/prod_$i.log 2>&1 || exit 1
  timeout -k 10 200 env TH_KERNEL_LIB=diag_libs/tn_var.so python -u scripts/tn_time.py > $OUT/var_$i.log 2>&1 || exit 1
done
python3 - $OUT <<'PY'
import json, sys, glob, collections
for kind in ("prod", "var"):
    tot = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{sys.argv[1]}/{kind}_*.log")):
        for l in open(f):
            if l.startswith("{"):
                d = json.loads(l); tot[d["shape"]].append(d["ms"])
    print(kind, {k: round(min(v), 4) for k, v in tot.items()}, "sum_of_mins", round(sum(min(v) for v in tot.values()), 4))
PY
