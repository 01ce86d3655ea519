"""Print 'shape=TFLOP/s' of the default TN schedule per shape from a bench_gemm_tn.py log."""
import json
import sys

out = []
for line in open(sys.argv[1]):
    if line.startswith("{"):
        r = json.loads(line)
        k = next(k for k in r if k.startswith("tn_s"))
        out.append(f"{r['gemm']}={r[k]['tflops']}")
print(" ".join(out))
