"""PMC probe of the TN weight-gradient kernel (hb, mode 9) against hipBLASLt on the same FLOPs:
C[4096, 4096] = A[32768, 4096]^T B[32768, 4096] as TN (hb and hipBLASLt) and as hipBLASLt NT on
K-contiguous copies.  Run under rocprofv3 --pmc (one pass per counter set), then summarise with
``python scripts/tn_pmc.py --summary DIR``."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from tensorhive_fixed_amd.ops import _lib
    from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_
    _lib.load()
    T, M, N = 32768, 4096, 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
    at, bt = a.t().contiguous(), b.t().contiguous()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        gemm_tn_(a, b, c, splitk=1, pingpong=9)
    for _ in range(10):
        torch.mm(at, bt.t(), out=c)
    for _ in range(10):
        torch.mm(a.t(), b, out=c)
    torch.cuda.synchronize()
    print("tn_pmc done", flush=True)


def summary(d):
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")[:70]
            rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in rows.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:34s} {sum(v) / len(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
