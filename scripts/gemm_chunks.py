"""Does splitting a wide Llama GEMM into column (N) chunks help hipBLASLt on MI355X?

Hypothesis: for x[T, K] @ W[N, K]^T with a wide N (gate|up: N = 28672, W = 235 MB) the weight no
longer fits the 256 MB Infinity Cache next to the activations, so a row-major tile walk streams it
from HBM once per tile row.  N-chunks of <= 64 MB keep each chunk's weight cache-resident.
Prints one JSON line per (shape, chunks, output form): ms and TFLOP/s (median of 20)."""
import json
import sys

import torch

T, D, F = 32768, 4096, 14336


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, dtype=torch.bfloat16, generator=g)  # noqa: E731
    cases = [("w13.fwd", r(T, D), r(2 * F, D)), ("wqkv.fwd", r(T, D), r(6144, D)),
             ("w2.dgrad", r(T, D), r(F, D))]  # dgrad on the transposed weight copy: N = 14336
    for name, x, w in cases:
        N = w.shape[0]
        out = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        ref = torch.mm(x, w.t())
        for chunks in (1, 2, 4, 8):
            if N % chunks:
                continue
            n = N // chunks
            parts = [w[i * n:(i + 1) * n] for i in range(chunks)]

            def strided():
                for i, p in enumerate(parts):
                    torch.mm(x, p.t(), out=out[:, i * n:(i + 1) * n])
            try:
                ms = timeit(strided)
                ok = torch.equal(out, ref)
            except RuntimeError as e:  # strided out not accepted
                ms, ok = None, str(e)[:80]
            fl = 2.0 * T * N * D
            print(json.dumps({"gemm": name, "N": N, "chunks": chunks, "form": "column slices of one output",
                              "ms": ms, "tflops": round(fl / ms / 1e9) if ms else None, "exact": ok}), flush=True)
        # token (M) chunks for comparison
        for chunks in (2, 4):
            m = T // chunks

            def mchunk():
                for i in range(chunks):
                    torch.mm(x[i * m:(i + 1) * m], w.t(), out=out[i * m:(i + 1) * m])
            ms = timeit(mchunk)
            print(json.dumps({"gemm": name, "N": N, "chunks": chunks, "form": "token slices",
                              "ms": ms, "tflops": round(2.0 * T * N * D / ms / 1e9)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
