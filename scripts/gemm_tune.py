"""Per-shape GEMM survey + TunableOp tuning for the Llama-3-8B training step on one MI355X.

    python scripts/gemm_tune.py survey            # TFLOP/s of every GEMM of the step, default heuristics
    python scripts/gemm_tune.py tune              # TunableOp: benchmark hipBLASLt/rocBLAS candidates per
                                                  # shape, write tensorhive_fixed_amd/ops/tuned/gemm_gfx950.csv
    python scripts/gemm_tune.py resume            # tune only the shapes missing from the table
    python scripts/gemm_tune.py check             # survey again with the tuned table loaded (tuning off)

The GEMMs are exactly the ones the payload issues (ops/linear.py, ops/mlp.py, ops/cross_entropy.py):
forward ``x @ W^T`` (addmm with the residual for wo / w2), input grad ``dy @ (W^T)^T`` on the
transposed weight copy (K-contiguous form), weight grad ``dy^T @ x`` written into the flat gradient
buffer -- for the gate|up projection on transposed operands ``(dy^T) @ (x^T)^T``.
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
TUNED = Path(os.environ.get("TH_TUNED_FILE", ROOT / "tensorhive_fixed_amd" / "ops" / "tuned" / "gemm_gfx950.csv"))
KINDS = set(os.environ.get("TH_TUNE_KINDS", "fwd,dgrad,wgrad").split(","))  # round 5: weight grads run on the TN kernel

T = int(os.environ.get("TH_TUNE_TOKENS", "32768"))  # tokens per micro-step (bench default MB 8 x 4096)
D, HQKV, FF, V = 4096, 6144, 14336, 128256
CH = 4096  # CE chunk


def shapes():
    """(name, kind, M, N, K, residual) with C[M,N] = A[M,K] @ B[K,N]."""
    out = []
    for name, n_out, k_in, res in (("wqkv", HQKV, D, False), ("wo", D, D, True), ("w13", 2 * FF, D, False),
                                   ("w2", D, FF, True)):
        out.append((name, "fwd", T, n_out, k_in, res))
        out.append((name, "dgrad", T, k_in, n_out, False))
        out.append((name, "wgrad", n_out, k_in, T, False))
    out.append(("head", "fwd", CH, V, D, False))
    out.append(("head", "dgrad", CH, D, V, False))
    out.append(("head", "wgrad", V, D, CH, True))  # accumulated over chunks (beta = 1)
    return out


def make(kind, M, N, K, res, dev, name=""):
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, dtype=torch.bfloat16, generator=g)  # noqa: E731
    if kind == "fwd":  # x[M,K] @ W[N,K]^T
        x, w = r(M, K), r(N, K)
        c = r(M, N) if res else None
        return (lambda: torch.addmm(c, x, w.t())) if res else (lambda: torch.mm(x, w.t()))
    if kind == "dgrad":
        dy = r(M, K)
        if name == "head":  # dlogits[M,V] @ W[V,D]
            w = r(K, N)
            return lambda: torch.mm(dy, w)
        wT = r(N, K)  # the transposed weight copy [in, out]: dy @ (W^T)^T, both operands K-contiguous
        return lambda: torch.mm(dy, wT.t())
    if name == "w13":  # dW = (dy^T)[N_out, T] @ (x^T)[K_in, T]^T
        dyT, xT = r(M, K), r(N, K)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        return lambda: torch.mm(dyT, xT.t(), out=out)
    # wgrad: dy^T[N_out, T] @ x[T, K_in] -> out [M=N_out, N=K_in]
    dy, x = r(K, M), r(K, N)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if res:
        return lambda: out.addmm_(dy.t(), x)
    return lambda: torch.mm(dy.t(), x, out=out)


def timeit(fn, iters=20):
    # current-stream syncs: a device-wide one would wait for TH_TUNE_EMU's channel kernel on its side stream
    for _ in range(3):
        fn()
    torch.cuda.current_stream().synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def survey(tag):
    dev = torch.device("cuda:0")
    tot_ms, tot_fl = 0.0, 0.0
    rows = []
    for name, kind, M, N, K, res in shapes():
        if kind not in KINDS:
            continue
        fn = make(kind, M, N, K, res, dev, name)
        ms = timeit(fn)
        fl = 2.0 * M * N * K
        per_step = 32 if name != "head" else T // CH
        tot_ms += ms * per_step
        tot_fl += fl * per_step
        rows.append({"gemm": f"{name}.{kind}", "M": M, "N": N, "K": K, "ms": round(ms, 4),
                     "tflops": round(fl / ms / 1e9, 1)})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"tag": tag, "gemm_ms_per_step": round(tot_ms, 1), "avg_tflops": round(tot_fl / tot_ms / 1e9, 1)}),
          flush=True)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "survey"
    tun = torch.cuda.tunable
    # TH_TUNE_EMU="cus=16": measure / tune with an emulated RCCL channel kernel holding that many CUs
    # (parallel/comm_emu.py) -- the table a multi-rank step wants, whose GEMMs share the chip with RCCL
    emu = None
    if os.environ.get("TH_TUNE_EMU"):
        sys.path.insert(0, str(ROOT))
        from tensorhive_fixed_amd.ops import _lib
        from tensorhive_fixed_amd.parallel.comm_emu import CommEmulator, parse

        _lib.load()
        emu = CommEmulator(parse(os.environ["TH_TUNE_EMU"] + ",copy=1,slice_ms=5000,buffer_mb=64"), torch.device("cuda"))
        emu.hold(float(os.environ.get("TH_TUNE_EMU_S", "700")))
        time.sleep(0.05)  # channel workgroups resident before the first GEMM
    try:
        _run(mode, tun)
    finally:
        if emu is not None:
            emu.stop()
            torch.cuda.synchronize()
            emu.side.synchronize()


def _run(mode, tun):
    if mode in ("tune", "resume"):
        TUNED.parent.mkdir(parents=True, exist_ok=True)
        if mode == "tune" and TUNED.exists():
            TUNED.unlink()
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_filename(str(TUNED))
        if mode == "resume" and TUNED.exists():
            tun.read_file(str(TUNED))  # already-tuned shapes are not tuned again
        tun.set_max_tuning_duration(int(os.environ.get("TH_TUNE_MS", "400")))
        tun.set_max_tuning_iterations(int(os.environ.get("TH_TUNE_ITERS", "20")))
        t0 = time.time()
        survey("tuning-pass")
        if hasattr(tun, "write_file"):  # older torch; 2.10 writes the table itself (on exit / per result)
            tun.write_file()
        print(json.dumps({"tuned_file": str(TUNED), "tuning_s": round(time.time() - t0, 1)}))
        return
    if mode == "check":
        tun.enable(True)
        tun.tuning_enable(False)
        tun.set_filename(str(TUNED))
        tun.read_file(str(TUNED))
    survey(mode)


if __name__ == "__main__":
    main()
