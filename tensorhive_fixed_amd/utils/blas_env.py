"""Guard against a hipBLASLt workspace too small for its stream-K kernels (round-3 verdict item 8).

With ``HIPBLASLT_WORKSPACE_SIZE=8192`` (KiB, i.e. 8 MiB) the persistent stream-K GEMM kernels
torch's heuristics pick for the Llama-3-8B shapes (``…_SK3_…MT256x256x64``) faulted with an
illegal address inside the library (``profiles/r03_gemm/hipblaslt_workspace_8MiB_fault.txt``,
reproduced by ``scripts/bench_hipblaslt_env.py`` with plain ``torch.mm``).  Such a run can take a
GPU down for every tenant, so bench.py and the training payload (what the torchrun template
starts) refuse any explicit workspace below :data:`MIN_KIB` instead of launching it.  Unset keeps
torch's own default.
"""
from __future__ import annotations

import os

MIN_KIB = 64 * 1024  # 64 MiB; torch's hipBLASLt default is at least this on ROCm 7
VARS = ("HIPBLASLT_WORKSPACE_SIZE", "CUBLASLT_WORKSPACE_SIZE")


class UnsafeBlasWorkspace(RuntimeError):
    pass


def check_blas_workspace(env: dict | None = None) -> None:
    env = os.environ if env is None else env
    for var in VARS:
        raw = env.get(var)
        if raw is None or str(raw).strip() == "":
            continue
        try:
            kib = int(str(raw).strip())
        except ValueError:
            raise UnsafeBlasWorkspace(f"{var}={raw!r} is not a size in KiB")
        if kib < MIN_KIB:
            raise UnsafeBlasWorkspace(
                f"{var}={kib} KiB is below {MIN_KIB} KiB: hipBLASLt's stream-K GEMM kernels fault with a "
                "workspace this small (profiles/r03_gemm/hipblaslt_workspace_8MiB_fault.txt); unset it or raise it")


def refuse_unsafe_blas_workspace(prog: str) -> None:
    """Exit with status 2 and a message (before any GPU work) when the workspace is unsafe."""
    try:
        check_blas_workspace()
    except UnsafeBlasWorkspace as e:
        import sys

        print(f"[{prog}] refusing to start: {e}", file=sys.stderr, flush=True)
        raise SystemExit(2)
