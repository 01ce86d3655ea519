"""ctypes binding of ``libthk.so`` (the gfx950 kernels built by :mod:`.build`).

Policy (loud failure, no silent fallback):
  * tensors on a GPU  -> the HIP kernel runs; if the library is missing or fails to load the
    call raises ``RuntimeError`` -- there is no eager/PyTorch fallback on device.
  * tensors on the CPU -> the callers in ``ops/*.py`` use their fp32 PyTorch reference
    implementation (used by the CPU unit tests and as the numerics oracle).

Kernels are launched on torch's *current* HIP stream (``torch.cuda.current_stream()``), so they
order correctly with hipBLASLt GEMMs and RCCL collectives issued by torch.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
_LIB_PATH = Path(os.environ.get("TH_KERNEL_LIB", _HERE / "libthk.so"))
_lock = threading.Lock()
_lib: C.CDLL | None = None

P = C.c_void_p
I = C.c_int
L = C.c_long
F = C.c_float

# name -> argtypes (every function returns int: 0 = ok, <0 = rejected shape, >0 = hipError)
_SIGS: dict[str, list] = {
    "th_rmsnorm_fwd": [P, P, P, P, I, I, F, P],
    "th_rmsnorm_add_fwd": [P, P, P, P, P, P, I, I, F, P],
    "th_rmsnorm_bwd": [P, P, P, P, P, P, P, I, I, I, I, P, P],
    "th_swiglu_fwd": [P, P, L, I, P],
    "th_swiglu_bwd": [P, P, P, L, I, P],
    "th_swiglu_bwd_t": [P, P, P, P, L, I, P],
    "th_rope_inplace": [P, P, P, L, I, I, I, I, F, P],
    "th_sumsq_bf16": [P, L, P, P, I, P],
    "th_adamw_step": [P, P, P, P, P, L, F, F, F, F, F, I, F, P, F, P],
    "th_adamw_step_f32g": [P, P, P, P, P, L, F, F, F, F, F, I, F, P, F, P],
    "th_sumsq_f32": [P, L, P, P, I, P],
    "th_ce_fwd_bwd": [P, L, P, P, P, L, I, F, I, P],
    "th_flash_attn_fwd": [P, P, P, P, P, I, I, I, I, I, I, L, L, L, L, F, I, P],
    "th_flash_attn_bwd": [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, L, L, L, L, F, I, P],
    "th_flash_attn_bwd_rope": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, L, L, L, L, F, P, P, I, P],
    "th_embedding_bwd": [P, P, P, P, L, I, I, P],
    "th_transpose_bf16": [P, P, L, L, L, I, P],
    "th_gemm_tn": [P, L, P, L, P, L, I, I, I, I, I, I, P, L, I, P],
    "th_comm_emu_launch": [P, P, L, L, L, L, P, I, L, I, P, P],
    "th_comm_emu_stop": [P, I, P],
}


def library_path() -> Path:
    return _LIB_PATH


def load(build_if_missing: bool = False) -> C.CDLL:
    """Load (once) and return the kernel library; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists() and build_if_missing:
            from . import build as _build

            _build.build()
        if not _LIB_PATH.exists():
            raise RuntimeError(
                f"gfx950 kernel library {_LIB_PATH} is missing: run "
                "`python -m tensorhive_fixed_amd.ops.build` (no eager fallback on GPU)")
        if "TH_KERNEL_LIB" not in os.environ:
            # a library built from other sources has other entry-point signatures: ctypes would pass
            # arguments the C side reads as different ones, so refuse it instead of launching anything
            from . import build as _build

            if _build.stamp_exists() and not _build.is_up_to_date():
                if build_if_missing:
                    _build.build()
                else:
                    raise RuntimeError(f"{_LIB_PATH} was built from different sources than ops/csrc: rebuild "
                                       "with `python -m tensorhive_fixed_amd.ops.build`")
        lib = C.CDLL(str(_LIB_PATH))
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = C.c_int
        _lib = lib
        return lib


def available() -> bool:
    try:
        load()
        return True
    except (RuntimeError, OSError):
        return False


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def call(name: str, *args) -> None:
    fn = getattr(load(), name, None)
    if fn is None:
        raise RuntimeError(f"kernel entry point {name} not present in {_LIB_PATH}")
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc} ({'bad shape' if rc < 0 else 'hipError'})")
