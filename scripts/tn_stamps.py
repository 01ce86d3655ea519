"""Where a TN hb wave's cycles go per k-tile: run the s_memtime-stamped build and print, per wave and k-tile,
the loop cycles and the cycles spent in each of the three waits (barrier at MFMA 20 after A's reads, barrier at
44 after B's reads, vmcnt + barrier at 88 for the next tile's DMA).

    bash scripts/build_variant_lib.sh tn_diag -DTH_TN_DIAG=1 gemm_tn
    TH_KERNEL_LIB=ab_libs/tn_diag.so python scripts/tn_stamps.py

The production libthk.so carries no stamps (gemm_tn.hip TH_TN_DIAG)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.gemm_tn import gemm_tn_  # noqa: E402

lib = _lib.load()
if not hasattr(lib, "th_tn_stamps"):
    sys.exit(f"{_lib.library_path()} is a production build: set TH_KERNEL_LIB to the TH_TN_DIAG library")
lib.th_tn_stamps.argtypes = [C.c_void_p, C.c_int]
lib.th_tn_stamps.restype = C.c_int
buf = (C.c_ulonglong * 8)()
for name, M, N, T in (("wo", 4096, 4096, 32768), ("wqkv", 6144, 4096, 32768)):
    a = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm_tn_(a, b, c, splitk=1, pingpong=9)
    torch.cuda.synchronize()
    assert lib.th_tn_stamps(buf, 1) == 0
    for _ in range(5):
        gemm_tn_(a, b, c, splitk=1, pingpong=9)
    torch.cuda.synchronize()
    assert lib.th_tn_stamps(buf, 0) == 0
    tiles = buf[0]
    per = lambda i: round(buf[i] / tiles, 1)  # noqa: E731
    print(json.dumps({"gemm": name, "wave_ktiles": tiles, "cycles_per_ktile": per(1), "wait_bar20": per(2),
                      "wait_bar44": per(3), "wait_vmcnt_bar88": per(4),
                      "mfma_floor": 128 * 16}), flush=True)
