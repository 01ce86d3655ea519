"""Where a kf wave's cycles go: run the s_memtime-stamped kf build (VAR 7663 = the default 7535 +
stamps; KF_STAMP_VAR picks another stamped variant) and print cycles per wave per 64-query tile by phase, plus the per-block overhead (prologue: K/V
fragments, first two tile DMAs; epilogue: rotary + stores).

    bash scripts/build_variant_lib.sh kf_diag -DTH_KF_DIAG=1     # the diagnostic library
    TH_KERNEL_LIB=ab_libs/kf_diag.so python scripts/kf_stamps.py  # B 4 and 8, S 4096, 32/8 heads, d 128

The production libthk.so has no stamped variants and no ``th_kf_stamps`` (flash_attn.hip TH_KF_DIAG).
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorhive_fixed_amd.ops import _lib  # noqa: E402
from tensorhive_fixed_amd.ops.attention import flash_bwd, flash_fwd  # noqa: E402

lib = _lib.load()
if not hasattr(lib, "th_kf_stamps"):
    sys.exit(f"{_lib.library_path()} is a production build: set TH_KERNEL_LIB to the TH_KF_DIAG library")
lib.th_kf_stamps.argtypes = [C.c_void_p, C.c_int]
lib.th_kf_stamps.restype = C.c_int
S, Hq, Hkv, D = 4096, 32, 8, 128
STAMP_FLAGS = 16 | (int(os.environ.get("KF_STAMP_VAR", "7663")) << 6) | (1 << 19)
buf = (C.c_ulonglong * 8)()
for B in (4, 8):
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    o, lse = flash_fwd(qkv, B, S, Hq, Hkv, D)
    do = torch.randn_like(o)
    flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=STAMP_FLAGS)  # warm
    torch.cuda.synchronize()
    assert lib.th_kf_stamps(buf, 1) == 0
    n = 5
    for _ in range(n):
        flash_bwd(do, qkv, o, lse, B, S, Hq, Hkv, D, flags=STAMP_FLAGS)
    torch.cuda.synchronize()
    assert lib.th_kf_stamps(buf, 0) == 0
    g = list(buf)
    tiles, blocks = g[5], g[6]
    names = ["barrier+dma_wait", "mfma_0_15+dma_pieces", "mfma_16_31", "mfma_32_47", "mfma_48_63"]
    per_tile = {k: round(g[i] / tiles, 1) for i, k in enumerate(names)}
    per_tile["sum"] = round(sum(g[:5]) / tiles, 1)
    out = {"B": B, "wave_tiles": tiles, "wave_blocks": blocks, "cycles_per_wave_tile": per_tile,
           "mfma_floor_per_tile": 64 * 32,
           "block_overhead_cycles": round((g[7] - sum(g[:5])) / blocks, 1),
           "tiles_per_block": round(tiles / blocks, 1)}
    print(json.dumps(out), flush=True)
