"""``tensorhive doctor``: environment checks for an MI355X node (new)."""
from __future__ import annotations

import json
import os
import shutil
import subprocess
from pathlib import Path


def _check(name, fn):
    try:
        ok, detail = fn()
    except Exception as e:  # noqa: BLE001
        ok, detail = False, f"{type(e).__name__}: {e}"
    return name, ok, detail


def run_checks() -> list[tuple[str, bool, str]]:
    out = []
    out.append(_check("rocm", lambda: (Path("/opt/rocm").exists(), os.path.realpath("/opt/rocm"))))
    out.append(_check("kfd", lambda: (Path("/dev/kfd").exists(), "/dev/kfd")))
    out.append(_check("hipcc", lambda: (shutil.which("hipcc") is not None or Path("/opt/rocm/bin/hipcc").exists(),
                                        "gfx950 cross-compiler")))

    def thk():
        from .ops import _lib
        from .ops import build as kb

        if not kb.is_up_to_date():
            kb.build()
        _lib.load()
        return True, str(_lib.library_path())

    out.append(_check("gfx950 kernels (libthk.so)", thk))

    def native():
        from .native import build as nb

        res = nb.build_all(strict=False)
        bad = [k for k, v in res.items() if v]
        return not bad, "built" if not bad else f"failed: {bad}"

    out.append(_check("native tools (th-run, libthsmi, th-smi, rccl-bench)", native))

    def smi():
        from .core.telemetry import AmdSmiBackend

        b = AmdSmiBackend()
        topo = b.topology("localhost")
        n = len(topo.get("gpus", []))
        links = {l["type"] for g in topo.get("gpus", []) for l in g.get("links", []) if l["type"] != "self"}
        b.close()
        return n > 0, f"{n} GPU(s), peer links: {sorted(links) or 'none'}"

    out.append(_check("amdsmi telemetry", smi))

    def hbm_tool():
        """The in-task HBM counter tool th-run injects: built, the rocprofiler-sdk it resolves at run time
        present, and no DT_NEEDED on the SDK (a tool that links it makes every task's HIP start ELF-scan
        all loaded libraries: +3.3 s per task under torch, profiles/r05_daemon/)."""
        from .core import hbm

        p = hbm.tool_path()
        if not p:
            return False, "libthhbm.so not built (HBM bytes fall back to the activity estimate)"
        sdk = sorted(Path("/opt/rocm/lib").glob("librocprofiler-sdk.so*"))
        if not sdk:
            return False, f"{p}: rocprofiler-sdk not installed"
        if shutil.which("readelf"):
            dyn = subprocess.run(["readelf", "-d", p], capture_output=True, text=True, timeout=30).stdout
            if any("(NEEDED)" in ln and "rocprofiler" in ln for ln in dyn.splitlines()):
                return False, f"{p} links librocprofiler-sdk: every task would start ~3 s later; rebuild it"
        return True, f"{p} (SDK {sdk[0].name}, resolved at run time)"

    out.append(_check("in-task HBM counter tool (libthhbm)", hbm_tool))

    def torch_rocm():
        import torch

        return torch.cuda.is_available() and torch.version.hip is not None, \
            f"torch {torch.__version__} hip {torch.version.hip} devices {torch.cuda.device_count()}"

    out.append(_check("torch (ROCm)", torch_rocm))

    def rccl():
        from .native.build import path_of

        p = path_of("rccl-bench")
        if not p.exists():
            return False, "rccl-bench not built"
        r = subprocess.run([str(p), "--min", str(8 << 20), "--max", str(8 << 20), "--iters", "3", "--op", "allreduce"],
                           capture_output=True, text=True, timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr.strip()[-200:]
        return r.returncode == 0, line

    out.append(_check("optional rccl all-reduce", rccl))
    return out


if __name__ == "__main__":
    for n, ok, d in run_checks():
        print(json.dumps({"check": n, "ok": ok, "detail": d}))
