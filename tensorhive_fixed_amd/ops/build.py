"""Build the gfx950 HIP kernels of tensorhive_fixed_amd into ONE in-tree shared library.

``python -m tensorhive_fixed_amd.ops.build`` compiles every ``csrc/*.hip`` with
``hipcc --offload-arch=gfx950`` (objects in parallel) and links ``ops/libthk.so``.  The library
exposes a plain C ABI (``extern "C" th_*``) that :mod:`tensorhive_fixed_amd.ops._lib` binds with
ctypes; no torch headers are involved, so a full rebuild takes seconds and the ``.so`` travels
with the repo snapshot to the GPU box.

There is no CUDA path and no hipify step: the sources are CDNA4 HIP written for gfx950 only.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB = HERE / "libthk.so"
BUILD_DIR = HERE / "_build"
ARCH = os.environ.get("TH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
          "-Wno-unused-result"]


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _digest() -> str:
    h = hashlib.sha256()
    for p in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()[:16]


def _stamp_path() -> Path:
    return BUILD_DIR / "libthk.stamp"


def stamp_exists() -> bool:
    return _stamp_path().exists()


def is_up_to_date() -> bool:
    return LIB.exists() and _stamp_path().exists() and _stamp_path().read_text().strip() == _digest()


def source_flags(src: Path) -> list[str]:
    """Per-source extra flags from a ``// th-build-flags: ...`` line in the file's first 40 lines
    (e.g. ``-fno-slp-vectorize`` for kernels whose f32 math runs beside MFMAs)."""
    for line in src.read_text().splitlines()[:40]:
        if line.startswith("// th-build-flags:"):
            return line.split(":", 1)[1].split()
    return []


def _compile(src: Path) -> Path:
    obj = BUILD_DIR / (src.stem + ".o")
    cmd = [HIPCC, *CFLAGS, *source_flags(src), "-I", str(CSRC), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    """Compile all kernels for gfx950 and link ``libthk.so``; returns the library path."""
    if not force and is_up_to_date():
        return LIB
    if not Path(HIPCC).exists() and shutil.which("hipcc") is None:
        raise RuntimeError("hipcc not found: cannot build the gfx950 kernels")
    BUILD_DIR.mkdir(exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    _stamp_path().write_text(_digest())
    if verbose:
        print(f"[thk] built {LIB} from {len(srcs)} sources for {ARCH}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
