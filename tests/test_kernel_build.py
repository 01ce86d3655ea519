"""The gfx950 kernel library build (ops/build.py) on the CPU: per-source flags, and every entry point
that ops/_lib.py binds is exported by the in-tree libthk.so (when it has been built)."""
import shutil
import subprocess
from pathlib import Path

import pytest

from tensorhive_fixed_amd.ops import _lib, build


def test_per_source_build_flags():
    flash = build.CSRC / "flash_attn.hip"
    assert build.source_flags(flash) == ["-fno-slp-vectorize"]
    for src in build._sources():
        flags = build.source_flags(src)
        assert all(f.startswith("-") for f in flags), (src.name, flags)
    assert build.source_flags(build.CSRC / "adamw.hip") == []


def test_source_flags_reads_only_the_header(tmp_path: Path):
    src = tmp_path / "k.hip"
    src.write_text("// th-build-flags: -DFOO=1 -fno-unroll-loops\n#include <x>\n")
    assert build.source_flags(src) == ["-DFOO=1", "-fno-unroll-loops"]
    late = tmp_path / "late.hip"
    late.write_text("\n" * 50 + "// th-build-flags: -DLATE\n")
    assert build.source_flags(late) == []


@pytest.mark.skipif(not build.LIB.exists() or shutil.which("nm") is None, reason="libthk.so not built")
def test_library_exports_every_bound_entry_point():
    out = subprocess.run(["nm", "-D", "--defined-only", str(build.LIB)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(name for name in _lib._SIGS if name not in exported)
    assert not missing, f"bound in ops/_lib.py but not exported by libthk.so: {missing}"


def test_bindings_match_the_c_declarations():
    """Argument counts of every ops/_lib.py binding equal those of its `extern "C"` definition."""
    import re

    decls = {}
    for src in build._sources():
        text = src.read_text()
        for m in re.finditer(r'extern "C" \w+\s+(th_\w+)\(([^)]*)\)', text):
            args = [a for a in m.group(2).replace("\n", " ").split(",") if a.strip() and a.strip() != "void"]
            decls[m.group(1)] = len(args)
    for name, argtypes in _lib._SIGS.items():
        assert name in decls, f"{name}: no extern \"C\" definition in ops/csrc"
        assert decls[name] == len(argtypes), f"{name}: C takes {decls[name]} args, binding has {len(argtypes)}"
