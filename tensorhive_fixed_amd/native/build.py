"""Build the native (non-kernel) components in-tree: ``python -m tensorhive_fixed_amd.native.build``.

Targets (all into ``native/bin`` / ``native/lib``; git-ignored, shipped with the repo snapshot):
  * ``bin/th-run``        -- C++ task supervisor (replaces GNU screen)              [g++]
  * ``lib/libthsmi.so``   -- amdsmi telemetry + process attribution (ctypes)        [g++ + libamd_smi]
  * ``bin/th-smi``        -- CLI / ``--stream`` agent over the same sampler          [g++ + libamd_smi]
  * ``bin/rccl-bench``    -- RCCL/xGMI collective + direct P2P all-reduce bench      [hipcc + librccl]
  * ``bin/th-counters``   -- device-wide HW counter sampler (rocprofiler-sdk)       [g++ + rocprofiler-sdk]
  * ``bin/th-probe``      -- per-node probe agent: the gfx950 probe kernel on every GPU [hipcc]
  * ``lib/libthhbm.so``   -- in-task HBM byte counters (rocprofiler-sdk tool library)  [g++ + rocprofiler-sdk]
The gfx950 training kernels (and the same probe kernel, for in-process use) are built by
:mod:`..ops.build` into ``libthk.so``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
BIN = HERE / "bin"
LIB = HERE / "lib"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
CXX = os.environ.get("CXX", "g++")
HIPCC = os.environ.get("HIPCC", f"{ROCM}/bin/hipcc")
ARCH = os.environ.get("TH_OFFLOAD_ARCH", "gfx950")
KSRC = HERE.parent / "ops" / "csrc"

TARGETS = {
    "th-run": (BIN / "th-run", [CXX, "-O2", "-std=c++17", "-Wall", str(HERE / "th_run.cpp")]),
    "libthsmi": (LIB / "libthsmi.so", [CXX, "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{ROCM}/include",
                                       str(HERE / "thsmi.cpp"), f"-L{ROCM}/lib", "-lamd_smi",
                                       f"-Wl,-rpath,{ROCM}/lib"]),
    "th-smi": (BIN / "th-smi", [CXX, "-O2", "-std=c++17", "-DTHSMI_MAIN", f"-I{ROCM}/include",
                                str(HERE / "thsmi.cpp"), f"-L{ROCM}/lib", "-lamd_smi", f"-Wl,-rpath,{ROCM}/lib"]),
    "th-counters": (BIN / "th-counters", [CXX, "-O2", "-std=c++17", f"-I{ROCM}/include",
                                          str(HERE / "th_counters.cpp"), f"-L{ROCM}/lib", "-lrocprofiler-sdk",
                                          "-lhsa-runtime64", f"-Wl,-rpath,{ROCM}/lib"]),
    "libthhbm": (LIB / "libthhbm.so", [CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", f"-I{ROCM}/include",
                                       str(HERE / "th_hbm_tool.cpp"), "-ldl",
                                       f"-Wl,-rpath,{ROCM}/lib"]),
    "th-probe": (BIN / "th-probe", [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", f"-I{KSRC}",
                                    str(HERE / "th_probe.hip")]),
    "rccl-bench": (BIN / "rccl-bench", [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}",
                                        str(HERE / "rccl_bench.hip"), f"-L{ROCM}/lib", "-lrccl",
                                        f"-Wl,-rpath,{ROCM}/lib"]),
}


# libthsmi's multi-threaded stress driver (built only for the sanitizer runs below)
_STRESS = [CXX, "-O2", "-std=c++17", "-pthread", f"-I{ROCM}/include", str(HERE / "thsmi.cpp"),
           str(HERE / "thsmi_stress.cpp"), f"-L{ROCM}/lib", "-lamd_smi", f"-Wl,-rpath,{ROCM}/lib"]

# Sanitizer builds of the host tools, built on demand by the sanitizer tests, never shipped.  Host
# code only -- GPU sanitizers are not used on this pool.
#   *-asan: AddressSanitizer + UBSan (th-run, th-smi, thsmi-stress)
#   *-tsan: ThreadSanitizer (th-run's forked monitor, libthsmi under 4 threads, the th-counters
#           reader with rocprofiler-sdk's own threads)
SANITIZE = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
SANITIZE_THREAD = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=thread"]
for _n, _cmd0, _kinds in (("th-run", None, ("asan", "tsan")), ("th-smi", None, ("asan", "tsan")),
                          ("thsmi-stress", _STRESS, ("asan", "tsan")), ("th-counters", None, ("tsan",))):
    _out, _cmd = (BIN / _n, _cmd0) if _cmd0 else TARGETS[_n]
    for _k in _kinds:
        _flags = SANITIZE if _k == "asan" else SANITIZE_THREAD
        TARGETS[f"{_n}-{_k}"] = (_out.with_name(f"{_out.name}-{_k}"),
                                 [_cmd[0]] + _flags + [c for c in _cmd[1:] if c not in ("-O2", "-O3")])
SANITIZED = {n for n in TARGETS if n.endswith(("-asan", "-tsan"))}
# headers / included sources a target depends on besides the sources on its command line
DEPS = {"th-probe": [KSRC / "probe.hip", KSRC / "th_common.h"]}


def sanitizer_env(report_dir: str) -> dict:
    """Environment for running a ``*-asan`` binary: reports go to files under ``report_dir`` (one per
    process, so forked monitors are covered too) and any finding makes the process fail."""
    return {"ASAN_OPTIONS": f"log_path={report_dir}/asan:detect_leaks=1:abort_on_error=0:exitcode=99:"
                            "verify_asan_link_order=0:detect_stack_use_after_return=1",
            "UBSAN_OPTIONS": f"log_path={report_dir}/ubsan:halt_on_error=1:print_stacktrace=1"}


def tsan_env(report_dir: str) -> dict:
    """Environment for a ``*-tsan`` binary: one report file per process, any race fails it."""
    supp = HERE / "tsan.supp"  # vendor-library findings only, each one justified in the file
    return {"TSAN_OPTIONS": f"log_path={report_dir}/tsan:halt_on_error=1:exitcode=66:second_deadlock_stack=1:"
                            f"suppressions={supp}"}


def tsan_argv(exe: str, *args: str) -> list[str]:
    """Command line for a ``*-tsan`` binary: under ``setarch -R`` (no address randomisation) when
    available -- ThreadSanitizer aborts with "unexpected memory mapping" on kernels whose mmap
    randomisation places libraries outside its shadow layout (seen on the MI355X boxes)."""
    import platform

    sa = shutil.which("setarch")
    return ([sa, platform.machine(), "-R"] if sa else []) + [exe, *args]


def path_of(name: str) -> Path:
    return TARGETS[name][0]


def _build_one(name: str, force: bool) -> tuple[str, str | None]:
    out, cmd = TARGETS[name]
    srcs = [Path(c) for c in cmd if c.endswith((".cpp", ".hip"))] + \
        DEPS.get(name.replace("-asan", "").replace("-tsan", ""), [])
    if not force and out.exists() and all(out.stat().st_mtime >= s.stat().st_mtime for s in srcs):
        return name, None
    if shutil.which(cmd[0]) is None and not Path(cmd[0]).exists():
        return name, f"compiler {cmd[0]} not found"
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_name(out.name + ".tmp")
    r = subprocess.run(cmd + ["-o", str(tmp)], capture_output=True, text=True)
    if r.returncode != 0:
        return name, r.stderr[-3000:]
    os.replace(tmp, out)
    return name, None


def build_all(force: bool = False, strict: bool = True) -> dict[str, str | None]:
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        results = dict(ex.map(lambda n: _build_one(n, force), [n for n in TARGETS if n not in SANITIZED]))
    errs = {k: v for k, v in results.items() if v}
    for k, v in errs.items():
        print(f"[native] {k}: FAILED\n{v}", file=sys.stderr)
    if errs and strict:
        raise RuntimeError(f"native build failed: {sorted(errs)}")
    return results


def th_run_binary() -> str:
    """Path of the th-run supervisor (built on demand; falls back to PATH)."""
    p = path_of("th-run")
    if not p.exists():
        try:
            _build_one("th-run", False)
        except Exception:  # noqa: BLE001
            pass
    if p.exists():
        return str(p)
    return shutil.which("th-run") or "th-run"


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("[native] built:", ", ".join(str(v[0]) for n, v in TARGETS.items() if n not in SANITIZED))
