"""Run every GPU-side *-tsan binary with halt_on_error=0 (all reports, not just the first), the
suppressions of native/tsan.supp applied; reports under gpurun_out/r03/tsan_all/."""
import os
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tensorhive_fixed_amd.native.build import _build_one, path_of, tsan_argv, tsan_env  # noqa: E402

out = Path("gpurun_out/r03/tsan_all")
out.mkdir(parents=True, exist_ok=True)
env = {**os.environ, **tsan_env(str(out.resolve()))}
env["TSAN_OPTIONS"] = env["TSAN_OPTIONS"].replace("halt_on_error=1", "halt_on_error=0")
for name, args in (("thsmi-stress-tsan", ["--iters", "40"]),
                   ("th-counters-tsan", ["--count", "3", "--window", "100", "--period", "200"])):
    _, err = _build_one(name, False)
    assert err is None, err
    r = subprocess.run(tsan_argv(str(path_of(name)), *args), capture_output=True, text=True, timeout=300, env=env)
    print(name, "rc", r.returncode, r.stdout[-300:].strip())
for p in sorted(out.iterdir()):
    txt = p.read_text()
    print(p.name, txt.count("WARNING: ThreadSanitizer"), "reports")
