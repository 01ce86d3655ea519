"""HBM bandwidth telemetry against a timed device stream (round-2 verdict, missing item 4):
libthsmi's ``hbm_bw`` (calibrated ``mem_activity_acc`` rate) must be within +-15 % of the GB/s a
tenant process measures for its own copy loop."""
import json
import subprocess
import sys
import time
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[2]


def test_hbm_bw_tracks_a_timed_copy_stream():
    from tensorhive_fixed_amd.core.telemetry import AmdSmiBackend

    be = AmdSmiBackend()
    try:
        p = subprocess.Popen([sys.executable, str(ROOT / "scripts" / "hbm_stream.py"), "5", "copy"],
                             stdout=subprocess.PIPE, text=True, cwd=ROOT)
        time.sleep(2.0)  # past allocation + warm-up
        vals = []
        t_end = time.time() + 2.5
        while time.time() < t_end:
            doc = be.sample("localhost")
            g = sorted(doc["GPU"].values(), key=lambda g: g["index"])[0]
            v = g["metrics"]["hbm_bw"]["value"]
            if v is not None:
                vals.append(v)
            time.sleep(0.25)
        out, _ = p.communicate(timeout=60)
        stream = json.loads(out.strip().splitlines()[-1])
    finally:
        be.close()
    assert vals, "hbm_bw never reported"
    measured = sorted(vals)[len(vals) // 2]
    print(f"hbm_bw telemetry median {measured:.0f} GB/s vs timed stream {stream['GBps']:.0f} GB/s")
    assert abs(measured - stream["GBps"]) <= 0.15 * stream["GBps"], (vals, stream)
