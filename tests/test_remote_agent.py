"""Remote-node telemetry through the node agent (round-3 verdict item 4).

The daemon reaches a remote node over one SSH channel; here the "SSH" hop is a transport whose
stream argv runs the command through ``bash -c`` on this machine (what ``ssh host CMD`` does on
the node), and the agent samples a scripted stub node.  What must arrive at the daemon is the
node's complete entry: probe-derived keys and the node's own in-task HBM counter files, merged
and authenticated on the node."""
import json
import os
import sys
import time

import pytest

from tensorhive_fixed_amd.core.telemetry import RemoteBackend
from tensorhive_fixed_amd.core.transport import Transport, TransportManager

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AGENT = f"{sys.executable} -m tensorhive_fixed_amd.agent"


class BashSSH(Transport):
    """``ssh node CMD`` stand-in: the remote command runs through bash on this machine."""

    def __init__(self, host):
        self.host = host
        self.cmds = []

    def stream_argv(self, command, user=None):
        self.cmds.append(command)
        return ["bash", "-c", f"cd {ROOT} && {command}"]

    def run(self, command, timeout=None, user=None, env=None):
        import subprocess

        from tensorhive_fixed_amd.core.transport import Result

        self.cmds.append(command)
        p = subprocess.run(["bash", "-c", f"cd {ROOT} && {command}"], capture_output=True, text=True, timeout=timeout)
        return Result(self.host, p.stdout, p.stderr, p.returncode)


def _tm(host="gpu-node-7"):
    t = BashSSH(host)
    return TransportManager({host: t}), t


def _wait_sample(be, host, pred=lambda e: True, timeout=60.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        e = be.sample(host)
        if e is not None and pred(e):
            return e
        time.sleep(0.1)
    raise AssertionError(f"no sample from {host}: {be.errors}")


def _counter_file(tmp_path, pid, bdf, rd, wr):
    (tmp_path / f"th-hbm-{pid}.json").write_text(json.dumps(
        {"pid": pid, "ts_ns": int(time.time() * 1e9), "window_ms": 1000.0,
         "gpus": [{"bdf": bdf, "rd_bytes": rd, "wr_bytes": wr}]}))


def test_agent_stream_carries_probe_and_counted_hbm(tmp_path):
    me = os.getpid()
    _counter_file(tmp_path, me, "0000:05:00.0", 1.5e12, 0.5e12)  # GPU 0's bdf in the stub
    tm, t = _tm()
    args = (f"--backend stub --stub-gpus 8 --stub-process 0:{me}:alice:17 --stub-process 1:424242:mallory "
            f"--hbm-glob '{tmp_path}/th-hbm-*.json'")
    be = RemoteBackend(tm, stream_ms=100, mode="agent", agent_cmd=AGENT, agent_args=args)
    try:
        e = _wait_sample(be, "gpu-node-7")
        gpus = sorted(e["GPU"].values(), key=lambda g: g["index"])
        assert len(gpus) == 8 and all(len(u) == 40 for u in e["GPU"])
        g0, g1 = gpus[0]["metrics"], gpus[1]["metrics"]
        assert g0["hbm_bw_source"]["value"] == "counters" and g0["hbm_bw"]["value"] == 2000.0
        assert g1["hbm_bw_source"]["value"] == "umc_activity"  # a foreign tenant, nothing counted
        assert "mfma_busy" in g0 and "mfma_contention" in g0 and "hbm_contention" in g0
        assert [p["owner"] for p in gpus[0]["processes"]] == ["alice"] and gpus[0]["processes"][0]["task_id"] == "17"
        assert be.node_mode("gpu-node-7") == "agent"
        assert t.cmds[0].startswith(f"exec {AGENT} --stream 100 --host gpu-node-7")
        # the stream keeps going: a newer line replaces the older one
        ts0 = be._latest["gpu-node-7"][0]
        _wait_sample(be, "gpu-node-7", lambda _: be._latest["gpu-node-7"][0] > ts0)
    finally:
        be.close()


def test_agent_unavailable_falls_back_to_th_smi(tmp_path):
    tm, t = _tm("old-node")
    fake_smi = tmp_path / "th-smi"
    fake_smi.write_text("#!/bin/bash\nwhile true; do echo '{\"gpus\": [{\"index\": 0, \"uuid\": \"GPU-"
                        + "a" * 36 + "\", \"metrics\": {}, \"processes\": []}]}'; sleep 0.05; done\n")
    fake_smi.chmod(0o755)
    be = RemoteBackend(tm, th_smi=str(fake_smi), stream_ms=50, mode="agent", agent_cmd="no-such-agent-binary")
    try:
        e = _wait_sample(be, "old-node")
        assert be.node_mode("old-node") == "th-smi" and list(e["GPU"]) == ["GPU-" + "a" * 36]
    finally:
        be.close()


def test_stale_stream_reports_the_node_down(tmp_path):
    """A channel that stops delivering (hung node, frozen agent) turns the node into 'down'."""
    hang = tmp_path / "agent-then-hang"
    hang.write_text(f"#!/bin/bash\n{AGENT} --once \"$@\"\nexec sleep 60\n")
    hang.chmod(0o755)
    tm, t = _tm("n1")
    be = RemoteBackend(tm, stream_ms=100, mode="agent", agent_cmd=str(hang), agent_args="--backend stub --stub-gpus 2",
                       stale_s=0.6)
    try:
        _wait_sample(be, "n1")
        time.sleep(1.0)
        assert be.sample("n1") is None
        # the silent-but-alive channel is killed and the next sample reconnects
        n = len(t.cmds)
        first = be._latest["n1"][0]
        _wait_sample(be, "n1", timeout=30)
        assert len(t.cmds) > n and be._latest["n1"][0] > first
    finally:
        be.close()


def test_one_shot_agent_mode(tmp_path):
    tm, t = _tm("n2")
    be = RemoteBackend(tm, stream_ms=None, mode="agent", agent_cmd=AGENT, agent_args="--backend stub --stub-gpus 3")
    e = be.sample("n2")
    assert e is not None and len(e["GPU"]) == 3 and "--once" in t.cmds[0]


def test_daemon_builds_agent_backends_for_ssh_nodes(cfg):
    from tensorhive_fixed_amd.core.telemetry import make_backend

    tm = TransportManager.from_config({"gpu9": {"user": "th", "port": 22, "transport": "ssh"}}, None, None, 5.0)
    be = make_backend("auto", "gpu9", tm, probe=True, probe_period=0.5, stream_ms=250, task_hbm=True)
    assert isinstance(be, RemoteBackend) and be.mode == "agent"
    assert "--probe" in be.agent_args and "--probe-period 0.5" in be.agent_args and "--task-hbm" in be.agent_args
    argv = be._argv("gpu9")
    assert argv[0] == "ssh" and argv[-1].startswith("exec python3 -m tensorhive_fixed_amd.agent --stream 250")


@pytest.mark.parametrize("flag", ["--once", "--stream 50"])
def test_agent_cli_emits_entries(flag):
    import subprocess

    cmd = f"{AGENT} {flag} --backend stub --stub-gpus 2 --host hx"
    p = subprocess.Popen(["bash", "-c", cmd], stdout=subprocess.PIPE, text=True, cwd=ROOT)
    line = p.stdout.readline()
    p.stdout.close()  # the channel closes: a streaming agent must exit by itself (EPIPE)
    assert p.wait(timeout=30) == 0
    doc = json.loads(line)
    assert doc["v"] == 1 and doc["host"] == "hx" and len(doc["entry"]["GPU"]) == 2
