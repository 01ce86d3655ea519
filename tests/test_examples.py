"""The examples/ launch recipes, end to end on CPU: every template is generated through the API
(POST /jobs/{id}/tasks/generate), and the generated command lines are run through ``bash -lc``
exactly as th-run runs them -- with 127.0.0.1 for the node names and gloo for RCCL."""
import json
import os
import re
import socket
import subprocess
from pathlib import Path

import pytest

from tests.helpers import api

ROOT = Path(__file__).resolve().parents[1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture()
def job_as(client, new_user, auth_headers, new_job):
    h = auth_headers(new_user)
    return lambda body: api(client, "post", f"/jobs/{new_job.id}/tasks/generate", h, body)


def _local(line: str, port: int) -> str:
    line = re.sub(r"node-[ab]", "127.0.0.1", line)
    line = line.replace("--backend=nccl", "--backend=gloo")
    line = re.sub(r":(29500|20011)\b", f":{port}", line)
    return line.replace(" torchrun ", " python -m torch.distributed.run ")


def _run_all(lines, timeout=240):
    env = {**os.environ, "PYTHONPATH": str(ROOT), "OMP_NUM_THREADS": "1"}
    procs = [subprocess.Popen(["bash", "-lc", l], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for l in lines]
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=timeout)
        outs.append((p.returncode, out))
    return outs


def test_pytorch_torch_template_runs(job_as):
    st, body = job_as({"template": "torch", "command": "python examples/PyTorch/train_ddp.py",
                       "placements": [{"hostname": "node-a", "gpus": [0, 1]}, {"hostname": "node-b", "gpus": [3]}]})
    assert st == 201 and len(body["tasks"]) == 3
    port = _port()
    lines = [_local(t["fullCommand"], port) + " --steps 3 --width 64" for t in body["tasks"]]
    assert all(f"--init-method=tcp://127.0.0.1:{port}" in l and "--world-size=3" in l for l in lines)
    outs = _run_all(lines)
    for rc, out in outs:
        assert rc == 0, out[-2000:]
        assert "replicas_identical=True" in out and "world=3" in out


def test_pytorch_torchrun_template_runs(job_as):
    st, body = job_as({"template": "torchrun", "module": "examples.PyTorch.train_ddp",
                       "placements": [{"hostname": "node-a", "gpus": [0, 1]}, {"hostname": "node-b", "gpus": "auto:1"}]})
    assert st == 201 and len(body["tasks"]) == 2
    cmds = [t["fullCommand"] for t in body["tasks"]]
    assert cmds[1].startswith("HIP_VISIBLE_DEVICES=auto:1 ") and "--nnodes=2" in cmds[0]
    port = _port()
    lines = [_local(c, port).replace("--nnodes=2", "--nnodes=2 --max-restarts=0") + " --steps 3 --width 64"
             for c in cmds]
    outs = _run_all(lines)
    text = "\n".join(o for _, o in outs)
    assert all(rc == 0 for rc, _ in outs), text[-3000:]
    assert text.count("replicas_identical=True world=3") + text.count("world=3 backend=gloo replicas_identical=True") >= 3


def test_tf2_tf_config_survives_the_shell(job_as):
    st, body = job_as({"template": "tf2", "command": "python examples/TF_CONFIG/tf_config_worker.py",
                       "placements": [{"hostname": "node-a", "role": "chief", "gpus": [0]},
                                      {"hostname": "node-a", "role": "worker", "gpus": [1]},
                                      {"hostname": "node-b", "role": "worker", "gpus": [0]}]})
    assert st == 201
    outs = _run_all([t["fullCommand"] for t in body["tasks"]], timeout=60)
    got = [re.search(r"task=(\S+) address=(\S+) workers=(\d+) gpus=(\S*)", o).groups() for _, o in outs]
    assert [rc for rc, _ in outs] == [0, 0, 0]
    assert got == [("chief:0", "node-a:2222", "3", "0"), ("worker:0", "node-a:2223", "3", "1"),
                   ("worker:1", "node-b:2222", "3", "0")]


def test_tf1_clusterspec_flags(job_as):
    st, body = job_as({"template": "tf1", "command": "python examples/TensorFlow_ClusterSpec/clusterspec_worker.py",
                       "placements": [{"hostname": "node-a", "role": "ps"},
                                      {"hostname": "node-a", "role": "worker", "gpus": [1]},
                                      {"hostname": "node-b", "role": "worker", "gpus": [0]}]})
    assert st == 201
    outs = _run_all([t["fullCommand"] for t in body["tasks"]], timeout=60)
    assert [rc for rc, _ in outs] == [0, 0, 0], outs
    heads = [o.splitlines()[0] for _, o in outs]
    assert heads[0].startswith("[tf1] job=ps:0 address=node-a:2222 ps=1 workers=2 gpus=''")
    assert heads[2].startswith("[tf1] job=worker:1 address=node-b:2224") and heads[2].endswith("gpus='0'")


@pytest.mark.parametrize("template,placement", [
    ("tf2", {"hostname": "node-a", "role": "chief", "gpus": "auto:1"}),
    ("tf1", {"hostname": "node-a", "role": "worker", "gpuCount": 2}),
    ("torch", {"hostname": "node-a", "gpus": "auto:2"}),
    ("torchrun", {"hostname": "node-a", "gpus": "auto"}),       # no count
    ("torchrun", {"hostname": "node-a", "gpus": "auto:x"}),
])
def test_count_placements_are_rejected_outside_torchrun(job_as, template, placement):
    """ADVICE r2 (job.py:386): device counts are a torchrun-only feature; elsewhere (and for a bare
    ``auto``) the request is refused with a 4xx instead of pinning GPU 0 or failing with a 500."""
    st, body = job_as({"template": template, "placements": [placement]})
    assert 400 <= st < 500, body


def test_torchrun_count_placement_is_accepted(job_as):
    st, body = job_as({"template": "torchrun", "placements": [{"hostname": "node-a", "gpus": "auto:2"}]})
    assert st == 201 and body["tasks"][0]["fullCommand"].startswith("HIP_VISIBLE_DEVICES=auto:2 ")
