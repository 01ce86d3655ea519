"""Dashboard server, CLI entry points, doctor/benchmark harnesses (reference ``cli.py``,
``app/web/AppServer.py``)."""
import json
import re
import shutil
import subprocess

import pytest
from click.testing import CliRunner

from tensorhive_fixed_amd import __version__


def test_web_app_serves_spa_and_config(cfg):
    from tensorhive_fixed_amd.app.server import STATIC, create_web_app

    c = create_web_app("http://h:1111/api").test_client()
    r = c.get("/static/config.json")
    assert r.status_code == 200 and r.get_json() == {"apiPath": "http://h:1111/api", "version": __version__}
    r = c.get("/")
    assert r.status_code == 200 and b"TensorHive" in r.data
    r = c.get("/reservations/deep/link")  # SPA fallback
    assert r.status_code == 200 and b"<script>" in r.data
    assert (STATIC / "index.html").exists()


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_spa_script_parses(tmp_path):
    from tensorhive_fixed_amd.app.server import STATIC

    js = re.search(r"<script>(.*)</script>", (STATIC / "index.html").read_text(), re.S).group(1)
    (tmp_path / "spa.js").write_text(js)
    r = subprocess.run(["node", "--check", str(tmp_path / "spa.js")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_spa_uses_only_known_endpoints():
    """Every API path the dashboard calls exists in the spec (catches drift between the two)."""
    from tensorhive_fixed_amd.api.spec import EXTRA_OPERATIONS, OPERATIONS
    from tensorhive_fixed_amd.app.server import STATIC

    src = (STATIC / "index.html").read_text()
    pats = [re.compile("^" + re.sub(r"\{[^}]+\}", "[^/?]+", op.path) + "$") for op in list(OPERATIONS) + list(EXTRA_OPERATIONS)]
    used = set(re.findall(r'call\("(?:GET|POST|PUT|DELETE)", [`"](/[^`"?]*)', src))
    used |= set(re.findall(r'"(/(?:users|groups|restrictions|schedules|resources))"', src))
    assert used
    for u in used:
        u = re.sub(r"\$\{[^}]+\}", "X", u.replace("${pick.value}", "users/X"))
        assert any(p.match(u) for p in pats), u


def test_cli_version_and_help():
    from tensorhive_fixed_amd.cli import main

    r = CliRunner().invoke(main, ["--version"])
    assert r.exit_code == 0 and r.output.strip() == __version__
    r = CliRunner().invoke(main, ["--help"])
    assert r.exit_code == 0 and "doctor" in r.output and "bench" in r.output


def test_cli_create_user_and_key(cfg, tables, monkeypatch, tmp_path):
    from tensorhive_fixed_amd.cli import main
    from tensorhive_fixed_amd.models.orm import Group, User

    monkeypatch.setattr("tensorhive_fixed_amd.database.configure", lambda *a, **k: None)
    inp = "\n".join(["firstadmin", "admin@x.org", "password1", "password1", "y", "y"]) + "\n"
    r = CliRunner().invoke(main, ["-c", str(cfg.directory), "create", "user"], input=inp)
    assert r.exit_code == 0, r.output
    u = User.find_by_username("firstadmin")
    assert set(u.role_names) == {"user", "admin"}
    assert [g.name for g in Group.get_default_groups()] == ["users"]
    assert u.get_restrictions(include_group=True)[0].is_global


def test_cli_profile_prints_rocprof_line(cfg, tables, monkeypatch, new_job_with_task):
    from tensorhive_fixed_amd.cli import main

    monkeypatch.setattr("tensorhive_fixed_amd.database.configure", lambda *a, **k: None)
    tid = new_job_with_task.tasks[0].id
    r = CliRunner().invoke(main, ["-c", str(cfg.directory), "profile", "--task", str(tid)])
    assert r.exit_code == 0, r.output
    assert r.output.startswith("rocprofv3 --kernel-trace --stats") and "-- python train.py --batch_size 32" in r.output
    r = CliRunner().invoke(main, ["-c", str(cfg.directory), "profile", "--task", str(tid), "--pmc", "SQ_WAVES,GRBM_COUNT"])
    assert "--pmc SQ_WAVES GRBM_COUNT" in r.output and "--kernel-trace" not in r.output


def test_cli_profile_keeps_env_in_front_and_creates_task(cfg, tables, monkeypatch, new_job_with_task, new_task_2):
    """rocprofv3 must start the program itself: env assignments go before it, never after `--`."""
    from tensorhive_fixed_amd.cli import main
    from tensorhive_fixed_amd.models.orm import Job, Task

    monkeypatch.setattr("tensorhive_fixed_amd.database.configure", lambda *a, **k: None)
    job = new_job_with_task
    job.add_task(new_task_2)
    r = CliRunner().invoke(main, ["-c", str(cfg.directory), "profile", "--task", str(new_task_2.id), "--create"])
    assert r.exit_code == 0, r.output
    line = r.output.splitlines()[0]
    assert line.startswith("HIP_VISIBLE_DEVICES=0 rocprofv3 --kernel-trace") and line.endswith("-- python eval.py")
    new_id = int(r.output.splitlines()[1].split()[-1])
    t = Task.get(new_id)
    assert t.full_command == line and t.hostname == "node-b" and t.gpu_id == 0
    assert new_id in [x.id for x in Job.get(job.id).tasks]


def test_cli_test_command_with_simulated_nodes(cfg):
    from tensorhive_fixed_amd.cli import main

    r = CliRunner().invoke(main, ["-c", str(cfg.directory), "test"])
    assert r.exit_code == 0 and "OK  node-a" in r.output


def test_poll_latency_benchmark():
    from tensorhive_fixed_amd import benchmarks

    out = benchmarks.poll_latency(requests=30, nodes=2, gpus=8, warmup=2)
    for mode in ("admin_inprocess", "user_inprocess", "user_socket"):
        res = out["results"][mode]["/api/nodes/metrics"]
        assert res["requests"] == 30 and 0 < res["p50_ms"] <= res["p99_ms"]
    assert out["user_visible_gpus"] == 8  # the restricted user sees half of 2 x 8 GPUs


def test_multitenant_benchmark_small():
    from tensorhive_fixed_amd import benchmarks

    out = benchmarks.multitenant(jobs_per_user=3, duration_s=(0.2, 0.4), arrival_s=0.05)
    assert out["jobs"] == out["completed"] == 9
    assert out["queue_wait_p50_ms"] <= out["queue_wait_p99_ms"]
    assert 0 < out["node_gpu_util"] <= 1
    assert out["violations"] == {"mallory": ["bob"]} and out["walled_ttys"] == ["pts/7"]


def test_doctor_reports_without_gpu(monkeypatch):
    from tensorhive_fixed_amd import doctor

    checks = {n: (ok, d) for n, ok, d in doctor.run_checks()}
    assert "rocm" in checks and "torch (ROCm)" in checks
    assert json.dumps([list(c) for c in checks.items()])  # serialisable
