"""Dashboard server, CLI entry points, doctor/benchmark harnesses (reference ``cli.py``,
``app/web/AppServer.py``)."""
import json
import os
import re
import shutil
import subprocess
from pathlib import Path

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
    assert r.status_code == 200 and b'<script type="module" src="/js/main.js">' in r.data
    r = c.get("/js/main.js")
    assert r.status_code == 200 and "javascript" in r.mimetype and b"route()" in r.data
    assert (STATIC / "index.html").exists()


SPA_JS = sorted((Path(__file__).resolve().parents[1] / "tensorhive_fixed_amd" / "app" / "static" / "js").glob("*.js"))
_CALL = re.compile(r'(?:call|raw)\(\s*"(GET|POST|PUT|DELETE)",\s*(["`])(/[^"`]*)\2')


def _spa_calls() -> set[tuple[str, str]]:
    """(method, path regex) of every API request in the dashboard modules; `${...}` is one segment."""
    out = set()
    for f in SPA_JS:
        for m in _CALL.finditer(f.read_text()):
            path = re.sub(r"\$\{[^}]*\}", "\x00", m.group(3))
            out.add((m.group(1), "^" + re.escape(path).replace("\x00", "[^/?]+") + "$"))
    return out


def _instance(path: str) -> str:
    return re.sub(r"\{[^}]+\}", "1", path)


def test_spa_modules_parse():
    assert {f.name for f in SPA_JS} >= {"main.js", "api.js", "ui.js", "nodes.js", "reservations.js", "jobs.js",
                                        "admin.js", "time.js", "launch.js", "chart.js"}
    if shutil.which("node") is None:
        pytest.skip("node not installed")
    for f in SPA_JS:
        r = subprocess.run(["node", "--check", str(f)], capture_output=True, text=True)
        assert r.returncode == 0, (f.name, r.stderr)


def test_spa_uses_only_known_endpoints():
    """Every API request the dashboard makes is an operation of the spec (catches drift)."""
    from tensorhive_fixed_amd.api.spec import EXTRA_OPERATIONS, OPERATIONS

    ops = [(op.method, _instance(op.path)) for op in list(OPERATIONS) + list(EXTRA_OPERATIONS)]
    calls = _spa_calls()
    assert len(calls) > 40
    for method, rx in calls:
        assert any(m == method and re.match(rx, p) for m, p in ops), (method, rx)


# (method, operation) pairs the reference Vue SPA issues (tensorhive/app/web/dev/src: api/*.js,
# components/**/*.vue, main.js); extracted once from its api.request(...) calls.  The dead
# /tasks/{id}/spawn|terminate calls of TasksOverview.vue (no such operations in its spec) are left out.
REFERENCE_SPA_OPERATIONS = [
    ("DELETE", "/groups/{id}"), ("DELETE", "/reservations/{id}"), ("DELETE", "/restrictions/{id}"),
    ("DELETE", "/tasks/{id}"), ("DELETE", "/user/delete/{id}"), ("DELETE", "/user/logout"),
    ("DELETE", "/user/logout/refresh_token"), ("DELETE", "/jobs/{job_id}/tasks/{task_id}"), ("DELETE", "/jobs/{id}"),
    ("GET", "/groups"), ("GET", "/jobs"), ("GET", "/jobs/{id}"), ("GET", "/jobs/{id}/execute"), ("GET", "/jobs/{id}/stop"),
    ("GET", "/nodes/{hostname}/gpu/metrics"), ("GET", "/nodes/{hostname}/cpu/metrics"), ("GET", "/nodes/hostnames"),
    ("GET", "/nodes/metrics"), ("GET", "/reservations"), ("GET", "/resources"), ("GET", "/restrictions"),
    ("GET", "/tasks"), ("GET", "/tasks/{id}"), ("GET", "/tasks/{id}/log"), ("GET", "/user/authorized_keys_entry"),
    ("GET", "/users"), ("GET", "/users/{id}"), ("GET", "/user/refresh"),
    ("POST", "/groups"), ("POST", "/reservations"), ("POST", "/restrictions"), ("POST", "/schedules"),
    ("POST", "/user/create"), ("POST", "/user/login"), ("POST", "/user/ssh_signup"), ("POST", "/jobs/{job_id}/tasks"),
    ("POST", "/jobs"),
    ("PUT", "/groups/{id}"), ("PUT", "/groups/{group_id}/users/{user_id}"), ("DELETE", "/groups/{group_id}/users/{user_id}"),
    ("PUT", "/reservations/{id}"), ("PUT", "/restrictions/{id}"), ("PUT", "/restrictions/{restriction_id}/users/{user_id}"),
    ("PUT", "/restrictions/{restriction_id}/groups/{group_id}"),
    ("PUT", "/restrictions/{restriction_id}/resources/{resource_uuid}"),
    ("PUT", "/restrictions/{restriction_id}/schedules/{schedule_id}"), ("PUT", "/tasks/{id}"), ("PUT", "/user"),
    ("PUT", "/jobs/{id}/dequeue"), ("PUT", "/jobs/{id}/enqueue"), ("PUT", "/jobs/{job_id}/tasks/{task_id}"),
    ("PUT", "/jobs/{id}"),
]


def test_spa_covers_every_reference_spa_operation():
    """The dashboard reaches every operation the reference SPA used, plus the new ones."""
    calls = _spa_calls()
    extra = [("PUT", "/user/password"), ("PUT", "/schedules/{id}"), ("DELETE", "/schedules/{id}"),
             ("POST", "/jobs/{id}/tasks/generate"), ("PUT", "/jobs/{id}/reservation/{reservation_id}"),
             ("GET", "/tasks/{id}/training"), ("GET", "/jobs/templates"), ("GET", "/nodes/topology"),
             ("GET", "/nodes/{hostname}/gpu/processes"), ("PUT", "/restrictions/{restriction_id}/hosts/{hostname}"),
             ("DELETE", "/restrictions/{restriction_id}/users/{user_id}"), ("GET", "/schedules")]
    missing = [(m, p) for m, p in REFERENCE_SPA_OPERATIONS + extra
               if not any(cm == m and re.match(rx, _instance(p)) for cm, rx in calls)]
    assert not missing, missing


def _node_eval(tmp_path, script: str):
    if shutil.which("node") is None:
        pytest.skip("node not installed")
    js = SPA_JS[0].parent
    f = tmp_path / "t.mjs"
    f.write_text(script.replace("@JS@", js.as_uri()))
    r = subprocess.run(["node", str(f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_spa_launch_previews_match_server(tmp_path):
    """launch.js previews (TF_CONFIG, ClusterSpec, rendered command) equal core/launcher.py + Task.render."""
    from tensorhive_fixed_amd.core import launcher

    pl = [{"hostname": "a", "role": "chief", "gpus": [0]}, {"hostname": "a", "role": "worker", "gpus": [1]},
          {"hostname": "b", "role": "worker", "gpus": [0]}, {"hostname": "b", "role": "ps", "gpus": []}]
    out = _node_eval(tmp_path, r"""
import { tf2Preview, tf1Preview, renderCommand, parseSegments, segmentsToText } from "@JS@/launch.js";
const pl = %s;
const segs = parseSegments("HIP_VISIBLE_DEVICES=0,1\nNCCL_DEBUG=WARN\nTF_CONFIG={\"task\":{\"type\":\"chief\"}}", "--nproc_per_node=2\n-m mod\n--flag\n--msg it's done");
console.log(JSON.stringify({ tf2: tf2Preview(pl, 2222), tf1: tf1Preview(pl, 2222), segs,
  cmd: renderCommand("torchrun", segs), back: segmentsToText(segs) }));
""" % json.dumps(pl))
    ref2 = launcher.tf2_tasks([(p["hostname"], p["role"], 0) for p in pl], 2222)
    assert [x["TF_CONFIG"] for x in out["tf2"]] == [
        json.dumps(json.loads(next(e["value"] for e in t["cmdsegments"]["envs"] if e["name"] == "TF_CONFIG")))
        .replace(" ", "") for t in ref2]
    ref1 = launcher.tf1_tasks(["b"], [("a", 0), ("a", 1), ("b", 0)], 2222)
    flags = [" ".join(p["name"] + p["value"] for p in t["cmdsegments"]["params"]) for t in ref1]
    assert [x["flags"] for x in out["tf1"]] == flags
    assert out["segs"]["params"] == [{"name": "--nproc_per_node=", "value": "2"}, {"name": "-m", "value": "mod"},
                                     {"name": "--flag", "value": ""}, {"name": "--msg", "value": "it's done"}]
    assert "TF_CONFIG='{\"task\":{\"type\":\"chief\"}}'" in out["cmd"] and "--msg 'it'\\''s done'" in out["cmd"]
    from tensorhive_fixed_amd.models.orm import Task
    t = Task(command="torchrun", hostname="h")
    assert out["cmd"] == t.render([(e["name"], e["value"]) for e in out["segs"]["envs"]],
                                  [(p["name"], p["value"]) for p in out["segs"]["params"]])
    assert out["back"]["params"].splitlines() == ["--nproc_per_node=2", "-m mod", "--flag", "--msg it's done"]


def test_spa_schedule_and_calendar_math(tmp_path):
    """time.js: UTC<->local schedule round trip, midnight-crossing windows, drag selection across
    days and GPU columns, client-side restriction coverage, usage averages."""
    out = _node_eval(tmp_path, """
import * as T from "@JS@/time.js";
const s = { scheduleDays: ["Monday", "Friday"], hourStart: "23:00", hourEnd: "02:00" };
const loc = T.scheduleToLocal(s, 120), back = T.scheduleToUtc(loc, 120);
const west = T.scheduleToLocal({ scheduleDays: ["Monday"], hourStart: "01:00", hourEnd: "05:00" }, -300);
const days = [new Date("2026-01-05T00:00:00Z"), new Date("2026-01-06T00:00:00Z")];
const sel = T.dragSelection({ day: 1, gpu: 2, slot: 3 }, { day: 0, gpu: 0, slot: 46 }, days, ["g0", "g1", "g2", "g3"], 30);
const r = [{ isGlobal: false, resources: [{ id: "g1" }], startsAt: "2026-01-01T00:00:00Z", endsAt: null,
             schedules: [{ scheduleDays: ["Monday"], hourStart: "08:00", hourEnd: "18:00" }] }];
console.log(JSON.stringify({ loc, back, west, sel,
  inWrap: [T.inSchedule(s, "2026-01-06T01:00:00Z"), T.inSchedule(s, "2026-01-06T03:00:00Z"), T.inSchedule(s, "2026-01-05T23:30:00Z")],
  allow: [T.allowedWindow(r, "g1", "2026-01-05T09:00:00Z", "2026-01-05T12:00:00Z"),
          T.allowedWindow(r, "g1", "2026-01-05T17:00:00Z", "2026-01-05T19:00:00Z"),
          T.allowedWindow(r, "g2", "2026-01-05T09:00:00Z", "2026-01-05T10:00:00Z")],
  lay: T.layoutDay([{ start: "2026-01-04T22:00:00Z", end: "2026-01-05T06:00:00Z" }], days[0]),
  use: T.usageSummary([{ gpuUtilAvg: 80, memUtilAvg: 40 }, { gpuUtilAvg: 60, memUtilAvg: null }, { gpuUtilAvg: null }]),
  valid: [T.validReservationRange("2026-01-05T00:00:00Z", "2026-01-05T00:20:00Z"), T.validReservationRange("2026-01-05T00:00:00Z", "2026-01-05T01:00:00Z")] }));
""")
    assert out["loc"]["hourStartLocal"] == "01:00" and out["loc"]["hourEndLocal"] == "04:00"
    assert out["loc"]["scheduleDaysLocal"] == ["Tuesday", "Saturday"]
    assert out["back"] == {"scheduleDays": ["Monday", "Friday"], "hourStart": "23:00", "hourEnd": "02:00"}
    assert out["west"]["scheduleDaysLocal"] == ["Sunday"] and out["west"]["hourStartLocal"] == "20:00"
    assert out["sel"] == {"start": "2026-01-05T23:00:00.000Z", "end": "2026-01-06T02:00:00.000Z", "gpus": ["g0", "g1", "g2"]}
    assert out["inWrap"] == [True, False, True]
    assert out["allow"] == [True, False, False]
    assert out["lay"] == [{"r": {"start": "2026-01-04T22:00:00Z", "end": "2026-01-05T06:00:00Z"}, "top": 0, "height": 0.25}]
    assert out["use"] == {"gpuUtilAvg": 70, "memUtilAvg": 40, "samples": 2}
    assert out["valid"][0] and out["valid"][1] is None


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


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_spa_end_to_end_against_live_api(tmp_path):
    """The dashboard modules run under node (tests/spa/dom.mjs: a minimal DOM + fetch over http)
    against a real threaded API server with a file database: every view renders, and users /
    schedules / groups are created through their dialogs, a drag over two GPU columns reserves
    both, the reservation card edits it, a job gets a task, a duplicate and three TF2 tasks from the
    launch editor, the router shows the account page, the password changes and logout revokes."""
    import threading
    from datetime import timedelta

    from werkzeug.serving import make_server

    from tensorhive_fixed_amd import benchmarks
    from tensorhive_fixed_amd.api.app import create_app
    from tensorhive_fixed_amd.core.daemon import Daemon
    from tensorhive_fixed_amd.core.telemetry import StubBackend
    from tensorhive_fixed_amd.models.orm import Restriction, Role, User
    from tensorhive_fixed_amd.utils import dates

    hosts = {"node-a": "fake"}
    with benchmarks.sandbox(hosts, stub_gpus=4) as (cfg, _d):
        stub = StubBackend(gpus_per_host=4)
        daemon = Daemon(cfg, backends={h: stub for h in hosts}, init_key=False, test_ssh=False)
        daemon.infrastructure.publish("node-a", stub.sample("node-a"))
        app = create_app(daemon)
        admin = User(username="spaadmin", password="admin password 1", email="a@example.org",
                     roles=[Role(name="user"), Role(name="admin")])
        admin.save()
        user = User(username="spaalice", password="alice password 1", email="alice@example.org",
                    roles=[Role(name="user")])
        user.save()
        r = Restriction(name="everything", starts_at=dates.utcnow() - timedelta(days=1), is_global=True)
        r.save()
        r.apply_to_user(user)
        r.apply_to_user(admin)
        app.test_client().get("/api/nodes/metrics", headers=benchmarks._headers(admin))  # registers the GPUs
        srv = make_server("127.0.0.1", 0, app, threaded=True)
        th = threading.Thread(target=srv.serve_forever, daemon=True)
        th.start()
        try:
            scen = Path(__file__).resolve().parent / "spa" / "scenario.mjs"
            p = subprocess.run(["node", str(scen), f"http://127.0.0.1:{srv.server_port}", "spaadmin",
                                "admin password 1", "spaalice", "alice password 1"],
                               capture_output=True, text=True, timeout=240, env={**os.environ, "TZ": "UTC"})
        finally:
            srv.shutdown()
            daemon.shutdown()
    assert p.returncode == 0, p.stderr[-3000:]
    doc = json.loads(p.stdout.strip().splitlines()[-1])
    (tmp_path / "spa_scenario.json").write_text(json.dumps(doc, indent=1))
    bad = [s for s in doc["steps"] if not s["ok"]]
    assert not doc["errors"], (doc["errors"][:3], [(s["name"], s["ok"], str(s.get("detail"))[:150]) for s in doc["steps"]])
    assert not bad, bad
    assert len(doc["steps"]) >= 23 and doc["requests"] > 60


def test_scaling_harness_efficiency_and_skips():
    from tensorhive_fixed_amd import benchmarks

    fake = {1: 24700.0, 2: 49000.0, 4: 97500.0, 8: 193000.0}
    out = benchmarks.scaling([1, 2, 4, 8], available=4,
                             run=lambda n: {"value": fake[n], "ms_per_step": 1000.0, "config": {"zero": int(n > 1)}})
    assert [p["n_gpus"] for p in out["points"]] == [1, 2, 4] and out["skipped"] == [8]
    eff = {p["n_gpus"]: p["efficiency"] for p in out["points"]}
    assert eff[1] == 1.0 and abs(eff[2] - 49000 / 49400) < 1e-4 and abs(eff[4] - 97500 / 98800) < 1e-4
    assert out["points"][2]["tokens_per_sec_per_gpu"] == 24375.0 and out["points"][1]["zero"] == 1


def test_scaling_bucket_sweep_records_each_size_and_the_best():
    from tensorhive_fixed_amd import benchmarks

    calls = []

    def run(n, b):
        calls.append((n, b))
        v = 24700.0 * n * (1.0 if n == 1 else (0.97 if b == 256 else 0.93))
        return {"value": v, "ms_per_step": 1000.0, "config": {"zero": int(n > 1)},
                "dist": {"world_size": n, "distinct_devices": n}}

    out = benchmarks.scaling([1, 2, 8], available=8, run=run, bucket_mbs=[64, 256])
    assert calls.count((1, 64)) == 1 and (1, 256) not in calls  # the 1-GPU point runs once
    assert sorted((p["n_gpus"], p["bucket_mb"]) for p in out["points"]) == [(1, 64), (2, 64), (2, 256), (8, 64), (8, 256)]
    assert out["best_bucket_mb"] == {"2": 256.0, "8": 256.0} and out["bucket_sweep_mb"] == [64.0, 256.0]
    p8 = next(p for p in out["points"] if p["n_gpus"] == 8 and p["bucket_mb"] == 256)
    assert p8["efficiency"] == 0.97 and p8["distinct_devices"] == 8 and p8["world_size"] == 8


SHELL_CASES = ['"a b"', "/data/*.tfrecord", "$HOME/x", "~/ckpt", "a b", "a;b", '"a;b"', "it's", "--x=1",
               '{"a": 1}', '{"cluster":{"w":["h:1"]}}', "a\\ b", "x\\", "'quoted already'", "a&&b", "(x)",
               "tcp://127.0.0.1:29500", "", "{a,b}", 'say "hi there"', "#1", "a#b", "x{1..3}",
               "{a}", "${HOME}", "--tag=#x", "{a,{c}}", "x{a,{b}}y", "{{a}}", "{x{1..2}}"]


def test_shell_value_keeps_one_word_values_and_js_agrees(tmp_path):
    """ADVICE r2 (orm.py:56): values the shell reads as ONE word are passed verbatim (user quoting,
    globs, $VARS keep their meaning); splitting values, unbalanced quotes, bare operators and JSON
    documents are single-quoted.  launch.js renders every case identically."""
    import shlex as _shlex

    from tensorhive_fixed_amd.models.orm import _shell_value

    expect = {'"a b"': '"a b"', "/data/*.tfrecord": "/data/*.tfrecord", "$HOME/x": "$HOME/x", "a b": "'a b'",
              "a;b": "'a;b'", '"a;b"': '"a;b"', "it's": "'it'\\''s'", '{"a": 1}': "'{\"a\": 1}'",
              "'quoted already'": "'quoted already'", "x\\": "'x\\'", "": "",
              # a leading # would comment out the rest of the command, a brace list
              # would expand into several words (shlex does neither, so check the rendering)
              "#1": "'#1'", "a#b": "a#b", "{a,b}": "'{a,b}'", "x{1..3}": "'x{1..3}'", "{a}": "{a}",
              "${HOME}": "${HOME}",
              # nested braces -- the OUTER list expands (bash: `a` and `{c}`)
              "{a,{c}}": "'{a,{c}}'", "x{a,{b}}y": "'x{a,{b}}y'", "{{a}}": "{{a}}", "{x{1..2}}": "'{x{1..2}}'"}
    for v, want in expect.items():
        assert _shell_value(v) == want, v
    for v in SHELL_CASES:  # every rendered value is exactly one shell word
        if v:
            assert len(_shlex.split(_shell_value(v))) == 1, v
    # ... and bash agrees (brace expansion and comments are bash's, not shlex's)
    import subprocess as _sp

    script = "\n".join(f"set -- {_shell_value(v)} END; echo $#" for v in SHELL_CASES if v)
    counts = _sp.run(["bash", "--norc", "-c", script], capture_output=True, text=True, cwd=tmp_path).stdout.split()
    assert counts == ["2"] * len([v for v in SHELL_CASES if v]), list(zip(SHELL_CASES, counts))
    out = _node_eval(tmp_path, r"""
import { shellValue } from "@JS@/launch.js";
console.log(JSON.stringify(%s.map(shellValue)));
""" % json.dumps(SHELL_CASES))
    assert out == [_shell_value(v) for v in SHELL_CASES]
