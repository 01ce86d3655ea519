// Jobs and tasks (reference: views/JobsOverview.vue, jobs_overview/JobsTable.vue, JobBulkActions.vue,
// JobCrudActions.vue, JobDetailsView.vue, job_details_view/job_info/*, job_tasks/TaskCreate.vue,
// TaskDuplicate.vue, TaskLog.vue, views/TasksOverview.vue).
//
// Overview: every job of the user (admins: of a chosen user or everyone) with bulk run / stop /
// kill / enqueue / dequeue / delete.  Details (10 s refresh, JobDetailsView.vue:121-127): edit
// name, description and the start/stop schedule; task table with edit, duplicate, detach, delete,
// a log viewer that follows the file every 5 s (TaskLog.vue:121) and the training curve parsed
// from the task's log (GET /tasks/{id}/training).  Task creator: host + GPU picker fed by the live
// node metrics (occupied GPUs marked), "auto:N" devices chosen by the allocator at launch, launch
// templates, env/param segment editor with a rendered preview, restart policy.  Distributed
// launch editor: torchrun / torch ranks / TF2 TF_CONFIG / TF1 ClusterSpec over a placement table,
// with the TF_CONFIG / ClusterSpec previewed before POST /jobs/{id}/tasks/generate creates them.
"use strict";
import { S, call, qs } from "./api.js";
import { LineChart, fmtNum } from "./chart.js";
import { gpuArg, parseSegments, renderCommand, segmentsToText, tf1Preview, tf2Preview, worldSize } from "./launch.js";
import { fmtDateTime, toApi } from "./time.js";
import { View, attempt, card, confirmBox, dtInput, dtValue, errToast, field, h, input, modal, pill, select, statusPill, table, toast } from "./ui.js";

let TEMPLATES = null;
async function templates() {
  if (!TEMPLATES) TEMPLATES = (await call("GET", "/jobs/templates").catch(() => ({ templates: {} }))).templates || {};
  return TEMPLATES;
}

const ACTIONS = {
  run: id => call("GET", `/jobs/${id}/execute`), stop: id => call("GET", `/jobs/${id}/stop` + qs({ gracefully: true })),
  kill: id => call("GET", `/jobs/${id}/stop` + qs({ gracefully: false })), enqueue: id => call("PUT", `/jobs/${id}/enqueue`),
  dequeue: id => call("PUT", `/jobs/${id}/dequeue`), delete: id => call("DELETE", `/jobs/${id}`),
};
const jobAction = (name, id) => ACTIONS[name](id);

// ------------------------------------------------------------------------ overview
export function jobsView(root, params) {
  if (params && params.id) return jobDetailsView(root, +params.id);
  const v = new View(root);
  const box = h("div", {});
  const chosen = new Set();
  let users = [], jobs = [];
  const userSel = select([["mine", "my jobs"], ["all", "all users"]], localStorage.getItem("th.jobs.who") || "mine");
  userSel.addEventListener("change", () => { localStorage.setItem("th.jobs.who", userSel.value); load(); });

  async function load() {
    const who = userSel.value;
    const d = await call("GET", "/jobs" + qs({ userId: who === "all" ? undefined : who === "mine" ? S.me : +who })).catch(e => { errToast(e); return null; });
    if (!v.alive || !d) return;
    jobs = d.jobs || [];
    // a job document carries no tasks (reference models/Job.py as_dict): mine come from one
    // GET /tasks, another user's per job
    const byJob = {};
    if (who === "mine") {
      const t = await call("GET", "/tasks" + qs({ syncAll: false })).catch(() => ({ tasks: [] }));
      (t.tasks || []).forEach(x => (byJob[x.jobId] = byJob[x.jobId] || []).push(x));
    } else {
      await Promise.all(jobs.slice(0, 100).map(j => call("GET", "/tasks" + qs({ jobId: j.id, syncAll: false }))
        .then(t => { byJob[j.id] = t.tasks || []; }).catch(() => null)));
    }
    if (!v.alive) return;
    jobs.forEach(j => { j.tasks = byJob[j.id] || []; });
    const uname = id => (users.find(u => u.id === id) || {}).username || id;
    box.replaceChildren(table([
      { label: h("input", { type: "checkbox", onchange: e => { jobs.forEach(j => e.target.checked ? chosen.add(j.id) : chosen.delete(j.id)); load(); } }),
        render: j => { const c = h("input", { type: "checkbox", checked: chosen.has(j.id) });
          c.addEventListener("click", e => e.stopPropagation());
          c.addEventListener("change", () => c.checked ? chosen.add(j.id) : chosen.delete(j.id)); return c; } },
      { label: "id", key: "id" }, { label: "name", render: j => h("a", { href: `#jobs/${j.id}` }, j.name) },
      { label: "owner", render: j => uname(j.userId) },
      { label: "status", render: j => [statusPill(j.status), j.isQueued ? pill("queued", "warn") : null] },
      { label: "tasks", render: j => (j.tasks || []).length },
      { label: "hosts", render: j => [...new Set((j.tasks || []).map(t => t.hostname))].join(", ") },
      { label: "start", render: j => fmtDateTime(j.startAt) || "-" }, { label: "stop", render: j => fmtDateTime(j.stopAt) || "-" },
      { label: "", render: j => h("span", { class: "row nowrap" }, ["run", "stop"].map(a =>
        h("button", { onclick: e => { e.stopPropagation(); attempt(() => jobAction(a, j.id), `${a}: ok`).then(load); } }, a))) },
    ], jobs, { onRow: j => { location.hash = `jobs/${j.id}`; }, empty: "no jobs yet" }));
  }

  const bulk = name => async () => {
    const ids = [...chosen];
    if (!ids.length) return toast("select jobs first", "warn");
    if (name === "delete" && !(await confirmBox(`Delete ${ids.length} job(s)?`))) return;
    const results = await Promise.all(ids.map(id => jobAction(name, id).then(() => null, e => `#${id}: ${e.message}`)));
    const errs = results.filter(Boolean);
    errs.length ? toast(errs.join("; "), "err", 8000) : toast(`${name}: ${ids.length} job(s)`);
    if (name === "delete") ids.forEach(id => chosen.delete(id));
    load();
  };

  function createDialog() {
    const n = input({ placeholder: "name", maxlength: 40 }), d = input({ placeholder: "description" });
    const sa = h("input", { type: "datetime-local" }), so = h("input", { type: "datetime-local" });
    modal("New job", h("div", {}, field("name", n), field("description", d),
      h("div", { class: "row" }, field("start at (optional)", sa, "the scheduler starts it then"), field("stop at (optional)", so))),
    [["Create", async () => {
      const body = { name: n.value.trim(), description: d.value, userId: S.me };
      if (sa.value) body.startAt = toApi(dtValue(sa));
      if (so.value) body.stopAt = toApi(dtValue(so));
      const r = await attempt(() => call("POST", "/jobs", body), "job created");
      if (!r) return false;
      location.hash = `jobs/${r.job.id}`;
    }, "pri"]]);
  }

  root.replaceChildren(card(null, h("div", { class: "row" },
    h("button", { class: "pri", onclick: createDialog }, "new job"), h("span", { class: "grow" }),
    h("span", { class: "mut" }, "selected:"), ["run", "stop", "kill", "enqueue", "dequeue", "delete"].map(a =>
      h("button", { class: a === "delete" ? "danger" : "", onclick: bulk(a) }, a)),
    S.admin ? userSel : null)), box);
  if (S.admin) call("GET", "/users").then(us => {
    users = us;
    const cur = userSel.value;
    userSel.replaceChildren(...[["mine", "my jobs"], ["all", "all users"], ...us.map(u => [u.id, u.username])].map(([val, l]) => h("option", { value: val }, l)));
    userSel.value = cur;
  }).catch(() => null);
  load();
  v.every(5000, load);
  return v;
}

// ------------------------------------------------------------------------ details
function jobDetailsView(root, id) {
  const v = new View(root);
  const info = h("div", {}), tasksBox = h("div", {}), logBox = h("div", {});
  let job = null, editing = false, openLog = null;

  async function load() {
    const [d, t] = await Promise.all([call("GET", `/jobs/${id}`), call("GET", "/tasks" + qs({ jobId: id, syncAll: false }))])
      .catch(e => { errToast(e); return [null, null]; });
    if (!v.alive || !d) return;
    job = d.job;
    job.tasks = (t && t.tasks) || [];
    if (!editing) renderInfo();
    renderTasks();
  }

  function renderInfo() {
    const n = input({ value: job.name, maxlength: 40 }), d = input({ value: job.description || "" });
    const sa = job.startAt ? dtInput(job.startAt) : h("input", { type: "datetime-local" });
    const so = job.stopAt ? dtInput(job.stopAt) : h("input", { type: "datetime-local" });
    [n, d, sa, so].forEach(x => x.addEventListener("focus", () => { editing = true; }));
    const save = async () => {
      const nv = { name: n.value.trim(), description: d.value, startAt: sa.value ? toApi(dtValue(sa)) : null,
                   stopAt: so.value ? toApi(dtValue(so)) : null };
      const r = await attempt(() => call("PUT", `/jobs/${id}`, nv), "job saved");
      if (r) { editing = false; load(); }
    };
    const act = a => h("button", { class: a === "delete" ? "danger" : a === "run" ? "pri" : "", onclick: async () => {
      if (a === "delete" && !(await confirmBox(`Delete job "${job.name}" and its tasks?`))) return;
      const r = await attempt(() => jobAction(a, id), `${a}: ok`);
      if (r !== undefined && a === "delete") { location.hash = "jobs"; return; }
      load();
    } }, a);
    info.replaceChildren(card(null,
      h("div", { class: "row" }, h("a", { href: "#jobs" }, "< jobs"), h("h3", {}, `#${job.id} ${job.name}`), statusPill(job.status),
        job.isQueued ? pill("queued", "warn") : null, h("span", { class: "grow" }),
        ["run", "stop", "kill", job.isQueued ? "dequeue" : "enqueue", "delete"].map(act)),
      h("div", { class: "row" }, field("name", n), field("description", d), field("start at", sa), field("stop at", so),
        h("button", { onclick: save }, "save"), h("button", { onclick: () => { editing = false; renderInfo(); } }, "revert"))));
  }

  function renderTasks() {
    tasksBox.replaceChildren(card(`Tasks (${(job.tasks || []).length})`,
      table([{ label: "id", key: "id" }, { label: "host", key: "hostname" },
        { label: "GPUs", render: t => (t.allocatedGpus && t.allocatedGpus.length ? t.allocatedGpus.join(",") : (t.gpuId === null || t.gpuId === undefined ? "-" : t.gpuId)) },
        { label: "command", render: t => h("code", { class: "cmd" }, t.fullCommand) },
        { label: "status", render: t => statusPill(t.status) }, { label: "pid", render: t => t.pid || "" },
        { label: "restarts", render: t => `${t.restarts || 0}/${t.maxRestarts || 0}` },
        { label: "", render: t => h("span", { class: "row nowrap" },
          h("button", { onclick: () => showLog(t) }, "log"),
          h("button", { onclick: () => taskDialog(job, t, false, load) }, "edit"),
          h("button", { onclick: () => taskDialog(job, t, true, load) }, "duplicate"),
          h("button", { title: "remove from this job, keep the task", onclick: () => attempt(() => call("DELETE", `/jobs/${id}/tasks/${t.id}`), "task detached").then(load) }, "detach"),
          h("button", { class: "danger", onclick: async () => {
            if (await confirmBox(`Delete task #${t.id}?`)) attempt(() => call("DELETE", `/tasks/${t.id}`), "task deleted").then(load);
          } }, "delete")) }],
      job.tasks || [], { empty: "no tasks: add one below" }),
      h("div", { class: "row" }, h("button", { class: "pri", onclick: () => taskDialog(job, null, false, load) }, "add task"),
        h("button", { onclick: () => launchDialog(job, load) }, "distributed launch"),
        h("button", { onclick: () => adoptDialog(job, load) }, "move a task here"))));
  }

  // log viewer: follows the file every 5 s while open; training curve from [th-train] lines
  function showLog(t) {
    if (openLog) openLog.dispose();
    const lv = new View(logBox), pre = h("pre", { class: "log" }), follow = h("input", { type: "checkbox", checked: true });
    const tail = h("input", { type: "checkbox", checked: true });
    const cv = h("canvas", {}), chart = new LineChart(cv, { unit: " tok/s", min: 0 });
    const stats = h("span", { class: "mut" }), state = h("span", {});
    openLog = lv;
    const poll = async () => {
      const cur = await call("GET", `/tasks/${t.id}`).catch(() => null);
      if (cur && cur.task) state.replaceChildren(statusPill(cur.task.status), cur.task.pid ? ` pid ${cur.task.pid}` : "");
      const d = await call("GET", `/tasks/${t.id}/log` + qs({ tail: tail.checked })).catch(e => ({ output_lines: [`(${e.message})`] }));
      if (!lv.alive) return;
      const atEnd = pre.scrollTop + pre.clientHeight >= pre.scrollHeight - 4;
      pre.textContent = (d.output_lines || []).join("\n");
      if (atEnd) pre.scrollTop = pre.scrollHeight;
      const m = await call("GET", `/tasks/${t.id}/training`).catch(() => null);
      if (m && m.series && m.series.length) {
        chart.set("tokens/s", m.series.map(p => [p.step, p.tokensPerSec]));
        chart.draw();
        const last = m.last || m.series[m.series.length - 1];
        stats.textContent = `step ${last.step} · loss ${fmtNum(last.loss)} · ${fmtNum(last.tokensPerSec)} tokens/s` + (last.world ? ` · world ${last.world}` : "");
      }
    };
    logBox.replaceChildren(card(`Task #${t.id} on ${t.hostname}`,
      h("div", { class: "row" }, h("label", {}, follow, " follow (5 s)"), h("label", {}, tail, " tail only"),
        h("button", { onclick: poll }, "refresh"), state, stats, h("span", { class: "grow" }),
        h("button", { onclick: () => { lv.dispose(); logBox.replaceChildren(); openLog = null; } }, "close")), cv, pre));
    tail.addEventListener("change", poll);
    poll();
    lv.every(5000, () => { if (follow.checked) poll(); });
  }

  const base = v.dispose.bind(v);
  v.dispose = () => { if (openLog) openLog.dispose(); base(); };
  root.replaceChildren(info, tasksBox, logBox);
  load();
  v.every(10000, load);
  return v;
}

// ------------------------------------------------------------------------ task create / edit / duplicate
async function gpuPicker(hostSel, onChange) {
  const box = h("div", { class: "row wrap" });
  let metrics = {};
  const chosen = new Set();
  const auto = h("input", { type: "number", min: 0, max: 64, value: 0, style: { width: "60px" }, title: "0 = pick GPUs below" });
  const draw = () => {
    const gpus = Object.entries(((metrics[hostSel.value] || {}).GPU) || {}).sort((a, b) => a[1].index - b[1].index);
    box.replaceChildren(...gpus.map(([uuid, g]) => {
      const procs = g.processes || [], util = ((g.metrics || {}).utilization || {}).value;
      const c = h("input", { type: "checkbox", checked: chosen.has(g.index), disabled: +auto.value > 0 });
      c.addEventListener("change", () => { c.checked ? chosen.add(g.index) : chosen.delete(g.index); onChange(); });
      return h("label", { class: "gpu-chip" + (procs.length ? " busy" : ""), title: `${uuid}\n${procs.map(p => `${p.owner}:${p.pid}`).join("\n")}` },
        c, ` ${g.index}`, h("small", { class: "mut" }, ` ${util === null || util === undefined ? "-" : util}%${procs.length ? " · " + procs.map(p => p.owner).join(",") : ""}`));
    }), h("span", { class: "mut" }, "or auto:"), auto);
  };
  auto.addEventListener("input", () => { draw(); onChange(); });
  hostSel.addEventListener("change", () => { chosen.clear(); draw(); onChange(); });
  metrics = await call("GET", "/nodes/metrics").catch(() => ({}));
  draw();
  return {
    el: box,
    value: () => +auto.value > 0 ? `auto:${+auto.value}` : [...chosen].sort((a, b) => a - b).join(","),
    set: val => {
      chosen.clear();
      if (typeof val === "string" && val.startsWith("auto:")) auto.value = +val.slice(5);
      else String(val || "").split(",").filter(x => x !== "" && !isNaN(+x)).forEach(x => chosen.add(+x));
      draw();
    },
    list: () => [...chosen].sort((a, b) => a - b), auto: () => +auto.value,
  };
}

async function taskDialog(job, task, duplicate, reload) {
  const hosts = await call("GET", "/nodes/hostnames").catch(() => []);
  const tpl = await templates();
  const hostSel = select(hosts.length ? hosts : [task ? task.hostname : ""], task ? task.hostname : hosts[0]);
  const cmd = input({ value: task ? task.command : "", placeholder: "python train.py", style: { minWidth: "360px" } });
  const segText = segmentsToText(task ? { envs: task.cmdsegments.envs.filter(e => e.name !== "HIP_VISIBLE_DEVICES"), params: task.cmdsegments.params } : { envs: [], params: [] });
  const envs = h("textarea", { rows: 4, cols: 44, placeholder: "NAME=value per line" }); envs.value = segText.envs;
  const params = h("textarea", { rows: 4, cols: 44, placeholder: "--flag value  or  --flag=value per line" }); params.value = segText.params;
  const restarts = input({ type: "number", min: 0, max: 100, value: task ? task.maxRestarts || 0 : 0, style: { width: "70px" } });
  const preview = h("code", { class: "cmd" });
  const tplSel = select([["", "custom"], ...Object.entries(tpl).map(([k, t]) => [k, `${k}: ${t.description || ""}`])], "");
  let picker = null;
  const segments = () => {
    const s = parseSegments(envs.value, params.value);
    const dev = picker ? picker.value() : "";
    if (dev !== "") s.envs.unshift({ name: "HIP_VISIBLE_DEVICES", value: dev });
    return s;
  };
  const update = () => { preview.textContent = renderCommand(cmd.value || "<command>", segments()); };
  picker = await gpuPicker(hostSel, update);
  if (task) {
    const dev = (task.cmdsegments.envs.find(e => e.name === "HIP_VISIBLE_DEVICES") || {}).value;
    picker.set(dev);
  }
  tplSel.addEventListener("change", () => {
    const t = tpl[tplSel.value];
    if (!t) return;
    cmd.value = t.command;
    const txt = segmentsToText({ envs: t.envs.filter(e => e.name !== "HIP_VISIBLE_DEVICES"), params: t.params });
    envs.value = txt.envs; params.value = txt.params; update();
  });
  [cmd, envs, params].forEach(x => x.addEventListener("input", update));
  update();
  const title = task ? (duplicate ? `Duplicate task #${task.id}` : `Edit task #${task.id}`) : `New task in job #${job.id}`;
  modal(title, h("div", {},
    task ? null : field("template", tplSel),
    h("div", { class: "row" }, field("host", hostSel), field("restart on failure (max)", restarts)),
    field("GPUs (HIP_VISIBLE_DEVICES)", picker.el, "busy GPUs are outlined; auto:N lets the allocator pick N free, NUMA-packed GPUs at launch"),
    field("command", cmd), h("div", { class: "row" }, field("environment", envs), field("parameters", params)),
    field("full command", preview)),
  [[task && !duplicate ? "Save" : "Create", async () => {
    if (!cmd.value.trim()) { toast("a command is required", "warn"); return false; }
    const body = { hostname: hostSel.value, command: cmd.value.trim(), cmdsegments: segments(), maxRestarts: +restarts.value || 0 };
    const ok = task && !duplicate
      ? await attempt(() => call("PUT", `/tasks/${task.id}`, body), "task saved")
      : await attempt(() => call("POST", `/jobs/${job.id}/tasks`, body), duplicate ? "task duplicated" : "task created");
    if (!ok) return false;
    reload();
  }, "pri"]]);
}

// Move one of the user's tasks of another job into this one (GET /tasks?jobId=null lists the
// tasks of all the caller's jobs, as the reference's FullCalendarInfo.vue used it)
async function adoptDialog(job, reload) {
  const d = await call("GET", "/tasks" + qs({ jobId: null, syncAll: false })).catch(e => { errToast(e); return null; });
  if (!d) return;
  const tasks = (d.tasks || []).filter(t => t.jobId === null || t.jobId === undefined || t.jobId !== job.id);
  const sel = select(tasks.map(t => [t.id, `#${t.id} ${t.hostname}: ${t.fullCommand.slice(0, 60)}`]));
  modal("Move a task into this job", tasks.length ? field("task", sel) : h("p", { class: "mut" }, "no tasks in other jobs"),
    tasks.length ? [["Add", async () => {
      const ok = await attempt(() => call("PUT", `/jobs/${job.id}/tasks/${sel.value}`), "task added");
      if (!ok) return false;
      reload();
    }, "pri"]] : []);
}

// ------------------------------------------------------------------------ distributed launch
async function launchDialog(job, reload) {
  const hosts = await call("GET", "/nodes/hostnames").catch(() => []);
  const metrics = await call("GET", "/nodes/metrics").catch(() => ({}));
  const kind = select([["torchrun", "torchrun (one task per node, RCCL)"], ["torch", "torch ranks (one task per GPU)"],
    ["tf2", "TensorFlow 2 (TF_CONFIG)"], ["tf1", "TensorFlow 1 (ClusterSpec)"]], "torchrun");
  const cmd = input({ placeholder: "python train.py  (torchrun: python module, default the Llama payload)", style: { minWidth: "380px" } });
  const port = input({ type: "number", value: 29500, style: { width: "90px" } });
  const rows = [];
  const rowsBox = h("div", {}), preview = h("pre", { class: "log small" });
  const gpuCount = host => Object.keys(((metrics[host] || {}).GPU) || {}).length;

  function addRow(host) {
    const r = { host: select(hosts, host || hosts[0]), role: select(["worker", "chief", "ps", "evaluator"], rows.length ? "worker" : "chief"),
                gpus: input({ placeholder: "0,1,2,3", style: { width: "120px" } }), auto: input({ type: "number", min: 0, value: 0, style: { width: "60px" } }) };
    r.gpus.value = Array.from({ length: gpuCount(r.host.value) }, (_, i) => i).join(",");
    [r.host, r.role, r.gpus, r.auto].forEach(x => x.addEventListener("input", refresh));
    r.host.addEventListener("change", () => { r.gpus.value = Array.from({ length: gpuCount(r.host.value) }, (_, i) => i).join(","); refresh(); });
    rows.push(r); drawRows(); refresh();
  }
  function placements() {
    return rows.map(r => {
      const list = r.gpus.value.split(",").map(x => x.trim()).filter(x => x !== "").map(Number);
      const n = +r.auto.value;
      return { hostname: r.host.value, role: r.role.value, gpus: gpuArg(list, kind.value === "torchrun" ? n : 0) };
    });
  }
  function drawRows() {
    rowsBox.replaceChildren(table([{ label: "host", render: r => r.host },
      { label: "role (TF)", render: r => r.role }, { label: "GPU indices", render: r => r.gpus },
      { label: "auto:N (torchrun)", render: r => r.auto },
      { label: "", render: r => h("button", { onclick: () => { rows.splice(rows.indexOf(r), 1); drawRows(); refresh(); } }, "x") }], rows));
  }
  function refresh() {
    const pl = placements(), base = +port.value || (kind.value.startsWith("tf") ? 2222 : 29500);
    if (kind.value === "tf2") preview.textContent = tf2Preview(pl, base).map(x => `${x.hostname}: TF_CONFIG=${x.TF_CONFIG}`).join("\n");
    else if (kind.value === "tf1") preview.textContent = tf1Preview(pl, base).map(x => `${x.hostname}: ${x.flags}`).join("\n");
    else preview.textContent = `world size ${worldSize(pl)}; rendezvous ${pl.length ? pl[0].hostname : "?"}:${base}` +
      (kind.value === "torchrun" ? "; one torchrun per node, --nproc_per_node = its GPU count" : "; one process per GPU with --rank/--world-size");
  }
  kind.addEventListener("change", () => { port.value = kind.value.startsWith("tf") ? 2222 : 29500; refresh(); });
  port.addEventListener("input", refresh);
  addRow(hosts[0]);
  modal(`Distributed launch for job #${job.id}`, h("div", {},
    h("div", { class: "row" }, field("template", kind), field("base port", port)), field("command / module", cmd),
    rowsBox, h("button", { onclick: () => addRow() }, "add node"), h("h4", {}, "Preview"), preview),
  [["Generate tasks", async () => {
    const pl = placements();
    if (!pl.length) { toast("add a node", "warn"); return false; }
    const body = { template: kind.value, placements: pl.map(p => ({ hostname: p.hostname, role: p.role, gpus: p.gpus })), masterPort: +port.value };
    if (cmd.value.trim()) body[kind.value === "torchrun" ? "module" : "command"] = cmd.value.trim();
    const r = await attempt(() => call("POST", `/jobs/${job.id}/tasks/generate`, body));
    if (!r) return false;
    toast(`${r.tasks.length} task(s) created`);
    reload();
  }, "pri"]]);
}

// ------------------------------------------------------------------------ tasks overview
export function tasksView(root) {
  const v = new View(root);
  const box = h("div", {});
  const sync = h("input", { type: "checkbox" });
  async function load() {
    const d = await call("GET", "/tasks" + qs({ syncAll: sync.checked })).catch(e => { errToast(e); return null; });
    if (!v.alive || !d) return;
    box.replaceChildren(table([{ label: "id", key: "id" }, { label: "job", render: t => t.jobId ? h("a", { href: `#jobs/${t.jobId}` }, `#${t.jobId}`) : "-" },
      { label: "host", key: "hostname" }, { label: "status", render: t => statusPill(t.status) }, { label: "pid", render: t => t.pid || "" },
      { label: "command", render: t => h("code", { class: "cmd" }, t.fullCommand) }], d.tasks || [], { empty: "no tasks" }));
  }
  sync.addEventListener("change", load);
  root.replaceChildren(card(null, h("div", { class: "row" }, h("label", {}, sync, " synchronise every task's state with its host"))), box);
  load();
  v.every(10000, load);
  return v;
}
