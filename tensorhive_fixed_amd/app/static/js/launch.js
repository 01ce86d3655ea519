// Pure helpers of the task creator (reference job_tasks/TaskCreate.vue:201-215,617-819): command
// rendering, segment-list parsing and the TF_CONFIG / ClusterSpec previews of a distributed launch.
// They mirror the server (models/orm.py Task.render, core/launcher.py tf2_tasks / tf1_tasks) and
// tests/test_webapp_cli.py runs them under node against the Python implementations.
"use strict";

// One shell word per value, as the server renders it (models/orm.py _shell_value): a value the
// shell already reads as one word stays as typed (the user's own quoting, globs, $VARS); values
// that would split, have an unbalanced quote, an unquoted operator, a leading # (comment) or a
// brace expansion ({a,b}, {1..3}), and JSON documents
// (TF_CONFIG), are single-quoted.  isOneShellWord mirrors _is_one_shell_word line for line.
export function isOneShellWord(v) {
  // braces: one entry per open '{' -- whether that level saw an unquoted ',' or '..'
  let words = 0, inWord = false, quote = "", braces = [], i = 0;
  while (i < v.length) {
    const c = v[i];
    if (quote === "'") {
      if (c === "'") quote = "";
    } else if (quote === '"') {
      if (c === "\\") i += 1;
      else if (c === '"') quote = "";
    } else if (" \t\n".includes(c)) {
      inWord = false; braces = [];
    } else if (";&|<>()".includes(c)) {
      return false;
    } else {
      if (!inWord) {
        if (c === "#") return false;
        words += 1; inWord = true;
      }
      if (c === "\\") i += 1;
      else if (c === "'" || c === '"') quote = c;
      else if (c === "{") braces.push(false);
      else if (braces.length && (c === "," || (c === "." && v.slice(i + 1, i + 2) === "."))) braces[braces.length - 1] = true;
      else if (c === "}" && braces.length) {
        if (braces.pop()) return false;
      }
    }
    i += 1;
  }
  return words === 1 && quote === "" && i === v.length;
}

function isJsonDocument(v) {
  const t = v.trimStart();
  if (!(t.startsWith("{") || t.startsWith("["))) return false;
  try { JSON.parse(v); return true; } catch (e) { return false; }
}

export function shellValue(v) {
  v = v === undefined || v === null ? "" : String(v);
  if (v === "" || (isOneShellWord(v) && !isJsonDocument(v))) return v;
  return "'" + v.replace(/'/g, "'\\''") + "'";
}

// ENV=v ... command param value ...; a parameter whose name ends with "=" (or " ") is joined
// without a separator, a parameter with an empty value is the bare name.
export function renderCommand(command, segs) {
  const parts = (segs.envs || []).map(e => `${e.name}=${shellValue(e.value)}`);
  parts.push(command);
  for (const p of segs.params || []) {
    const v = shellValue(p.value);
    if (v === "") parts.push(p.name);
    else if (p.name.endsWith("=") || p.name.endsWith(" ")) parts.push(p.name + v);
    else parts.push(`${p.name} ${v}`);
  }
  return parts.filter(x => x !== "").join(" ");
}

// "NAME=value" per line -> envs; "--name value" / "--name=value" per line -> params
export function parseSegments(envText, paramText) {
  const lines = t => (t || "").split("\n").map(l => l.trim()).filter(Boolean);
  const envs = lines(envText).map(l => {
    const i = l.indexOf("=");
    return i < 0 ? { name: l, value: "" } : { name: l.slice(0, i), value: l.slice(i + 1) };
  });
  const params = lines(paramText).map(l => {
    const eq = l.indexOf("="), sp = l.indexOf(" ");
    if (eq >= 0 && (sp < 0 || eq < sp)) return { name: l.slice(0, eq + 1), value: l.slice(eq + 1) };
    return sp < 0 ? { name: l, value: "" } : { name: l.slice(0, sp), value: l.slice(sp + 1).trim() };
  });
  return { envs, params };
}

export function segmentsToText(segs) {
  return {
    envs: (segs.envs || []).map(e => `${e.name}=${e.value === null || e.value === undefined ? "" : e.value}`).join("\n"),
    params: (segs.params || []).map(p => p.name.endsWith("=") ? p.name + (p.value || "") : `${p.name} ${p.value || ""}`.trim()).join("\n"),
  };
}

// placements [{hostname, role, gpus}] -> TF_CONFIG of every task (core/launcher.py tf2_tasks):
// ports auto-increment per host from basePort, indices count per task type.
export function tf2Preview(placements, basePort = 2222) {
  const next = {}, addrs = [];
  for (const p of placements) {
    const port = next[p.hostname] === undefined ? basePort : next[p.hostname];
    next[p.hostname] = port + 1;
    addrs.push([p.role || "worker", `${p.hostname}:${port}`]);
  }
  const cluster = {};
  for (const [t, a] of addrs) (cluster[t] = cluster[t] || []).push(a);
  const counters = {};
  return placements.map(p => {
    const t = p.role || "worker", idx = counters[t] || 0;
    counters[t] = idx + 1;
    return { hostname: p.hostname, TF_CONFIG: JSON.stringify({ cluster, task: { type: t, index: idx } }) };
  });
}

// ClusterSpec flags (core/launcher.py tf1_tasks): ps first, then workers, ports from basePort
export function tf1Preview(placements, basePort = 2222) {
  const ps = placements.filter(p => p.role === "ps"), workers = placements.filter(p => p.role !== "ps");
  const psHosts = ps.map((p, i) => `${p.hostname}:${basePort + i}`).join(",");
  const workerHosts = workers.map((p, i) => `${p.hostname}:${basePort + ps.length + i}`).join(",");
  return ps.map((p, i) => ({ hostname: p.hostname, flags: `--ps_hosts=${psHosts} --worker_hosts=${workerHosts} --job_name=ps --task_index=${i}` }))
    .concat(workers.map((p, i) => ({ hostname: p.hostname, flags: `--ps_hosts=${psHosts} --worker_hosts=${workerHosts} --job_name=worker --task_index=${i}` })));
}

// World size of a launch (torchrun: GPUs per node summed; "auto:N" counts N)
export function worldSize(placements) {
  return placements.reduce((n, p) => n + (typeof p.gpus === "string" ? +(p.gpus.split(":")[1] || 0) : (p.gpus || []).length || 1), 0);
}

// GPU argument of a placement for the API: [indices] or "auto:N"
export function gpuArg(indices, autoCount) {
  return autoCount ? `auto:${autoCount}` : indices;
}
