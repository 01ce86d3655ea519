// Nodes overview (reference: views/NodesOverview.vue, nodes_overview/WatchGenerator.vue, WatchBox.vue).
// A sub-second poll of GET /nodes/metrics (the daemon samples every 0.25 s; the reference polled
// every 5 s) drives host cards with every MI355X metric, per-host sample age, GPU processes with
// their owners and tasks, and user-defined "watch" charts (host x resource x metric) that follow
// the per-host metric endpoints, as the reference's watch boxes did.
"use strict";
import { S, call, qs } from "./api.js";
import { LineChart, fmtNum } from "./chart.js";
import { View, attempt, card, field, h, modal, pill, select, table } from "./ui.js";

export const GPU_METRICS = {
  utilization: ["GPU util", "%", 100], mem_util: ["HBM activity", "%", 100], mfma_busy: ["MFMA busy (counters)", "%", 100],
  mfma_contention: ["MFMA contention (probe)", "%", 100], gpu_busy: ["GPU busy (counters)", "%", 100],
  mfma_tflops: ["MFMA TFLOP/s (counters)", " TF", null],
  hbm_bw: ["HBM bandwidth", " GB/s", null], hbm_contention: ["HBM contention (probe)", "%", 100],
  power: ["power", " W", null], energy: ["power (accumulator)", " W", null], temp: ["edge temp", " C", null],
  hotspot_temp: ["hotspot temp", " C", null], mem_temp: ["HBM temp", " C", null], mem_used: ["VRAM used", " MiB", null],
  mem_free: ["VRAM free", " MiB", null], mem_total: ["VRAM total", " MiB", null], gfx_clock: ["gfx clock", " MHz", null],
  mem_clock: ["mem clock", " MHz", null], xgmi_read: ["xGMI read", " GB/s", null], xgmi_write: ["xGMI write", " GB/s", null],
  fan_speed: ["fan", "%", 100],
};
export const CPU_METRICS = { utilization: ["CPU util", "%", 100], mem_used: ["RAM used", " MiB", null],
  mem_free: ["RAM free", " MiB", null], mem_total: ["RAM total", " MiB", null] };

const mv = (m, k) => (m && m[k] && m[k].value !== null && m[k].value !== undefined) ? m[k].value : null;
const WATCH_KEY = "th.watches";

function loadWatches() { try { return JSON.parse(localStorage.getItem(WATCH_KEY)) || []; } catch (e) { return []; } }
function saveWatches(w) { localStorage.setItem(WATCH_KEY, JSON.stringify(w)); }

function bar(v, max) {
  const pct = v === null ? 0 : Math.max(0, Math.min(100, v / (max || 100) * 100));
  return h("span", { class: "bar" }, h("span", { style: { width: pct + "%" } }));
}

function gpuRow(uuid, g) {
  const m = g.metrics || {};
  const procs = g.processes || [];
  return h("tr", {},
    h("td", {}, g.index), h("td", { title: uuid }, (g.name || "GPU").replace("AMD Instinct ", "")),
    h("td", {}, bar(mv(m, "utilization")), " ", fmtNum(mv(m, "utilization")), "%"),
    h("td", {}, fmtNum(mv(m, "mem_used")), " / ", fmtNum(mv(m, "mem_total")), " MiB"),
    h("td", { title: "source: " + (mv(m, "hbm_bw_source") || "umc_activity") },
      fmtNum(mv(m, "hbm_bw")), " GB/s", mv(m, "hbm_bw_source") === "partial" ? " (partial)" : ""),
    // MFMA: the counter value where th-counters runs, else the probe's contention estimate (~)
    mv(m, "mfma_busy") !== null ? h("td", { title: "SQ_VALU_MFMA_BUSY_CYCLES" }, fmtNum(mv(m, "mfma_busy")) + "%")
      : h("td", { title: "probe contention, not busy cycles" },
        mv(m, "mfma_contention") === null ? "-" : "~" + fmtNum(mv(m, "mfma_contention")) + "%"),
    h("td", {}, fmtNum(mv(m, "power")), " W"),
    h("td", {}, fmtNum(mv(m, "temp")), " / ", fmtNum(mv(m, "hotspot_temp")), " C"),
    h("td", {}, fmtNum(mv(m, "xgmi_read")), " / ", fmtNum(mv(m, "xgmi_write"))),
    h("td", {}, procs.length ? procs.map(p => pill(`${p.owner || "?"}:${p.pid}${p.task_id ? " task " + p.task_id : ""}`,
      p.owner === S.username ? "ok" : "warn")) : h("span", { class: "mut" }, "idle")));
}

function hostCard(host, entry, onProcs) {
  const age = S.hostAge[host];
  const stale = age !== undefined && age > 5000;
  const gpus = Object.entries((entry && entry.GPU) || {}).sort((a, b) => a[1].index - b[1].index);
  const cpu = entry && entry.CPU ? Object.values(entry.CPU)[0] : null;
  return card(null,
    h("div", { class: "row" }, h("b", {}, host),
      age !== undefined ? pill(stale ? `STALE ${(age / 1000).toFixed(0)} s` : `${age} ms old`, stale ? "err" : "mut") : null,
      cpu ? h("span", { class: "mut" }, `CPU ${fmtNum(mv(cpu.metrics, "utilization"))}% · RAM ${fmtNum(mv(cpu.metrics, "mem_used"))}` +
        ` / ${fmtNum(mv(cpu.metrics, "mem_total"))} MiB`) : null,
      h("span", { class: "grow" }), h("button", { onclick: () => onProcs(host) }, "processes")),
    h("table", {}, h("tr", {}, ["#", "GPU", "util", "VRAM", "HBM", "MFMA", "power", "temp edge/hot",
      "xGMI r/w GB/s", "processes"].map(t => h("th", {}, t))), gpus.map(([u, g]) => gpuRow(u, g))));
}

class WatchBox {
  // one chart: a metric of every GPU (or the CPU) of one host, fed from /nodes/{host}/{gpu|cpu}/metrics
  constructor(w, onRemove) {
    this.w = w;
    const meta = (w.resource === "cpu" ? CPU_METRICS : GPU_METRICS)[w.metric] || [w.metric, "", null];
    this.canvas = h("canvas", {});
    this.chart = new LineChart(this.canvas, { unit: meta[1], max: meta[2], min: 0 });
    this.el = card(null, h("div", { class: "row" }, h("b", {}, `${w.host} · ${w.resource.toUpperCase()} · ${meta[0]}`),
      h("span", { class: "grow" }), h("button", { onclick: onRemove }, "remove")), this.canvas);
    this.names = {};
  }
  async poll() {
    const d = await call("GET", `/nodes/${encodeURIComponent(this.w.host)}/${this.w.resource}/metrics` + qs({ metric_type: this.w.metric }));
    const now = Date.now();
    for (const [id, m] of Object.entries(d)) {
      const name = this.names[id] || (this.names[id] = id.startsWith("CPU") ? "CPU" : "GPU " + Object.keys(this.names).length);
      this.chart.push(name, now, m && m.value !== undefined ? m.value : null);
    }
    this.chart.draw();
  }
}

export function nodesView(root) {
  const v = new View(root);
  const hostsBox = h("div", {});
  const watchBox = h("div", { class: "grid2" });
  let infra = {}, period = +(localStorage.getItem("th.poll") || 500), timer = null;
  let watches = loadWatches().map(w => new WatchBox(w, () => removeWatch(w)));

  function removeWatch(w) {
    watches = watches.filter(x => x.w !== w);
    saveWatches(watches.map(x => x.w));
    renderWatches();
  }
  function renderWatches() { watchBox.replaceChildren(...watches.map(x => x.el)); }

  async function showProcs(host) {
    const d = await attempt(() => call("GET", `/nodes/${encodeURIComponent(host)}/gpu/processes`));
    if (!d) return;
    const rows = Object.entries(d).flatMap(([uuid, ps]) => (ps || []).map(p => ({ uuid, ...p })));
    modal(`GPU processes on ${host}`, table([{ label: "GPU", render: r => (infra[host].GPU[r.uuid] || {}).index },
      { label: "pid", key: "pid" }, { label: "owner", key: "owner" }, { label: "task", render: r => r.task_id || "" },
      { label: "VRAM MiB", render: r => fmtNum((r.vram || 0) / 1048576) }, { label: "command", key: "command" }], rows));
  }

  async function tick() {
    const d = await call("GET", "/nodes/metrics").catch(() => null);
    if (!v.alive) return;
    if (d) {
      infra = d;
      hostsBox.replaceChildren(...Object.keys(d).sort().map(host => hostCard(host, d[host], showProcs)));
    }
    await Promise.all(watches.map(x => x.poll().catch(() => null)));
  }
  function restart() {
    if (timer) clearInterval(timer);
    timer = v.every(period, tick);
  }

  const hostSel = select([], null), resSel = select([["gpu", "GPU"], ["cpu", "CPU"]], "gpu");
  const metricSel = select(Object.entries(GPU_METRICS).map(([k, m]) => [k, m[0]]), "utilization");
  resSel.addEventListener("change", () => {
    const src = resSel.value === "cpu" ? CPU_METRICS : GPU_METRICS;
    metricSel.replaceChildren(...Object.entries(src).map(([k, m]) => h("option", { value: k }, m[0])));
  });
  const periodSel = select([[250, "0.25 s"], [500, "0.5 s"], [1000, "1 s"], [2000, "2 s"], [5000, "5 s"]], period);
  periodSel.addEventListener("change", () => { period = +periodSel.value; localStorage.setItem("th.poll", period); restart(); });
  call("GET", "/nodes/hostnames").then(hs => hostSel.replaceChildren(...hs.map(x => h("option", { value: x }, x)))).catch(() => null);

  const gen = card("Watch a metric",
    h("div", { class: "row" }, field("node", hostSel), field("resource", resSel), field("metric", metricSel),
      h("button", { class: "pri", onclick: () => {
        if (!hostSel.value) return;
        const w = { host: hostSel.value, resource: resSel.value, metric: metricSel.value };
        watches.push(new WatchBox(w, () => removeWatch(w)));
        saveWatches(watches.map(x => x.w)); renderWatches();
      } }, "add chart"),
      h("span", { class: "grow" }), field("refresh", periodSel),
      h("button", { onclick: () => showTopology() }, "topology")));

  async function showTopology() {
    const t = await attempt(() => call("GET", "/nodes/topology"));
    if (!t) return;
    modal("GPU topology (NUMA / xGMI)", h("pre", {}, JSON.stringify(t, null, 1)));
  }

  root.replaceChildren(gen, watchBox, hostsBox);
  renderWatches();
  tick();
  restart();
  return v;
}
