// Reservations (reference: views/ReservationsOverview.vue, reserve_resources/FullCalendar.vue,
// FullCalendarReserve.vue, FullCalendarInfo.vue, MySchedule.vue).
//
// A resource-column calendar: one column per (day, GPU), rows of 30 minutes.  Dragging across
// cells selects a time range on a range of GPU columns (reference FullCalendar.vue:151 `select`)
// and opens the reserve dialog, which creates one reservation per GPU.  Cells the user's
// restrictions do not cover are shaded (GET /restrictions?user_id=, the same permission union
// core/verifier.py checks on the server).  Clicking a reservation opens its card
// (FullCalendarInfo.vue:340-357,510-548): edit title / description / time / GPU, cancel, the
// GPU- and memory-utilisation averages the usage logger wrote into it, and the owner's jobs
// that can be attached to run inside it.  "My schedule" lists the user's upcoming reservations.
"use strict";
import { S, call, qs } from "./api.js";
import { fmtNum } from "./chart.js";
import {
  allowedWindow, dragSelection, fmtDateTime, fmtDuration, layoutDay, startOfDay, toApi, usageSummary,
  validReservationRange,
} from "./time.js";
import { View, attempt, card, confirmBox, dtInput, dtValue, errToast, field, h, input, modal, pill, select, table, toast } from "./ui.js";

const SLOT_MIN = 30, SLOTS = 48, ROW_PX = 14;
const OWN = "#e4572e", OTHER = "#3d6bb3", CANCELLED = "#3a3f4b";

function usageBars(r) {
  const b = (label, v) => h("div", { class: "row" }, h("span", { class: "mut", style: { width: "120px" } }, label),
    h("span", { class: "bar wide" }, h("span", { style: { width: (v === null || v === undefined ? 0 : v) + "%" } })),
    v === null || v === undefined ? h("span", { class: "mut" }, "no samples yet") : `${v}%`);
  return [b("avg GPU util", r.gpuUtilAvg), b("avg HBM util", r.memUtilAvg)];
}

export function reservationsView(root) {
  const v = new View(root);
  let resources = [], users = {}, restrictions = [], reservations = [], selected = [];
  let origin = startOfDay(new Date()), days = +(localStorage.getItem("th.cal.days") || 3);
  const grid = h("div", { class: "cal-wrap" }), side = h("div", {}), gpuPicker = h("div", { class: "gpu-picker" });
  const daySel = select([[1, "1 day"], [2, "2 days"], [3, "3 days"], [5, "5 days"], [7, "week"]], days);
  const title = h("span", { class: "mut" });

  const dayStarts = () => Array.from({ length: days }, (_, i) => new Date(origin.getTime() + i * 864e5));
  const uname = id => (users[id] || {}).username || `user ${id}`;
  const canEdit = r => S.admin || r.userId === S.me;

  async function loadStatic() {
    const [res, us, rs] = await Promise.all([
      call("GET", "/resources"),
      call("GET", "/users").catch(() => []),
      call("GET", "/restrictions" + qs({ user_id: S.me, include_user_groups: true })).catch(() => []),
    ]);
    resources = res.slice().sort((a, b) => (a.hostname || "").localeCompare(b.hostname || "") || String(a.name).localeCompare(String(b.name)));
    users = Object.fromEntries(us.map(u => [u.id, u]));
    restrictions = rs;
    const saved = JSON.parse(localStorage.getItem("th.cal.gpus") || "null");
    selected = (saved || resources.map(r => r.id)).filter(id => resources.some(r => r.id === id));
    if (!selected.length) selected = resources.map(r => r.id);
    renderPicker();
  }

  function renderPicker() {
    const byHost = {};
    resources.forEach(r => (byHost[r.hostname || "?"] = byHost[r.hostname || "?"] || []).push(r));
    gpuPicker.replaceChildren(...Object.entries(byHost).map(([host, rs]) => {
      const all = h("input", { type: "checkbox", checked: rs.every(r => selected.includes(r.id)) });
      all.addEventListener("change", () => { toggle(rs.map(r => r.id), all.checked); });
      return h("div", { class: "row" }, h("label", {}, all, " ", h("b", {}, host)), rs.map(r => {
        const c = h("input", { type: "checkbox", checked: selected.includes(r.id) });
        c.addEventListener("change", () => toggle([r.id], c.checked));
        const ok = allowedWindow(restrictions, r.id, new Date(), new Date(Date.now() + 36e5), 30);
        return h("label", { title: r.id, class: ok ? "" : "mut" }, c, ` ${r.name || r.id.slice(4, 12)}`);
      }));
    }));
  }

  function toggle(ids, on) {
    selected = on ? [...new Set([...selected, ...ids])] : selected.filter(x => !ids.includes(x));
    selected = resources.map(r => r.id).filter(id => selected.includes(id));
    localStorage.setItem("th.cal.gpus", JSON.stringify(selected));
    renderPicker(); load();
  }

  async function load() {
    const ds = dayStarts(), end = new Date(ds[ds.length - 1].getTime() + 864e5);
    title.textContent = `${ds[0].toDateString()} - ${new Date(end - 1).toDateString()}`;
    if (!selected.length) { reservations = []; draw(); return; }
    const rs = await call("GET", "/reservations" + qs({ resources_ids: selected, start: toApi(ds[0]), end: toApi(end) })).catch(e => { errToast(e); return null; });
    if (!v.alive || rs === null) return;
    reservations = rs;
    draw();
    renderMine();
  }

  // ---------------------------------------------------------------- grid + drag select
  function draw() {
    const ds = dayStarts(), cols = [];
    ds.forEach((d, di) => selected.forEach((id, gi) => cols.push({ day: di, gpu: gi, id, d })));
    const res = Object.fromEntries(resources.map(r => [r.id, r]));
    const head1 = h("tr", {}, h("th", { class: "cal-time" }, ""), ds.map(d =>
      h("th", { colspan: selected.length, class: "cal-day" }, d.toLocaleDateString(undefined, { weekday: "short", month: "short", day: "numeric" }))));
    const head2 = h("tr", {}, h("th", { class: "cal-time" }, ""), cols.map(c =>
      h("th", { class: "cal-gpu", title: `${res[c.id].hostname} ${c.id}` }, `${(res[c.id].hostname || "").slice(0, 6)}:${res[c.id].name || ""}`)));
    let anchor = null, hoverCell = null;
    const cells = [];
    const mark = () => {
      cells.forEach(x => x.el.classList.remove("sel"));
      if (!anchor || !hoverCell) return;
      const s = dragSelection(anchor, hoverCell, ds, selected, SLOT_MIN);
      cells.forEach(x => {
        const t = ds[x.day].getTime() + x.slot * SLOT_MIN * 60000;
        if (t >= s.start.getTime() && t < s.end.getTime() && s.gpus.includes(selected[x.gpu])) x.el.classList.add("sel");
      });
    };
    const rows = [];
    const now = Date.now();
    for (let s = 0; s < SLOTS; s++) {
      const tr = h("tr", {}, h("td", { class: "cal-time" }, s % 2 ? "" : `${String(s / 2).padStart(2, "0")}:00`));
      for (const c of cols) {
        const t0 = c.d.getTime() + s * SLOT_MIN * 60000;
        const ok = allowedWindow(restrictions, c.id, new Date(t0), new Date(t0 + SLOT_MIN * 60000), SLOT_MIN);
        const td = h("td", { class: "cal-cell" + (ok ? "" : " denied") + (t0 + SLOT_MIN * 60000 < now ? " past" : "") });
        const cell = { day: c.day, gpu: c.gpu, slot: s, el: td };
        cells.push(cell);
        td.addEventListener("mousedown", e => { if (e.button === 0) { anchor = hoverCell = cell; mark(); e.preventDefault(); } });
        td.addEventListener("mouseenter", () => { if (anchor) { hoverCell = cell; mark(); } });
        tr.append(td);
      }
      rows.push(tr);
    }
    const tbl = h("table", { class: "cal" }, head1, head2, rows);
    tbl.addEventListener("mouseup", () => {
      if (!anchor) return;
      const s = dragSelection(anchor, hoverCell || anchor, ds, selected, SLOT_MIN);
      anchor = hoverCell = null; mark();
      reserveDialog(s.start, s.end, s.gpus);
    });
    tbl.addEventListener("mouseleave", () => { if (anchor) { anchor = hoverCell = null; mark(); } });
    // reservation blocks: absolutely positioned over the first row of their column
    const layer = h("div", { class: "cal-layer" });
    grid.replaceChildren(h("div", { class: "cal-scroll" }, tbl, layer));
    requestAnimationFrame(() => {
      const firstRow = rows[0];
      if (!firstRow) return;
      const top0 = firstRow.offsetTop, dayPx = ROW_PX * SLOTS;
      cols.forEach((c, ci) => {
        const td = firstRow.children[ci + 1];
        const mine = reservations.filter(r => r.resourceId === c.id);
        for (const x of layoutDay(mine, c.d)) {
          const r = x.r;
          layer.append(h("div", {
            class: "cal-block" + (r.isCancelled ? " cancelled" : ""),
            title: `${r.title} - ${uname(r.userId)}\n${fmtDateTime(r.start)} - ${fmtDateTime(r.end)}`,
            style: { left: td.offsetLeft + 1 + "px", width: td.offsetWidth - 2 + "px", top: top0 + x.top * dayPx + "px",
                     height: Math.max(6, x.height * dayPx - 1) + "px",
                     background: r.isCancelled ? CANCELLED : r.userId === S.me ? OWN : OTHER },
            onclick: () => infoDialog(r),
          }, r.title));
        }
      });
      const nowLine = now - ds[0].getTime();
      if (nowLine > 0 && nowLine < days * 864e5) {
        const di = Math.floor(nowLine / 864e5), frac = (nowLine % 864e5) / 864e5;
        const a = firstRow.children[1 + di * selected.length], b = firstRow.children[(di + 1) * selected.length];
        if (a && b) layer.append(h("div", { class: "cal-now", style: { left: a.offsetLeft + "px",
          width: b.offsetLeft + b.offsetWidth - a.offsetLeft + "px", top: top0 + frac * dayPx + "px" } }));
      }
    });
  }

  // ---------------------------------------------------------------- dialogs
  function reserveDialog(start, end, gpus) {
    const t = input({ placeholder: "title", maxlength: 60 }), d = input({ placeholder: "description", maxlength: 200 });
    const s = dtInput(start), e = dtInput(end);
    const res = Object.fromEntries(resources.map(r => [r.id, r]));
    const boxes = gpus.map(id => ({ id, el: h("input", { type: "checkbox", checked: true }) }));
    const who = S.admin ? select(Object.values(users).map(u => [u.id, u.username]), S.me) : null;
    const warn = h("div", { class: "warn" });
    const check = () => {
      const a = dtValue(s), b = dtValue(e), bad = validReservationRange(a, b);
      const denied = boxes.filter(x => x.el.checked && !allowedWindow(restrictions, x.id, a, b));
      warn.textContent = bad || (denied.length && !S.admin ? `your restrictions do not cover ${denied.length} of the GPUs in this window` : "");
    };
    [s, e].forEach(x => x.addEventListener("change", check));
    check();
    modal("Reserve GPUs", h("div", {},
      field("title", t), field("description", d),
      h("div", { class: "row" }, field("start", s), field("end", e)),
      who ? field("on behalf of", who) : null,
      h("div", { class: "row wrap" }, boxes.map(x => h("label", {}, x.el, ` ${res[x.id].hostname}:${res[x.id].name || x.id.slice(4, 12)}`))),
      warn),
    [["Reserve", async () => {
      const a = dtValue(s), b = dtValue(e), bad = validReservationRange(a, b);
      if (bad) { toast(bad, "warn"); return false; }
      if (!t.value.trim()) { toast("a title is required", "warn"); return false; }
      let ok = 0;
      for (const x of boxes.filter(x => x.el.checked)) {
        try {
          await call("POST", "/reservations", { title: t.value.trim(), description: d.value, resourceId: x.id,
            userId: who ? +who.value : S.me, start: toApi(a), end: toApi(b) });
          ok++;
        } catch (err) { toast(`${res[x.id].hostname}:${res[x.id].name}: ${err.message}`, "err", 6000); }
      }
      if (ok) toast(`${ok} reservation(s) created`);
      load();
    }, "pri"]]);
  }

  async function infoDialog(r) {
    const res = Object.fromEntries(resources.map(x => [x.id, x]));
    const g = res[r.resourceId] || {};
    const editable = canEdit(r) && new Date(r.end) > new Date();
    const started = new Date(r.start) <= new Date();
    const t = input({ value: r.title, maxlength: 60, disabled: !editable }), d = input({ value: r.description || "", maxlength: 200, disabled: !editable });
    const s = dtInput(r.start), e = dtInput(r.end);
    if (!editable || (started && !S.admin)) s.disabled = true;
    if (!editable) e.disabled = true;
    const gpuSel = select(resources.map(x => [x.id, `${x.hostname}:${x.name || x.id.slice(4, 12)}`]), r.resourceId, { disabled: !editable });
    const jobsBox = h("div", {});
    const body = h("div", {},
      h("div", { class: "row" }, pill(r.isCancelled ? "cancelled" : started ? (new Date(r.end) < new Date() ? "finished" : "in progress") : "upcoming",
        r.isCancelled ? "mut" : started ? "ok" : "warn"), h("span", { class: "mut" }, `by ${r.userName || uname(r.userId)} · ${g.hostname || ""} · ${fmtDuration(new Date(r.end) - new Date(r.start))}`)),
      field("title", t), field("description", d), h("div", { class: "row" }, field("start", s), field("end", e)), field("GPU", gpuSel),
      h("h4", {}, "Usage during the reservation"), usageBars(r), jobsBox);
    if (r.userId === S.me && !r.isCancelled && new Date(r.end) > new Date()) attachJobs(r, jobsBox);
    const buttons = [];
    if (editable) buttons.push(["Save", async () => {
      const nv = {};
      if (t.value !== r.title) nv.title = t.value;
      if (d.value !== (r.description || "")) nv.description = d.value;
      if (gpuSel.value !== r.resourceId) nv.resourceId = gpuSel.value;
      if (!s.disabled && dtValue(s).getTime() !== new Date(r.start).getTime()) nv.start = toApi(dtValue(s));
      if (dtValue(e).getTime() !== new Date(r.end).getTime()) nv.end = toApi(dtValue(e));
      if (!Object.keys(nv).length) return;
      const bad = validReservationRange(nv.start || r.start, nv.end || r.end);
      if (bad) { toast(bad, "warn"); return false; }
      const ok = await attempt(() => call("PUT", `/reservations/${r.id}`, nv), "reservation updated");
      if (ok === undefined) return false;
      load();
    }, "pri"]);
    if (canEdit(r) && (!started || S.admin)) buttons.push(["Cancel reservation", async () => {
      if (!(await confirmBox(`Cancel "${r.title}"?`))) return false;
      const ok = await attempt(() => call("DELETE", `/reservations/${r.id}`), "reservation cancelled");
      if (ok === undefined) return false;
      load();
    }, "danger"]);
    modal(`Reservation #${r.id}`, body, buttons);
  }

  async function attachJobs(r, box) {
    const d = await call("GET", "/jobs" + qs({ userId: S.me })).catch(() => ({ jobs: [] }));
    const free = await call("GET", "/tasks" + qs({ jobId: null, syncAll: false })).catch(() => ({ tasks: [] }));
    const jobs = (d.jobs || []).filter(j => j.status !== "running");
    const count = {};
    (free.tasks || []).forEach(t => { count[t.jobId] = (count[t.jobId] || 0) + 1; });
    const sel = select(jobs.map(j => [j.id, `#${j.id} ${j.name} (${count[j.id] || 0} task(s))`]));
    const sib = h("input", { type: "checkbox", checked: true });
    box.replaceChildren(h("h4", {}, "Run a job inside this reservation"),
      jobs.length ? h("div", { class: "row" }, sel, h("label", { title: "also use my other reservations of the same window on this node" }, sib, " + sibling GPUs"),
        h("button", { onclick: () => attempt(async () => {
          await call("PUT", `/jobs/${sel.value}/reservation/${r.id}` + qs({ siblings: sib.checked }));
        }, "job attached: its tasks run on the reserved GPUs at the reservation start") }, "attach"))
        : h("p", { class: "mut" }, "no stopped jobs to attach"),
      h("p", { class: "mut" }, "the job's tasks get the reserved GPUs as HIP_VISIBLE_DEVICES and start / stop at the reservation window"));
  }

  // ---------------------------------------------------------------- my schedule
  const mineBox = h("div", {});
  async function renderMine() {
    const all = resources.map(x => x.id);
    if (!all.length) return;
    const from = new Date(), to = new Date(Date.now() + 14 * 864e5);
    const rs = await call("GET", "/reservations" + qs({ resources_ids: all, start: toApi(from), end: toApi(to) })).catch(() => []);
    const mine = rs.filter(r => r.userId === S.me && !r.isCancelled).sort((a, b) => new Date(a.start) - new Date(b.start));
    const past = reservations.filter(r => r.userId === S.me && new Date(r.end) < new Date());
    const u = usageSummary(past);
    const res = Object.fromEntries(resources.map(x => [x.id, x]));
    mineBox.replaceChildren(card("My schedule (next 14 days)",
      table([{ label: "when", render: r => `${fmtDateTime(r.start)} - ${fmtDateTime(r.end)}` },
        { label: "GPU", render: r => `${(res[r.resourceId] || {}).hostname}:${(res[r.resourceId] || {}).name || ""}` },
        { label: "title", key: "title" },
        { label: "", render: r => new Date(r.start) <= new Date() ? pill("now", "ok") : pill("in " + fmtDuration(new Date(r.start) - new Date()), "mut") }],
      mine, { onRow: infoDialog, empty: "no upcoming reservations" }),
      u.samples ? h("p", { class: "mut" }, `finished reservations in view: avg GPU util ${fmtNum(u.gpuUtilAvg)}%, HBM ${fmtNum(u.memUtilAvg)}%`) : null));
  }

  // ---------------------------------------------------------------- toolbar
  const shift = n => { origin = new Date(origin.getTime() + n * 864e5); load(); };
  daySel.addEventListener("change", () => { days = +daySel.value; localStorage.setItem("th.cal.days", days); load(); });
  const toolbar = h("div", { class: "row" },
    h("button", { onclick: () => shift(-days) }, "<"), h("button", { onclick: () => { origin = startOfDay(new Date()); load(); } }, "today"),
    h("button", { onclick: () => shift(days) }, ">"), daySel, title, h("span", { class: "grow" }),
    h("span", { class: "legend" }, h("i", { style: { background: OWN } }), "mine ", h("i", { style: { background: OTHER } }), "others ",
      h("i", { class: "denied" }), "not allowed by your restrictions"),
    h("button", { class: "pri", onclick: () => reserveDialog(new Date(Math.ceil(Date.now() / 18e5) * 18e5),
      new Date(Math.ceil(Date.now() / 18e5) * 18e5 + 36e5), selected) }, "new reservation"));

  root.replaceChildren(card(null, toolbar, gpuPicker), card(null, h("p", { class: "mut" },
    "Drag over the grid to reserve: the selection spans every GPU column between the first and last cell."), grid), mineBox, side);
  loadStatic().then(load).catch(errToast);
  v.every(30000, load);
  return v;
}
