// DOM helpers shared by the views: element builder, toasts, modal dialogs, form fields, tables.
"use strict";

export const $ = (sel, el = document) => el.querySelector(sel);

export function h(tag, attrs = {}, ...kids) {
  const e = document.createElement(tag);
  for (const [k, v] of Object.entries(attrs || {})) {
    if (k.startsWith("on") && typeof v === "function") e.addEventListener(k.slice(2), v);
    else if (k === "html") e.innerHTML = v;
    else if (k === "style" && typeof v === "object") Object.assign(e.style, v);
    else if (k === "value") e.value = v;
    else if (k === "checked") e.checked = !!v;
    else if (v !== undefined && v !== null && v !== false) e.setAttribute(k, v === true ? "" : v);
  }
  for (const c of kids.flat(Infinity)) {
    if (c === null || c === undefined || c === false) continue;
    e.append(c instanceof Node ? c : document.createTextNode(String(c)));
  }
  return e;
}

export function toast(msg, cls = "ok", ms = 4000) {
  const t = h("div", { class: "toast " + cls }, msg);
  $("#toasts").append(t);
  setTimeout(() => t.remove(), ms);
}

export function errToast(e) { toast(e && e.message ? e.message : String(e), "err", 6000); }

// Run an async action; toast its error.  Returns the action's value (undefined on error).
export async function attempt(fn, okMsg) {
  try {
    const v = await fn();
    if (okMsg) toast(okMsg);
    return v;
  } catch (e) { errToast(e); return undefined; }
}

export function modal(title, body, buttons = [], onClose = null) {
  let closed = false;
  const close = () => { if (closed) return; closed = true; back.remove(); if (onClose) onClose(); };
  const card = h("div", { class: "modal" }, h("h3", {}, title), body,
    h("div", { class: "row end" }, buttons.map(([label, fn, cls]) =>
      h("button", { class: cls || "", onclick: async () => { if ((await fn(close)) !== false) close(); } }, label)),
      h("button", { onclick: close }, "Close")));
  const back = h("div", { class: "backdrop", onclick: e => { if (e.target === back) close(); } }, card);
  document.body.append(back);
  const first = card.querySelector("input,select,textarea");
  if (first) first.focus();
  return close;
}

export function confirmBox(text) {
  return new Promise(resolve => {
    let ok = false;
    modal("Confirm", h("p", {}, text), [["OK", () => { ok = true; }, "pri"]], () => resolve(ok));
  });
}

export function field(label, input, hint) {
  return h("label", { class: "field" }, h("span", {}, label), input, hint ? h("small", { class: "mut" }, hint) : null);
}

export const input = (attrs = {}) => h("input", attrs);
export const select = (options, value, attrs = {}) => {
  const s = h("select", attrs, options.map(o => {
    const [v, l] = Array.isArray(o) ? o : [o, o];
    return h("option", { value: v }, l);
  }));
  if (value !== undefined && value !== null) s.value = value;
  return s;
};

// datetime-local <-> Date
export function dtInput(d) {
  const x = d ? new Date(d) : new Date();
  const pad = n => String(n).padStart(2, "0");
  return h("input", { type: "datetime-local",
    value: `${x.getFullYear()}-${pad(x.getMonth() + 1)}-${pad(x.getDate())}T${pad(x.getHours())}:${pad(x.getMinutes())}` });
}
export const dtValue = inp => inp.value ? new Date(inp.value) : null;

export function table(cols, rows, opts = {}) {
  const head = h("tr", {}, cols.map(c => h("th", {}, c.label)));
  const body = rows.map(r => h("tr", { class: opts.rowClass ? opts.rowClass(r) : "",
    onclick: opts.onRow ? () => opts.onRow(r) : null },
    cols.map(c => h("td", {}, c.render ? c.render(r) : r[c.key]))));
  return h("table", { class: opts.onRow ? "click" : "" }, head, body.length ? body :
    h("tr", {}, h("td", { colspan: cols.length, class: "mut" }, opts.empty || "nothing here")));
}

export function pill(text, cls = "") { return h("span", { class: "pill " + cls }, text); }

export function statusPill(s) {
  const cls = { running: "ok", pending: "warn", terminated: "mut", unsynchronized: "err", not_running: "" }[s] || "";
  return pill(s, cls);
}

export function card(title, ...kids) { return h("section", { class: "card" }, title ? h("h3", {}, title) : null, kids); }

// Re-render helper with a poll timer that stops when the view is replaced
export class View {
  constructor(root) { this.root = root; this.timers = []; this.alive = true; }
  every(ms, fn) { const t = setInterval(() => { if (this.alive) fn(); }, ms); this.timers.push(t); return t; }
  dispose() { this.alive = false; this.timers.forEach(clearInterval); this.timers = []; }
}
