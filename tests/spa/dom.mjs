// Minimal DOM + browser globals for running the dashboard modules under node (no jsdom here):
// enough of Element / Text / document / localStorage / fetch (over node's http) / timers for the
// views to render, for tests to find elements and fire events, and for every API request to reach
// the real server.  Timers from setInterval are recorded, never repeated (tests call tick()).
import http from "http";

export class Node {
  constructor() { this.parentNode = null; this.childNodes = []; }
  get children() { return this.childNodes.filter(c => c instanceof Element); }
  append(...kids) {
    for (const k of kids) {
      const n = k instanceof Node ? k : new Text(String(k));
      if (n.parentNode) n.parentNode._detach(n);
      n.parentNode = this;
      this.childNodes.push(n);
    }
  }
  appendChild(n) { this.append(n); return n; }
  replaceChildren(...kids) { for (const c of this.childNodes) c.parentNode = null; this.childNodes = []; this.append(...kids); }
  _detach(n) { this.childNodes = this.childNodes.filter(c => c !== n); n.parentNode = null; }
  remove() { if (this.parentNode) this.parentNode._detach(this); }
  get textContent() { return this.childNodes.map(c => c.textContent).join(""); }
  set textContent(v) { this.replaceChildren(new Text(String(v))); }
}

export class Text extends Node {
  constructor(t) { super(); this.data = t; }
  get textContent() { return this.data; }
  set textContent(v) { this.data = String(v); }
}

class ClassList {
  constructor(el) { this.el = el; }
  _get() { return (this.el.getAttribute("class") || "").split(/\s+/).filter(Boolean); }
  add(...c) { this.el.setAttribute("class", [...new Set([...this._get(), ...c])].join(" ")); }
  remove(...c) { this.el.setAttribute("class", this._get().filter(x => !c.includes(x)).join(" ")); }
  contains(c) { return this._get().includes(c); }
}

const CTX = new Proxy({}, { get: (_t, k) => k === "measureText" ? () => ({ width: 10 }) : () => {} });

export class Element extends Node {
  constructor(tag) {
    super();
    this.tagName = tag.toUpperCase();
    this.attributes = {};
    this.style = {};
    this.listeners = {};
    this.classList = new ClassList(this);
    this.disabled = false;
    this.checked = false;
    this.offsetTop = 0; this.offsetLeft = 0; this.offsetWidth = 50; this.clientWidth = 300; this.clientHeight = 100;
    this.scrollTop = 0; this.scrollHeight = 0;
    this.width = 300; this.height = 150;
  }
  setAttribute(k, v) {
    this.attributes[k] = String(v);
    if (k === "disabled") this.disabled = true;
    if (k === "checked") this.checked = true;
  }
  getAttribute(k) { return k in this.attributes ? this.attributes[k] : null; }
  get id() { return this.getAttribute("id"); }
  get className() { return this.getAttribute("class") || ""; }
  set innerHTML(v) { this.replaceChildren(new Text(String(v))); }
  get options() { return this.querySelectorAll("option"); }
  get selectedOptions() { return this.options.filter(o => o.selected); }
  get value() {
    if (this._value !== undefined) return this._value;
    if (this.tagName === "SELECT") { const o = this.options[0]; return o ? o.value : ""; }
    if (this.tagName === "OPTION") return this.getAttribute("value") !== null ? this.getAttribute("value") : this.textContent;
    return this.getAttribute("value") || "";
  }
  set value(v) { this._value = String(v); }
  addEventListener(t, fn) { (this.listeners[t] = this.listeners[t] || []).push(fn); }
  removeEventListener(t, fn) { this.listeners[t] = (this.listeners[t] || []).filter(f => f !== fn); }
  dispatch(type, props = {}) {
    const ev = { type, target: this, button: 0, key: "", offsetX: 0, preventDefault() {}, stopPropagation() { this._stop = true; }, ...props };
    let n = this;
    const results = [];
    while (n && !ev._stop) {
      for (const fn of (n.listeners && n.listeners[type]) || []) results.push(fn(ev));
      n = n.parentNode;
    }
    return Promise.all(results.map(r => Promise.resolve(r).catch(e => { globalThis.__errors.push(e); })));
  }
  click() { return this.dispatch("click"); }
  focus() {}
  getContext() { return CTX; }
  matches(sel) {
    return sel.split(",").some(one => {
      const m = one.trim().match(/^([a-zA-Z0-9]*)((?:[.#][\w-]+)*)$/);
      if (!m) return false;
      if (m[1] && this.tagName !== m[1].toUpperCase()) return false;
      for (const part of m[2].match(/[.#][\w-]+/g) || []) {
        if (part[0] === "." && !this.classList.contains(part.slice(1))) return false;
        if (part[0] === "#" && this.id !== part.slice(1)) return false;
      }
      return true;
    });
  }
  querySelectorAll(sel) {
    const out = [];
    const walk = n => { for (const c of n.children) { if (c.matches(sel)) out.push(c); walk(c); } };
    walk(this);
    return out;
  }
  querySelector(sel) { return this.querySelectorAll(sel)[0] || null; }
}

class Storage {
  constructor() { this.m = new Map(); }
  getItem(k) { return this.m.has(k) ? this.m.get(k) : null; }
  setItem(k, v) { this.m.set(k, String(v)); }
  removeItem(k) { this.m.delete(k); }
  clear() { this.m.clear(); }
}

export function install(baseUrl) {
  const document = {
    createElement: t => new Element(t),
    createTextNode: t => new Text(t),
    body: new Element("body"),
    querySelector(sel) { return this.body.querySelector(sel); },
  };
  for (const [tag, id] of [["div", "nav"], ["div", "who"], ["main", "main"], ["div", "toasts"], ["span", "ver"]]) {
    const e = new Element(tag);
    e.setAttribute("id", id);
    document.body.append(e);
  }
  const timers = [];
  Object.assign(globalThis, {
    Node, Element, Text, document,
    window: globalThis, devicePixelRatio: 1,
    localStorage: new Storage(),
    location: {  // like a browser: the hash reads back with its "#"
      _h: "", get hash() { return this._h; }, set hash(v) { v = String(v); this._h = v && v[0] !== "#" ? "#" + v : v; },
    },
    requestAnimationFrame: fn => setTimeout(fn, 0),
    __errors: [], __requests: [], __timers: timers,
    atob: b64 => Buffer.from(b64, "base64").toString("binary"),  // node 12 has no atob
  });
  globalThis.setInterval = (fn, ms) => { timers.push({ fn, ms }); return timers.length; };
  globalThis.clearInterval = () => {};
  globalThis.fetch = (url, opts = {}) => new Promise((resolve, reject) => {
    const u = new URL(url.startsWith("http") ? url : baseUrl + url);
    globalThis.__requests.push(`${opts.method || "GET"} ${u.pathname}${u.search}`);
    const req = http.request(u, { method: opts.method || "GET", headers: opts.headers || {} }, res => {
      let body = "";
      res.setEncoding("utf8");
      res.on("data", c => { body += c; });
      res.on("end", () => resolve({
        ok: res.statusCode >= 200 && res.statusCode < 300, status: res.statusCode, statusText: res.statusMessage,
        headers: { get: k => res.headers[k.toLowerCase()] || null },
        text: async () => body, json: async () => JSON.parse(body),
      }));
    });
    req.on("error", reject);
    if (opts.body) req.write(opts.body);
    req.end();
  });
  process.on("unhandledRejection", e => { globalThis.__errors.push(e); });
  return document;
}

// let pending promise chains and setTimeout(0) callbacks run
export async function settle(rounds = 30) {
  for (let i = 0; i < rounds; i++) await new Promise(r => setTimeout(r, 5));
}

export function text(el) { return el.textContent.replace(/\s+/g, " "); }

export function findButton(root, label) {
  return root.querySelectorAll("button").find(b => b.textContent.trim() === label) || null;
}
