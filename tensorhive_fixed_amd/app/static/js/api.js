// REST client + session (reference: src/api/index.js, main.js:92-128 axios interceptors, store.js).
// Every request goes through call(method, path, body): bearer token, one refresh-and-retry on 401,
// logout when the refresh itself is rejected.  All API traffic of the dashboard is in this form,
// so tests/test_webapp_cli.py can extract the (method, path) set statically.
"use strict";

export const S = {
  api: "/api", token: null, refresh: null, me: null, username: null, admin: false,
  hostAge: {}, version: "", listeners: new Set(),
};

const LS = window.localStorage;

export function jwtClaims(tok) {
  try { return JSON.parse(atob(tok.split(".")[1].replace(/-/g, "+").replace(/_/g, "/"))); } catch (e) { return {}; }
}

export function setSession(access, refresh, username) {
  S.token = access;
  if (refresh) S.refresh = refresh;
  const c = jwtClaims(access);
  S.me = c.identity !== undefined ? c.identity : c.sub;
  S.admin = ((c.user_claims || c.claims || {}).roles || c.roles || []).includes("admin");
  if (username) S.username = username;
  LS.setItem("th.token", access);
  if (refresh) LS.setItem("th.refresh", refresh);
  if (username) LS.setItem("th.username", username);
}

export function restoreSession(version) {
  if (LS.getItem("th.version") !== version) {  // a new server version drops cached state (reference main.js)
    ["th.token", "th.refresh", "th.username"].forEach(k => LS.removeItem(k));
    LS.setItem("th.version", version);
  }
  const t = LS.getItem("th.token");
  if (t) setSession(t, LS.getItem("th.refresh"), LS.getItem("th.username"));
  return !!t;
}

export function onLogout(fn) { S.listeners.add(fn); }

function clearSession() {
  S.token = S.refresh = S.me = S.username = null;
  S.admin = false;
  ["th.token", "th.refresh", "th.username"].forEach(k => LS.removeItem(k));
  S.listeners.forEach(fn => fn());
}

async function raw(method, path, body, token) {
  const hdr = { "Content-Type": "application/json" };
  if (token) hdr.Authorization = "Bearer " + token;
  return fetch(S.api + path, { method, headers: hdr, body: body === undefined || body === null ? undefined : JSON.stringify(body) });
}

async function parse(r) {
  const txt = await r.text();
  let data;
  try { data = txt ? JSON.parse(txt) : {}; } catch (e) { data = { msg: txt }; }
  return data;
}

export class ApiError extends Error {
  constructor(status, msg, body) { super(msg); this.status = status; this.body = body; }
}

export async function call(method, path, body = null, retry = true) {
  let r = await raw(method, path, body, S.token);
  if (r.status === 401 && retry && S.refresh && path !== "/user/login") {
    const rr = await raw("GET", "/user/refresh", null, S.refresh);  // access token expired: refresh once
    if (rr.ok) {
      const d = await parse(rr);
      setSession(d.access_token);
      return call(method, path, body, false);
    }
    clearSession();
    throw new ApiError(401, "session expired", {});
  }
  const ages = r.headers.get("X-Host-Sample-Age-Ms");
  if (ages) S.hostAge = Object.fromEntries(ages.split(",").filter(Boolean).map(kv => {
    const i = kv.lastIndexOf("="); return [kv.slice(0, i), +kv.slice(i + 1)];
  }));
  const data = await parse(r);
  if (!r.ok) throw new ApiError(r.status, (data && (data.msg || data.detail || data.title)) || r.statusText, data);
  return data;
}

export async function login(username, password) {
  const d = await call("POST", "/user/login", { username, password }, false);
  setSession(d.access_token, d.refresh_token, username);
  return d;
}

// Logout revokes BOTH tokens (access: DELETE /user/logout, refresh: DELETE /user/logout/refresh_token).
export async function logout() {
  const acc = S.token, ref = S.refresh;
  clearSession();
  try { if (acc) await raw("DELETE", "/user/logout", null, acc); } catch (e) { /* offline */ }
  try { if (ref) await raw("DELETE", "/user/logout/refresh_token", null, ref); } catch (e) { /* offline */ }
}

export function qs(params) {
  const q = new URLSearchParams();
  for (const [k, v] of Object.entries(params)) {
    if (v === undefined) continue;
    q.append(k, v === null ? "null" : Array.isArray(v) ? v.join(",") : String(v));
  }
  const s = q.toString();
  return s ? "?" + s : "";
}
