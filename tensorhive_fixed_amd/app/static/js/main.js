// Dashboard shell (reference: main.js router + axios interceptors, App.vue, TheDash.vue,
// TheLogin.vue): hash router, navigation, login / self sign-up (with the authorized_keys line the
// sign-up needs), account page (self-service password change, PUT /user/password), logout that
// revokes both tokens.
"use strict";
import { S, call, login, logout, onLogout, restoreSession } from "./api.js";
import { adminView } from "./admin.js";
import { jobsView, tasksView } from "./jobs.js";
import { nodesView } from "./nodes.js";
import { reservationsView } from "./reservations.js";
import { $, attempt, card, field, h, input, modal, toast } from "./ui.js";

const VIEWS = {
  nodes: ["Nodes", nodesView], reservations: ["Reservations", reservationsView], jobs: ["Jobs", jobsView],
  tasks: ["Tasks", tasksView], account: ["Account", accountView], admin: ["Admin", adminView, true],
};
let current = null;

function loginView(root) {
  const u = input({ placeholder: "username", autocomplete: "username" });
  const p = input({ type: "password", placeholder: "password", autocomplete: "current-password" });
  const go = async () => {
    const ok = await attempt(() => login(u.value.trim(), p.value));
    if (ok) { if (!location.hash || location.hash === "#login") location.hash = "nodes"; route(); }
  };
  p.addEventListener("keydown", e => { if (e.key === "Enter") go(); });
  root.replaceChildren(h("div", { class: "login" }, card("Sign in", field("username", u), field("password", p),
    h("div", { class: "row" }, h("button", { class: "pri", onclick: go }, "Login"), h("span", { class: "grow" }),
      h("a", { onclick: signupDialog }, "create an account")))));
}

// Self sign-up (POST /user/ssh_signup): the server verifies the user can log in to the nodes over
// SSH with TensorHive's public key, so the dialog shows the authorized_keys line to install first.
async function signupDialog() {
  const key = await call("GET", "/user/authorized_keys_entry").catch(() => null);
  const u = input({ placeholder: "username (your login on the nodes)" }), m = input({ placeholder: "e-mail" });
  const p = input({ type: "password" }), p2 = input({ type: "password" });
  modal("Create an account", h("div", {},
    h("p", { class: "mut" }, "Append this line to ~/.ssh/authorized_keys on the nodes first:"),
    h("pre", { class: "log small" }, key === null ? "(not available)" : typeof key === "string" ? key : JSON.stringify(key)),
    field("username", u), field("e-mail", m), field("password", p), field("repeat password", p2)),
  [["Sign up", async () => {
    if (p.value !== p2.value) { toast("passwords differ", "warn"); return false; }
    const r = await attempt(() => call("POST", "/user/ssh_signup", { username: u.value.trim(), email: m.value, password: p.value }, false));
    if (!r) return false;
    toast("account created: sign in");
  }, "pri"]]);
}

function accountView(root) {
  const box = h("div", {});
  (async () => {
    const me = (await call("GET", `/users/${S.me}`)).user;
    const old = input({ type: "password", autocomplete: "current-password" }), nw = input({ type: "password", autocomplete: "new-password" });
    const nw2 = input({ type: "password", autocomplete: "new-password" });
    const topo = await call("GET", "/nodes/topology").catch(() => null);
    box.replaceChildren(
      card(me.username, h("p", { class: "mut" }, `${me.email} · roles ${(me.roles || []).join(", ")} · groups ${(me.groups || []).map(g => g.name).join(", ") || "-"}`)),
      card("Change password", h("div", { class: "row" }, field("current", old), field("new", nw), field("repeat", nw2),
        h("button", { class: "pri", onclick: async () => {
          if (nw.value !== nw2.value) return toast("passwords differ", "warn");
          const r = await attempt(() => call("PUT", "/user/password", { oldPassword: old.value, newPassword: nw.value }), "password changed");
          if (r) { old.value = nw.value = nw2.value = ""; }
        } }, "change"))),
      topo ? card("GPU topology (NUMA / xGMI)", h("pre", { class: "log small" }, JSON.stringify(topo, null, 1))) : null);
  })().catch(e => box.replaceChildren(h("p", { class: "err" }, e.message)));
  root.replaceChildren(box);
  return null;
}

function route() {
  if (current && current.dispose) current.dispose();
  current = null;
  const main = $("#main");
  if (!S.token) {
    $("#nav").replaceChildren();
    $("#who").replaceChildren();
    return loginView(main);
  }
  const [name, arg] = (location.hash.slice(1) || "nodes").split("/");
  const key = VIEWS[name] && (!VIEWS[name][2] || S.admin) ? name : "nodes";
  $("#nav").replaceChildren(...Object.entries(VIEWS).filter(([, x]) => !x[2] || S.admin).map(([k, [label]]) =>
    h("a", { href: "#" + k, class: k === key ? "on" : "" }, label)));
  $("#who").replaceChildren(h("span", {}, `${S.username || "user " + S.me}${S.admin ? " (admin)" : ""} `),
    h("a", { onclick: async () => { await logout(); location.hash = "login"; route(); } }, "logout"));
  main.replaceChildren();
  try { current = VIEWS[key][1](main, arg ? { id: arg } : {}); } catch (e) { main.append(h("p", { class: "err" }, e.message)); }
}

(async () => {
  let version = "";
  try {
    const c = await (await fetch("/static/config.json")).json();
    S.api = c.apiPath; version = c.version;
    $("#ver").textContent = "v" + c.version;
  } catch (e) { /* served without the daemon: keep /api */ }
  restoreSession(version);
  onLogout(() => { location.hash = "login"; });
  window.addEventListener("hashchange", route);
  route();
})();
