// Administration (reference: views/UsersOverview.vue, users_overview/UsersInfo.vue, GroupsInfo.vue,
// utils/scheduleUtils.js).
//
// Users: create, edit (username / e-mail / password / admin role, PUT /user), delete, group
// membership.  Groups: create, rename, default flag, members.  Restrictions: create, edit
// (name, validity, global), delete, and the targets they apply to -- users, groups, GPUs, whole
// hosts, weekly schedules -- as chips with add / remove.  Schedules: create and edit in LOCAL
// time; the API stores UTC (scheduleToUtc / scheduleToLocal in time.js shift the hours and, when
// the window start crosses midnight, the days).
"use strict";
import { call } from "./api.js";
import { WEEKDAYS, fmtDateTime, scheduleToLocal, scheduleToUtc, toApi } from "./time.js";
import { View, attempt, card, confirmBox, dtInput, dtValue, errToast, field, h, input, modal, pill, select, table, toast } from "./ui.js";

function chip(text, onRemove, title) {
  return h("span", { class: "chip", title: title || "" }, text, onRemove ? h("a", { onclick: onRemove, title: "remove" }, " x") : null);
}

// apply (on) / remove a restriction to / from a target
const TARGETS = {
  users: (r, t, on) => on ? call("PUT", `/restrictions/${r}/users/${t}`) : call("DELETE", `/restrictions/${r}/users/${t}`),
  groups: (r, t, on) => on ? call("PUT", `/restrictions/${r}/groups/${t}`) : call("DELETE", `/restrictions/${r}/groups/${t}`),
  resources: (r, t, on) => on ? call("PUT", `/restrictions/${r}/resources/${t}`) : call("DELETE", `/restrictions/${r}/resources/${t}`),
  hosts: (r, t, on) => on ? call("PUT", `/restrictions/${r}/hosts/${t}`) : call("DELETE", `/restrictions/${r}/hosts/${t}`),
  schedules: (r, t, on) => on ? call("PUT", `/restrictions/${r}/schedules/${t}`) : call("DELETE", `/restrictions/${r}/schedules/${t}`),
};

function dayPicker(days) {
  const boxes = WEEKDAYS.map(d => ({ d, el: h("input", { type: "checkbox", checked: days.includes(d) }) }));
  return { el: h("span", { class: "row wrap" }, boxes.map(b => h("label", {}, b.el, " " + b.d.slice(0, 3)))),
           value: () => boxes.filter(b => b.el.checked).map(b => b.d) };
}

export function adminView(root) {
  const v = new View(root);
  const usersBox = h("div", {}), groupsBox = h("div", {}), restrBox = h("div", {}), schedBox = h("div", {});
  let D = { users: [], groups: [], restrictions: [], schedules: [], resources: [] };
  const reload = async () => {
    const [users, groups, restrictions, schedules, resources] = await Promise.all([
      call("GET", "/users"), call("GET", "/groups"), call("GET", "/restrictions"), call("GET", "/schedules"), call("GET", "/resources")]);
    if (!v.alive) return;
    D = { users, groups, restrictions, schedules, resources };
    drawUsers(); drawGroups(); drawRestrictions(); drawSchedules();
  };
  const run = (fn, msg) => attempt(fn, msg).then(r => { reload(); return r; });

  // ---------------------------------------------------------------- users
  function userDialog(u) {
    const name = input({ value: u ? u.username : "", maxlength: 40 }), mail = input({ value: u ? u.email : "" });
    const pw = input({ type: "password", placeholder: u ? "unchanged" : "password" });
    const admin = h("input", { type: "checkbox", checked: u ? (u.roles || []).includes("admin") : false });
    const groups = D.groups.map(g => ({ g, el: h("input", { type: "checkbox", checked: u ? (u.groups || []).some(x => x.id === g.id) : g.isDefault }) }));
    modal(u ? `Edit ${u.username}` : "New user", h("div", {}, field("username", name), field("e-mail", mail), field("password", pw),
      h("label", {}, admin, " administrator"), h("h4", {}, "groups"), h("div", { class: "row wrap" }, groups.map(x => h("label", {}, x.el, " " + x.g.name)))),
    [[u ? "Save" : "Create", async () => {
      let id = u ? u.id : null;
      if (u) {
        const nv = { id: u.id };
        if (name.value !== u.username) nv.username = name.value;
        if (mail.value !== u.email) nv.email = mail.value;
        if (pw.value) nv.password = pw.value;
        const roles = admin.checked ? ["user", "admin"] : ["user"];
        if (roles.join() !== [...(u.roles || [])].sort((a, b) => (a === "user" ? -1 : 1)).join()) nv.roles = roles;
        if (Object.keys(nv).length > 1 && !(await attempt(() => call("PUT", "/user", nv)))) return false;
      } else {
        const r = await attempt(() => call("POST", "/user/create", { username: name.value, email: mail.value, password: pw.value,
          roles: admin.checked ? ["user", "admin"] : ["user"] }));
        if (!r) return false;
        id = r.user.id;
      }
      const fresh = u ? u : (await call("GET", `/users/${id}`)).user;
      for (const x of groups) {
        const member = (fresh.groups || []).some(g => g.id === x.g.id);
        if (x.el.checked && !member) await attempt(() => call("PUT", `/groups/${x.g.id}/users/${id}`));
        if (!x.el.checked && member) await attempt(() => call("DELETE", `/groups/${x.g.id}/users/${id}`));
      }
      toast(u ? "user saved" : "user created");
      reload();
    }, "pri"]]);
  }
  function drawUsers() {
    usersBox.replaceChildren(card("Users", h("div", { class: "row" }, h("button", { class: "pri", onclick: () => userDialog(null) }, "new user")),
      table([{ label: "id", key: "id" }, { label: "username", key: "username" }, { label: "e-mail", key: "email" },
        { label: "roles", render: u => (u.roles || []).map(r => pill(r, r === "admin" ? "warn" : "")) },
        { label: "groups", render: u => (u.groups || []).map(g => chip(g.name)) },
        { label: "restrictions", render: u => D.restrictions.filter(r => (r.users || []).some(x => x.id === u.id)).map(r => chip(r.name || `#${r.id}`)) },
        { label: "created", render: u => fmtDateTime(u.createdAt) },
        { label: "", render: u => h("span", { class: "row nowrap" }, h("button", { onclick: () => userDialog(u) }, "edit"),
          h("button", { class: "danger", onclick: async () => { if (await confirmBox(`Delete user ${u.username}?`)) run(() => call("DELETE", `/user/delete/${u.id}`), "user deleted"); } }, "delete")) }],
      D.users)));
  }

  // ---------------------------------------------------------------- groups
  function groupDialog(g) {
    const name = input({ value: g ? g.name : "", maxlength: 40 }), def = h("input", { type: "checkbox", checked: g ? g.isDefault : false });
    modal(g ? `Edit group ${g.name}` : "New group", h("div", {}, field("name", name),
      h("label", {}, def, " default group (new users join it)")),
    [[g ? "Save" : "Create", async () => {
      const body = { name: name.value, isDefault: def.checked };
      const r = g ? await attempt(() => call("PUT", `/groups/${g.id}`, body)) : await attempt(() => call("POST", "/groups", body));
      if (!r) return false;
      reload();
    }, "pri"]]);
  }
  function drawGroups() {
    groupsBox.replaceChildren(card("Groups", h("div", { class: "row" }, h("button", { class: "pri", onclick: () => groupDialog(null) }, "new group")),
      table([{ label: "id", key: "id" }, { label: "name", key: "name" }, { label: "default", render: g => g.isDefault ? pill("default", "ok") : "" },
        { label: "members", render: g => {
          const add = select([["", "+ add"], ...D.users.filter(u => !(g.users || []).some(x => x.id === u.id)).map(u => [u.id, u.username])], "");
          add.addEventListener("change", () => add.value && run(() => call("PUT", `/groups/${g.id}/users/${add.value}`), "member added"));
          return h("span", { class: "row wrap" }, (g.users || []).map(u => chip(u.username, () => run(() => call("DELETE", `/groups/${g.id}/users/${u.id}`), "member removed"))), add);
        } },
        { label: "restrictions", render: g => D.restrictions.filter(r => (r.groups || []).some(x => x.id === g.id)).map(r => chip(r.name || `#${r.id}`)) },
        { label: "", render: g => h("span", { class: "row nowrap" }, h("button", { onclick: () => groupDialog(g) }, "edit"),
          h("button", { class: "danger", onclick: async () => { if (await confirmBox(`Delete group ${g.name}?`)) run(() => call("DELETE", `/groups/${g.id}`), "group deleted"); } }, "delete")) }],
      D.groups)));
  }

  // ---------------------------------------------------------------- restrictions
  function restrictionDialog(r) {
    const name = input({ value: r ? r.name || "" : "" });
    const s = dtInput(r ? r.startsAt : new Date()), e = r && r.endsAt ? dtInput(r.endsAt) : h("input", { type: "datetime-local" });
    const glob = h("input", { type: "checkbox", checked: r ? r.isGlobal : false });
    modal(r ? `Edit restriction ${r.name || r.id}` : "New restriction", h("div", {}, field("name", name),
      h("div", { class: "row" }, field("valid from", s), field("until (empty = forever)", e)),
      h("label", {}, glob, " global (covers every GPU)")),
    [[r ? "Save" : "Create", async () => {
      const body = { name: name.value, startsAt: toApi(dtValue(s)), endsAt: e.value ? toApi(dtValue(e)) : null, isGlobal: glob.checked };
      const x = r ? await attempt(() => call("PUT", `/restrictions/${r.id}`, body)) : await attempt(() => call("POST", "/restrictions", body));
      if (!x) return false;
      reload();
    }, "pri"]]);
  }
  function targetCell(r, kind, items, label, keyOf, all) {
    const apply = (t, on) => TARGETS[kind](r.id, encodeURIComponent(t), on);
    const add = select([["", "+"], ...all.filter(a => !items.some(i => keyOf(i) === keyOf(a))).map(a => [keyOf(a), label(a)])], "");
    add.addEventListener("change", () => add.value && run(() => apply(add.value, true), "restriction applied"));
    return h("span", { class: "row wrap" }, items.map(i => chip(label(i), () => run(() => apply(keyOf(i), false), "restriction removed"))), add);
  }
  function drawRestrictions() {
    const hosts = [...new Set(D.resources.map(x => x.hostname).filter(Boolean))].map(x => ({ id: x }));
    const gpuLabel = g => `${g.hostname || ""}:${g.name || g.id.slice(4, 12)}`;
    const schedLabel = s => { const l = scheduleToLocal(s); return `${l.scheduleDaysLocal.map(d => d.slice(0, 2)).join("")} ${l.hourStartLocal}-${l.hourEndLocal}`; };
    restrBox.replaceChildren(card("Restrictions", h("div", { class: "row" }, h("button", { class: "pri", onclick: () => restrictionDialog(null) }, "new restriction"),
      h("span", { class: "mut" }, "a user may reserve / use a GPU only inside the union of the restrictions covering it")),
      table([{ label: "id", key: "id" }, { label: "name", render: r => r.name || "" },
        { label: "valid", render: r => `${fmtDateTime(r.startsAt)} - ${r.endsAt ? fmtDateTime(r.endsAt) : "forever"}` },
        { label: "scope", render: r => r.isGlobal ? pill("global", "warn") : "" },
        { label: "users", render: r => targetCell(r, "users", r.users || [], u => u.username, u => u.id, D.users) },
        { label: "groups", render: r => targetCell(r, "groups", r.groups || [], g => g.name, g => g.id, D.groups) },
        { label: "GPUs", render: r => r.isGlobal ? h("span", { class: "mut" }, "all") : targetCell(r, "resources", r.resources || [], gpuLabel, g => g.id, D.resources) },
        { label: "hosts", render: r => r.isGlobal ? "" : targetCell(r, "hosts", [], x => x.id, x => x.id, hosts) },
        { label: "schedules (local)", render: r => targetCell(r, "schedules", r.schedules || [], schedLabel, s => s.id, D.schedules) },
        { label: "", render: r => h("span", { class: "row nowrap" }, h("button", { onclick: () => restrictionDialog(r) }, "edit"),
          h("button", { class: "danger", onclick: async () => { if (await confirmBox(`Delete restriction ${r.name || r.id}?`)) run(() => call("DELETE", `/restrictions/${r.id}`), "restriction deleted"); } }, "delete")) }],
      D.restrictions)));
  }

  // ---------------------------------------------------------------- schedules (edited in local time)
  function scheduleDialog(s) {
    const l = s ? scheduleToLocal(s) : { scheduleDaysLocal: WEEKDAYS.slice(0, 5), hourStartLocal: "08:00", hourEndLocal: "18:00" };
    const days = dayPicker(l.scheduleDaysLocal);
    const a = input({ type: "time", value: l.hourStartLocal }), b = input({ type: "time", value: l.hourEndLocal });
    const utc = h("p", { class: "mut" });
    const show = () => {
      const u = scheduleToUtc({ scheduleDaysLocal: days.value(), hourStartLocal: a.value || "00:00", hourEndLocal: b.value || "00:00" });
      utc.textContent = `stored as UTC: ${u.scheduleDays.map(d => d.slice(0, 3)).join(",")} ${u.hourStart}-${u.hourEnd}`;
    };
    [a, b].forEach(x => x.addEventListener("input", show));
    days.el.addEventListener("change", show);
    show();
    modal(s ? `Edit schedule #${s.id}` : "New schedule", h("div", {}, field("days (local)", days.el),
      h("div", { class: "row" }, field("from (local)", a), field("to (local)", b, "a window may pass midnight")), utc),
    [[s ? "Save" : "Create", async () => {
      if (!days.value().length) { toast("pick at least one day", "warn"); return false; }
      const body = scheduleToUtc({ scheduleDaysLocal: days.value(), hourStartLocal: a.value, hourEndLocal: b.value });
      const x = s ? await attempt(() => call("PUT", `/schedules/${s.id}`, body)) : await attempt(() => call("POST", "/schedules", body));
      if (!x) return false;
      reload();
    }, "pri"]]);
  }
  function drawSchedules() {
    schedBox.replaceChildren(card("Schedules", h("div", { class: "row" }, h("button", { class: "pri", onclick: () => scheduleDialog(null) }, "new schedule"),
      h("span", { class: "mut" }, `shown in local time (UTC${new Date().getTimezoneOffset() <= 0 ? "+" : "-"}${Math.abs(new Date().getTimezoneOffset() / 60)})`)),
      table([{ label: "id", key: "id" },
        { label: "days", render: s => scheduleToLocal(s).scheduleDaysLocal.map(d => d.slice(0, 3)).join(", ") },
        { label: "from", render: s => scheduleToLocal(s).hourStartLocal }, { label: "to", render: s => scheduleToLocal(s).hourEndLocal },
        { label: "UTC", render: s => h("span", { class: "mut" }, `${s.scheduleDays.map(d => d.slice(0, 3)).join(",")} ${s.hourStart}-${s.hourEnd}`) },
        { label: "used by", render: s => D.restrictions.filter(r => (r.schedules || []).some(x => x.id === s.id)).map(r => chip(r.name || `#${r.id}`)) },
        { label: "", render: s => h("span", { class: "row nowrap" }, h("button", { onclick: () => scheduleDialog(s) }, "edit"),
          h("button", { class: "danger", onclick: async () => { if (await confirmBox(`Delete schedule #${s.id}?`)) run(() => call("DELETE", `/schedules/${s.id}`), "schedule deleted"); } }, "delete")) }],
      D.schedules)));
  }

  root.replaceChildren(usersBox, groupsBox, restrBox, schedBox);
  reload().catch(errToast);
  return v;
}
