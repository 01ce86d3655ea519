// End-to-end dashboard scenario under node against a live API server (tests/test_webapp_cli.py):
// every view renders, and the main flows run through their real buttons and dialogs.
// argv: <base url> <admin user> <admin password> <plain user> <plain password>
import { findButton, install, settle, text } from "./dom.mjs";

const [base, adminName, adminPw, userName, userPw] = process.argv.slice(2);
const JS = new URL("../../tensorhive_fixed_amd/app/static/js/", import.meta.url).href;
const doc = install(base);
const realFetch = globalThis.fetch;
globalThis.fetch = (url, opts) => url === "/static/config.json"
  ? Promise.resolve({ ok: true, status: 200, json: async () => ({ apiPath: "/api", version: "test" }), headers: { get: () => null } })
  : realFetch(url, opts);
const winListeners = {};
globalThis.addEventListener = (t, fn) => { (winListeners[t] = winListeners[t] || []).push(fn); };

const out = { steps: [], errors: [] };
const step = (name, ok, detail) => { out.steps.push({ name, ok: !!ok, detail }); };
let api, h;  // modules load after install(): api.js reads window.localStorage at import
(async () => {  // node 12: no top-level await
api = await import(JS + "api.js");
({ h } = await import(JS + "ui.js"));
const modal = () => doc.body.querySelectorAll(".modal").slice(-1)[0] || null;
const input = (root, ph) => root.querySelectorAll("input").find(i => i.getAttribute("placeholder") === ph);
const closeModals = () => doc.body.querySelectorAll(".backdrop").forEach(b => b.remove());

async function asAdmin() { await api.login(adminName, adminPw); }
async function asUser() { await api.login(userName, userPw); }

try {
  // ------------------------------------------------------------------ admin: users, groups, schedules
  await asAdmin();
  step("login admin", api.S.admin && api.S.token, api.S.me);
  const { adminView } = await import(JS + "admin.js");
  let root = h("div", {});
  adminView(root);
  await settle();
  step("admin view lists users", text(root).includes(userName), text(root).slice(0, 200));
  findButton(root, "new user").click();
  await settle(5);
  let m = modal();
  m.querySelectorAll("input")[0].value = "spauser";
  m.querySelectorAll("input")[1].value = "spa@example.org";
  m.querySelectorAll("input")[2].value = "spa password 1";
  await findButton(m, "Create").click();
  await settle();
  const users = await api.call("GET", "/users");
  step("create user through dialog", users.some(u => u.username === "spauser"), users.map(u => u.username));
  closeModals();
  findButton(root, "new schedule").click();
  await settle(5);
  m = modal();
  await findButton(m, "Create").click();
  await settle();
  const sch = await api.call("GET", "/schedules");
  step("create schedule (local -> UTC)", sch.length === 1 && sch[0].scheduleDays.length >= 4, sch);
  closeModals();
  findButton(root, "new group").click();
  await settle(5);
  m = modal();
  m.querySelectorAll("input")[0].value = "spagroup";
  await findButton(m, "Create").click();
  await settle();
  const groups = await api.call("GET", "/groups");
  step("create group", groups.some(g => g.name === "spagroup"), groups.map(g => g.name));
  closeModals();

  // ------------------------------------------------------------------ nodes
  const { nodesView } = await import(JS + "nodes.js");
  root = h("div", {});
  const nv = nodesView(root);
  await settle();
  step("nodes view shows hosts", text(root).includes("node-a"), text(root).slice(0, 200));
  nv.dispose();

  // ------------------------------------------------------------------ reservations: drag-select + card
  await asUser();
  const { reservationsView } = await import(JS + "reservations.js");
  root = h("div", {});
  const rv = reservationsView(root);
  await settle(60);
  const cells = root.querySelectorAll("td").filter(td => td.classList.contains("cal-cell"));
  step("calendar grid rendered", cells.length >= 48, cells.length);
  // tomorrow (day 1 of the default 3-day view): 20:00-22:00 on the first two GPU columns
  const ngpu = root.querySelectorAll("th").filter(t => t.classList.contains("cal-gpu")).length / 3;
  const cell = (day, gpu, slot) => cells[slot * (3 * ngpu) + day * ngpu + gpu];
  await cell(1, 0, 40).dispatch("mousedown");
  await cell(1, 1, 43).dispatch("mouseenter");
  const tbl = root.querySelectorAll("table").find(t => t.classList.contains("cal"));
  await tbl.dispatch("mouseup");
  await settle(5);
  m = modal();
  step("drag-select opens the reserve dialog", m && text(m).includes("Reserve GPUs"), m && text(m).slice(0, 120));
  input(m, "title").value = "spa reservation";
  await findButton(m, "Reserve").click();
  await settle(40);
  const resources = await api.call("GET", "/resources");
  const t0 = new Date(Date.now() - 864e5).toISOString(), t1 = new Date(Date.now() + 3 * 864e5).toISOString();
  const rs = await api.call("GET", "/reservations" + api.qs({ resources_ids: resources.map(r => r.id), start: t0, end: t1 }));
  const mine = rs.filter(r => r.title === "spa reservation");
  step("two GPU columns -> two reservations of 2 h", mine.length === 2 &&
       mine.every(r => new Date(r.end) - new Date(r.start) === 2 * 3600e3), mine.map(r => [r.resourceId, r.start, r.end]));
  closeModals();
  await settle(20);
  const block = root.querySelectorAll("div").find(d => d.classList.contains("cal-block"));
  step("reservation blocks drawn", !!block, null);
  if (block) {
    await block.click();
    await settle(20);
    m = modal();
    step("reservation card with usage averages", m && text(m).includes("avg GPU util"), m && text(m).slice(0, 160));
    m.querySelectorAll("input")[0].value = "renamed reservation";
    await findButton(m, "Save").click();
    await settle(20);
    const after = await api.call("GET", "/reservations" + api.qs({ resources_ids: resources.map(r => r.id), start: t0, end: t1 }));
    step("edit reservation title", after.some(r => r.title === "renamed reservation"), after.map(r => r.title));
    closeModals();
  }
  rv.dispose();

  // ------------------------------------------------------------------ jobs: create, task, duplicate, launch
  const { jobsView, tasksView } = await import(JS + "jobs.js");
  root = h("div", {});
  let jv = jobsView(root, {});
  await settle();
  findButton(root, "new job").click();
  await settle(5);
  m = modal();
  input(m, "name").value = "spajob";
  await findButton(m, "Create").click();
  await settle(10);
  const jobId = +location.hash.split("/")[1];
  step("create job -> details route", jobId > 0, location.hash);
  jv.dispose();
  closeModals();
  root = h("div", {});
  jv = jobsView(root, { id: jobId });
  await settle(30);
  step("job details render", text(root).includes("spajob"), text(root).slice(0, 160));
  findButton(root, "add task").click();
  await settle(30);
  m = modal();
  m.querySelectorAll("input").find(i => i.getAttribute("placeholder") === "python train.py").value = "python train.py";
  m.querySelectorAll("textarea")[1].value = "--epochs 3\n--lr=0.1";
  await findButton(m, "Create").click();
  await settle(30);
  let job = ({ tasks: (await api.call("GET", "/tasks" + api.qs({ jobId }))).tasks });
  step("add task with params", job.tasks.length === 1 && job.tasks[0].fullCommand.includes("--epochs 3 --lr=0.1"),
       job.tasks.map(t => t.fullCommand));
  closeModals();
  await settle(30);
  const dup = findButton(root, "duplicate");
  if (dup) {
    dup.click();
    await settle(30);
    m = modal();
    await findButton(m, "Create").click();
    await settle(30);
  }
  job = ({ tasks: (await api.call("GET", "/tasks" + api.qs({ jobId }))).tasks });
  step("duplicate task", job.tasks.length === 2 && job.tasks[1].fullCommand === job.tasks[0].fullCommand,
       job.tasks.map(t => t.fullCommand));
  closeModals();
  await settle(30);
  findButton(root, "distributed launch").click();
  await settle(30);
  m = modal();
  const kind = m.querySelectorAll("select")[0];
  kind.value = "tf2";
  await kind.dispatch("change");
  await settle(5);
  const preview = m.querySelectorAll("pre")[0];
  step("TF_CONFIG preview", preview && text(preview).includes("TF_CONFIG="), preview && text(preview).slice(0, 160));
  await findButton(m, "Generate tasks").click();
  await settle(30);
  job = ({ tasks: (await api.call("GET", "/tasks" + api.qs({ jobId }))).tasks });
  step("generate TF2 tasks", job.tasks.length === 3 && job.tasks[2].fullCommand.includes("TF_CONFIG="), job.tasks.length);
  closeModals();
  await settle(30);
  const logBtn = findButton(root, "log");
  if (logBtn) { logBtn.click(); await settle(30); }
  step("log viewer opens", text(root).includes(`Task #`), null);
  jv.dispose();
  root = h("div", {});
  const tv = tasksView(root);
  await settle(30);
  step("tasks overview", text(root).includes("python train.py"), text(root).slice(0, 120));
  tv.dispose();

  // ------------------------------------------------------------------ shell: routing + account + logout
  location.hash = "account";
  await import(JS + "main.js");
  await settle(40);
  step("account page via router", text(doc.body.querySelector("#main")).includes("Change password"),
       text(doc.body.querySelector("#main")).slice(0, 120));
  const main = doc.body.querySelector("#main");
  const pw = main.querySelectorAll("input");
  pw[0].value = userPw; pw[1].value = "new password 9"; pw[2].value = "new password 9";
  await findButton(main, "change").click();
  await settle(20);
  await api.logout();
  let relogin = true;
  try { await api.login(userName, "new password 9"); } catch (e) { relogin = false; }
  step("self-service password change", relogin, null);
  const tok = api.S.refresh;
  await api.logout();
  const rr = await realFetch("/api/user/refresh", { headers: { Authorization: "Bearer " + tok } });
  step("logout revokes the refresh token", rr.status === 401, rr.status);
} catch (e) {
  out.errors.push(String(e && e.stack || e));
}
out.errors.push(...globalThis.__errors.map(e => String(e && e.stack || e)));
out.requests = globalThis.__requests.length;
console.log(JSON.stringify(out));
process.exit(0);
})();
