// Date / schedule helpers (pure functions; unit-tested with node in tests/test_webapp_cli.py).
// Reference: src/utils/scheduleUtils.js (UTC <-> local conversion of restriction schedules).
"use strict";

export const WEEKDAYS = ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"];

// API input format: %Y-%m-%dT%H:%M:%S.%fZ (utils/dates.py INPUT_FORMAT)
export function toApi(d) { return new Date(d).toISOString(); }

// API output is naive UTC with "+00:00"
export function fromApi(s) { return s ? new Date(s) : null; }

export function fmtDateTime(d) {
  if (!d) return "";
  const x = new Date(d);
  return x.toLocaleDateString(undefined, { month: "short", day: "numeric" }) + " " +
    x.toLocaleTimeString(undefined, { hour: "2-digit", minute: "2-digit" });
}

export function fmtDuration(ms) {
  const m = Math.round(ms / 60000);
  if (m < 60) return m + " min";
  const h = Math.floor(m / 60), r = m % 60;
  if (h < 48) return h + " h" + (r ? " " + r + " min" : "");
  return (h / 24).toFixed(1) + " d";
}

// "HH:MM" +/- minutes, wrapped to a day; returns [hhmm, dayShift]
export function shiftHour(hhmm, minutes) {
  const [h, m] = hhmm.split(":").map(Number);
  let t = h * 60 + m + minutes, shift = 0;
  while (t < 0) { t += 1440; shift -= 1; }
  while (t >= 1440) { t -= 1440; shift += 1; }
  return [String(Math.floor(t / 60)).padStart(2, "0") + ":" + String(t % 60).padStart(2, "0"), shift];
}

function shiftDays(days, by) {
  const out = days.map(d => WEEKDAYS[((WEEKDAYS.indexOf(d) + by) % 7 + 7) % 7]);
  return [...new Set(out)].sort((a, b) => WEEKDAYS.indexOf(a) - WEEKDAYS.indexOf(b));
}

// A UTC schedule {scheduleDays, hourStart, hourEnd} seen from a zone `offsetMin` minutes east of
// UTC (JS: -new Date().getTimezoneOffset()).  The days move with the START of the window: a
// window that starts Monday 23:00 UTC starts Tuesday 01:00 in UTC+2.  (The reference shifted the
// days only when the window wrapped past midnight, which mislabels windows such as 23:00-23:30.)
export function scheduleToLocal(s, offsetMin = -new Date().getTimezoneOffset()) {
  const [start, dayShift] = shiftHour(s.hourStart, offsetMin);
  const [end] = shiftHour(s.hourEnd, offsetMin);
  return { ...s, hourStartLocal: start, hourEndLocal: end, scheduleDaysLocal: shiftDays(s.scheduleDays, dayShift) };
}

export function scheduleToUtc(local, offsetMin = -new Date().getTimezoneOffset()) {
  const [start, dayShift] = shiftHour(local.hourStartLocal, -offsetMin);
  const [end] = shiftHour(local.hourEndLocal, -offsetMin);
  return { scheduleDays: shiftDays(local.scheduleDaysLocal, dayShift), hourStart: start, hourEnd: end };
}

// Is `date` inside a UTC schedule window?  (windows that pass midnight continue into the next day)
export function inSchedule(s, date) {
  const d = new Date(date);
  const day = WEEKDAYS[(d.getUTCDay() + 6) % 7], prev = WEEKDAYS[(d.getUTCDay() + 5) % 7];
  const t = d.getUTCHours() * 60 + d.getUTCMinutes();
  const [sh, sm] = s.hourStart.split(":").map(Number), [eh, em] = s.hourEnd.split(":").map(Number);
  const a = sh * 60 + sm, b = eh * 60 + em;
  if (a <= b) return s.scheduleDays.includes(day) && t >= a && t < b;
  return (s.scheduleDays.includes(day) && t >= a) || (s.scheduleDays.includes(prev) && t < b);
}

export function startOfDay(d) { const x = new Date(d); x.setHours(0, 0, 0, 0); return x; }
export function addMinutes(d, m) { return new Date(new Date(d).getTime() + m * 60000); }

// Calendar slot math: index of the slot containing `t` for slots of `slotMin` from `origin`
export function slotIndex(origin, slotMin, t) {
  return Math.floor((new Date(t) - new Date(origin)) / (slotMin * 60000));
}

// Reservation length bounds of the server (models/orm.py Reservation.MIN/MAX_DURATION)
export const MIN_RESERVATION_MIN = 30, MAX_RESERVATION_MIN = 8 * 24 * 60;

export function validReservationRange(start, end) {
  const m = (new Date(end) - new Date(start)) / 60000;
  if (!(m > 0)) return "end must be after start";
  if (m < MIN_RESERVATION_MIN) return "a reservation lasts at least 30 minutes";
  if (m > MAX_RESERVATION_MIN) return "a reservation lasts at most 8 days";
  return null;
}

// ---------------------------------------------------------------- calendar selection
// The calendar is a grid of columns (day d, GPU g) x rows (slot s of `slotMin` minutes).  A drag
// from cell a to cell b selects the GPUs between the two columns' GPUs (in display order) and the
// time between the earlier cell's start and the later cell's end, even across days
// (reference FullCalendar.vue:151 `select` callback + FullCalendarReserve.vue).
export function dragSelection(a, b, dayStarts, gpuIds, slotMin) {
  const t = c => new Date(dayStarts[c.day]).getTime() + c.slot * slotMin * 60000;
  const ta = t(a), tb = t(b);
  const lo = Math.min(ta, tb), hi = Math.max(ta, tb) + slotMin * 60000;
  const g0 = Math.min(a.gpu, b.gpu), g1 = Math.max(a.gpu, b.gpu);
  return { start: new Date(lo), end: new Date(hi), gpus: gpuIds.slice(g0, g1 + 1) };
}

// Lay reservations of one column (one GPU, one day) out as [top, height] fractions of the day;
// overlapping cancelled entries keep their slot (they are drawn struck out).
export function layoutDay(reservations, dayStart) {
  const d0 = new Date(dayStart).getTime(), d1 = d0 + 864e5;
  return reservations
    .map(r => ({ r, s: Math.max(d0, new Date(r.start).getTime()), e: Math.min(d1, new Date(r.end).getTime()) }))
    .filter(x => x.e > x.s)
    .map(x => ({ r: x.r, top: (x.s - d0) / 864e5, height: (x.e - x.s) / 864e5 }));
}

// Does the set of restrictions of a user (GET /restrictions?user_id=..&include_user_groups=true)
// allow GPU `uuid` over the whole window [start, end)?  Mirrors core/verifier.py: a restriction
// covers the GPU if it is global or lists it; the window must be inside the union of the covering
// restrictions' [startsAt, endsAt) x schedule windows.  Checked per `stepMin` minutes.
export function restrictionCovers(r, uuid) {
  return r.isGlobal || (r.resources || []).some(x => x.id === uuid);
}

export function restrictionAllowsAt(r, t) {
  const x = new Date(t).getTime();
  if (x < new Date(r.startsAt).getTime()) return false;
  if (r.endsAt && x >= new Date(r.endsAt).getTime()) return false;
  const sch = r.schedules || [];
  return !sch.length || sch.some(s => inSchedule(s, t));
}

export function allowedWindow(restrictions, uuid, start, end, stepMin = 15) {
  const cover = restrictions.filter(r => restrictionCovers(r, uuid));
  if (!cover.length) return false;
  for (let t = new Date(start).getTime(); t < new Date(end).getTime(); t += stepMin * 60000)
    if (!cover.some(r => restrictionAllowsAt(r, t))) return false;
  return true;
}

// Mean of the reservation usage averages that are known (gpuUtilAvg / memUtilAvg, C67).
export function usageSummary(reservations) {
  const g = reservations.map(r => r.gpuUtilAvg).filter(v => v !== null && v !== undefined);
  const m = reservations.map(r => r.memUtilAvg).filter(v => v !== null && v !== undefined);
  const avg = a => a.length ? Math.round(a.reduce((x, y) => x + y, 0) / a.length) : null;
  return { gpuUtilAvg: avg(g), memUtilAvg: avg(m), samples: g.length };
}
