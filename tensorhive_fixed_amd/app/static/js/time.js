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
