// Canvas time-series chart (the reference used Chart.js in WatchBox.vue / WatchGenerator.vue):
// several series, y axis with ticks, time axis, hover read-out.  No dependencies.
"use strict";

export const PALETTE = ["#e4572e", "#29bf12", "#00a5cf", "#ffc914", "#9c51b6", "#ff6f91", "#6cc1a6", "#b8b8b8"];

export class LineChart {
  constructor(canvas, { unit = "", min = 0, max = null, height = 120 } = {}) {
    this.c = canvas; this.unit = unit; this.min = min; this.max = max; this.height = height;
    this.series = new Map();  // name -> {points: [[t, v]], color}
    this.hover = null;
    canvas.addEventListener("mousemove", e => { this.hover = e.offsetX; this.draw(); });
    canvas.addEventListener("mouseleave", () => { this.hover = null; this.draw(); });
  }
  push(name, t, v, keep = 600) {
    let s = this.series.get(name);
    if (!s) { s = { points: [], color: PALETTE[this.series.size % PALETTE.length] }; this.series.set(name, s); }
    s.points.push([t, v]);
    if (s.points.length > keep) s.points.splice(0, s.points.length - keep);
  }
  set(name, points) {
    const s = this.series.get(name) || { color: PALETTE[this.series.size % PALETTE.length] };
    s.points = points; this.series.set(name, s);
  }
  draw() {
    const dpr = window.devicePixelRatio || 1, W = this.c.clientWidth || 300, H = this.height;
    this.c.width = W * dpr; this.c.height = H * dpr; this.c.style.height = H + "px";
    const g = this.c.getContext("2d");
    g.scale(dpr, dpr);
    g.clearRect(0, 0, W, H);
    const all = [...this.series.values()].flatMap(s => s.points).filter(p => p[1] !== null && p[1] !== undefined);
    if (!all.length) { g.fillStyle = "#8b93a1"; g.fillText("no data", 8, 16); return; }
    const t0 = Math.min(...all.map(p => p[0])), t1 = Math.max(...all.map(p => p[0])) || t0 + 1;
    let lo = this.min === null ? Math.min(...all.map(p => p[1])) : this.min;
    let hi = this.max === null ? Math.max(...all.map(p => p[1])) : this.max;
    if (hi <= lo) hi = lo + 1;
    const L = 44, R = 6, T = 6, B = 16;
    const x = t => L + (t - t0) / Math.max(1, t1 - t0) * (W - L - R), y = v => T + (1 - (v - lo) / (hi - lo)) * (H - T - B);
    g.strokeStyle = "#262b36"; g.fillStyle = "#8b93a1"; g.font = "10px system-ui"; g.lineWidth = 1;
    for (let i = 0; i <= 4; i++) {
      const v = lo + (hi - lo) * i / 4, yy = y(v);
      g.beginPath(); g.moveTo(L, yy); g.lineTo(W - R, yy); g.stroke();
      g.fillText(fmtNum(v) + this.unit, 2, yy + 3);
    }
    g.fillText(new Date(t0).toLocaleTimeString(), L, H - 3);
    const lbl = new Date(t1).toLocaleTimeString();
    g.fillText(lbl, W - R - g.measureText(lbl).width, H - 3);
    for (const [, s] of this.series) {
      g.strokeStyle = s.color; g.lineWidth = 1.5; g.beginPath();
      let pen = false;
      for (const [t, v] of s.points) {
        if (v === null || v === undefined) { pen = false; continue; }
        if (!pen) { g.moveTo(x(t), y(v)); pen = true; } else g.lineTo(x(t), y(v));
      }
      g.stroke();
    }
    if (this.hover !== null && this.hover > L) {
      const t = t0 + (this.hover - L) / (W - L - R) * (t1 - t0);
      g.strokeStyle = "#8b93a1"; g.beginPath(); g.moveTo(this.hover, T); g.lineTo(this.hover, H - B); g.stroke();
      let row = 0;
      for (const [name, s] of this.series) {
        let best = null;
        for (const p of s.points) if (best === null || Math.abs(p[0] - t) < Math.abs(best[0] - t)) best = p;
        if (!best || best[1] === null) continue;
        g.fillStyle = s.color;
        g.fillText(`${name}: ${fmtNum(best[1])}${this.unit}`, Math.min(this.hover + 6, W - 150), T + 10 + 11 * row++);
      }
    }
  }
}

export function fmtNum(v) {
  if (v === null || v === undefined || Number.isNaN(v)) return "-";
  const a = Math.abs(v);
  if (a >= 1e6) return (v / 1e6).toFixed(1) + "M";
  if (a >= 1e4) return (v / 1e3).toFixed(1) + "k";
  if (a >= 100) return v.toFixed(0);
  if (a >= 10) return v.toFixed(1);
  return v.toFixed(2);
}
