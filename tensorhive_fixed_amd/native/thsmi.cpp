// libthsmi / th-smi: MI355X telemetry sampler for tensorhive_fixed_amd (SURVEY N01 + N05).
//
// Replaces the reference's `nvidia-smi --query-gpu` + `nvidia-smi pmon` + one `ps -o user <pid>`
// SSH round trip PER PROCESS (tensorhive/core/monitors/GPUMonitor.py:20-158).  One call returns,
// for every GPU of the node: identity (40-char "GPU-<uuid>", HIP index, BDF, NUMA node, KFD id),
// the reference's metric keys (utilization, mem_util, mem_free/used/total MiB, temp, power,
// fan_speed = null on the passively cooled MI355X) plus MI355X extras (hotspot/HBM temperature,
// gfx/mem clocks, energy, xGMI read/write throughput from the PMFW accumulators), and the GPU's
// processes already attributed to a UNIX owner, with the TensorHive task they CLAIM
// (TENSORHIVE_TASK_ID from /proc/<pid>/environ) and the facts that claim is checked against:
// session id, process group and parent chain (core/attribution.py accepts the claim only for a
// process inside that task's th-run session running as the task's uid).  Process discovery has two sources:
//   * amdsmi + KFD sysfs (/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>) -- these are HOST pids;
//     a pid is only trusted when the process it names in OUR /proc really has /dev/kfd open
//     (inside a container, a host pid may be absent or name an unrelated process);
//   * DRM fdinfo of the amdgpu render nodes (/proc/<pid>/fdinfo/<fd>: drm-pdev, drm-client-id,
//     drm-memory-vram) -- pids of our own PID namespace, per device BDF, with VRAM.
// CPU utilisation is a /proc/stat delta between two calls (no `sleep 1`).
//
// C ABI (ctypes):  thsmi_init() -> 0 | <0,  thsmi_sample_json(buf, cap) -> bytes | -needed,
//                  thsmi_topology_json(buf, cap), thsmi_shutdown().
// CLI: th-smi [--json] [--stream MS] [--topology]
#include <amd_smi/amdsmi.h>
#include <dirent.h>
#include <pwd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace {

struct Gpu {
  amdsmi_processor_handle h;
  int hip_index = -1;
  std::string uuid, name, bdf;
  int numa = -1;
  uint64_t kfd_id = 0;
  // previous accumulators for rates
  uint64_t xr_prev = 0, xw_prev = 0, energy_prev = 0;
  uint64_t ts_prev = 0;
  // HBM bandwidth from gpu_metrics.mem_activity_acc, rate taken over >= 1 s windows (the firmware
  // table refreshes in steps; a 0.25 s delta is too coarse).
  uint64_t mem_acc_prev = 0, mem_ts_prev = 0;
  double hbm_gbps = -1;
};

// GB/s per unit/s of mem_activity_acc on MI355X, fitted against timed device streams on two boxes:
// add 5.78 TB/s, copy 5.01 TB/s, half-duty add 2.89 TB/s -> 0.0938 / 0.0973 / 0.0945
// (profiles/r02_telemetry/hbm_calibration.jsonl); copy 4.80 TB/s on a second box -> 0.0820
// (gpu_tests_fullwidth_hbm_probe.log).  The accumulator counts UMC activity, not bytes, so the
// factor moves with the box and the access mix; 0.0897 is the minimax fit (max error 8.5 % over
// these four).  Override with TENSORHIVE_HBM_GBPS_PER_ACC.
double hbm_gbps_per_acc() {
  static double k = [] {
    const char* e = getenv("TENSORHIVE_HBM_GBPS_PER_ACC");
    return (e && *e) ? atof(e) : 0.0897;
  }();
  return k;
}

std::mutex g_mu;
bool g_init = false;
std::vector<Gpu> g_gpus;
// The monitor's own processes (this process, the th-probe agent, th-counters, ...) are never
// tenants: they are dropped from every process list (reference: InfrastructureManager.py:57,70-76
// filtered its own non-tenant commands).  Set with thsmi_set_ignored_pids / th-smi --ignore-pid.
std::set<long> g_ignored;

bool ignored_pid(long pid) { return pid == (long)getpid() || g_ignored.count(pid) > 0; }
unsigned long long g_cpu_prev_total = 0, g_cpu_prev_idle = 0;

uint64_t now_ns() {
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + t.tv_nsec;
}

std::string esc(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  return o;
}

std::string num(double v) {
  char b[64];
  snprintf(b, sizeof b, "%.6g", v);
  return b;
}

std::string metric(const char* unit, bool ok, double v) {
  return std::string("{\"value\":") + (ok ? num(v) : "null") + ",\"unit\":\"" + unit + "\"}";
}

std::string read_file(const std::string& p, size_t cap = 1 << 16) {
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) return "";
  std::string s;
  s.resize(cap);
  size_t n = fread(&s[0], 1, cap, f);
  fclose(f);
  s.resize(n);
  return s;
}

// ------------------------------------------------------------------ process attribution (N05)
struct ProcInfo {
  std::string owner, cmd, task_id;
  long uid = -1;
  long ppid = -1, pgid = -1, sid = -1;
  std::vector<long> ancestors;  // parent, grandparent, ... (init and kernel threads excluded)
};

// ppid / pgrp / session from /proc/<pid>/stat ("pid (comm) state ppid pgrp session ..."; comm may
// hold spaces and parentheses, so parse after the LAST ')').
bool read_stat_ids(long pid, long& ppid, long& pgid, long& sid) {
  const std::string st = read_file("/proc/" + std::to_string(pid) + "/stat", 4096);
  const size_t rp = st.rfind(')');
  if (rp == std::string::npos) return false;
  char state = 0;
  return sscanf(st.c_str() + rp + 1, " %c %ld %ld %ld", &state, &ppid, &pgid, &sid) == 4;
}

ProcInfo resolve_pid(long pid) {
  ProcInfo pi;
  const std::string base = "/proc/" + std::to_string(pid);
  std::string st = read_file(base + "/status");
  const char* u = strstr(st.c_str(), "\nUid:");
  if (u) {
    pi.uid = strtol(u + 5, nullptr, 10);
    struct passwd pw, *res = nullptr;
    char buf[4096];
    if (getpwuid_r((uid_t)pi.uid, &pw, buf, sizeof buf, &res) == 0 && res) pi.owner = res->pw_name;
    else pi.owner = std::to_string(pi.uid);
  }
  std::string cl = read_file(base + "/cmdline", 4096);
  for (char& c : cl)
    if (c == 0) c = ' ';
  while (!cl.empty() && cl.back() == ' ') cl.pop_back();
  pi.cmd = cl;
  // Session, process group and the parent chain: what the daemon checks a claimed task id against
  // (a th-run task's processes share its session, or descend from its monitor -- core/attribution.py).
  // The environment below is user-writable; these are not.
  if (read_stat_ids(pid, pi.ppid, pi.pgid, pi.sid)) {
    long cur = pi.ppid;
    for (int depth = 0; cur > 1 && depth < 64; ++depth) {
      pi.ancestors.push_back(cur);
      long pp = -1, pg = -1, sd = -1;
      if (!read_stat_ids(cur, pp, pg, sd)) break;
      cur = pp;
    }
  }
  std::string env = read_file(base + "/environ", 1 << 20);  // readable for own / same-uid / root
  const char* key = "TENSORHIVE_TASK_ID=";
  for (size_t i = 0; i < env.size();) {
    size_t j = env.find('\0', i);
    if (j == std::string::npos) j = env.size();
    if (env.compare(i, strlen(key), key) == 0) pi.task_id = env.substr(i + strlen(key), j - i - strlen(key));
    i = j + 1;
  }
  return pi;
}

// KFD sysfs: pid -> set of kfd gpu ids it has memory on
std::map<uint64_t, std::set<long>> kfd_processes() {
  std::map<uint64_t, std::set<long>> out;
  DIR* d = opendir("/sys/class/kfd/kfd/proc");
  if (!d) return out;
  struct dirent* e;
  while ((e = readdir(d)) != nullptr) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    long pid = atol(e->d_name);
    std::string pdir = std::string("/sys/class/kfd/kfd/proc/") + e->d_name;
    DIR* pd = opendir(pdir.c_str());
    if (!pd) continue;
    struct dirent* f;
    while ((f = readdir(pd)) != nullptr) {
      if (strncmp(f->d_name, "vram_", 5) == 0) out[strtoull(f->d_name + 5, nullptr, 10)].insert(pid);
    }
    closedir(pd);
  }
  closedir(d);
  return out;
}

// does /proc/<pid>/fd contain an open /dev/kfd?  (same-uid or root can read the links)
bool has_kfd_open(long pid) {
  const std::string fdd = "/proc/" + std::to_string(pid) + "/fd";
  DIR* d = opendir(fdd.c_str());
  if (!d) return false;
  bool found = false;
  char tgt[256];
  struct dirent* e;
  while (!found && (e = readdir(d)) != nullptr) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    const std::string l = fdd + "/" + e->d_name;
    ssize_t n = readlink(l.c_str(), tgt, sizeof tgt - 1);
    if (n > 0) {
      tgt[n] = 0;
      found = strcmp(tgt, "/dev/kfd") == 0;
    }
  }
  closedir(d);
  return found;
}

// DRM fdinfo scan: bdf -> pid -> VRAM bytes (summed over distinct drm clients of the process)
std::map<std::string, std::map<long, uint64_t>> drm_processes() {
  std::map<std::string, std::map<long, uint64_t>> out;
  DIR* pd = opendir("/proc");
  if (!pd) return out;
  struct dirent* pe;
  char tgt[256];
  while ((pe = readdir(pd)) != nullptr) {
    if (pe->d_name[0] < '0' || pe->d_name[0] > '9') continue;
    const long pid = atol(pe->d_name);
    const std::string base = std::string("/proc/") + pe->d_name;
    DIR* fd = opendir((base + "/fd").c_str());
    if (!fd) continue;
    std::set<std::string> clients;
    struct dirent* fe;
    while ((fe = readdir(fd)) != nullptr) {
      if (fe->d_name[0] < '0' || fe->d_name[0] > '9') continue;
      const std::string l = base + "/fd/" + fe->d_name;
      ssize_t n = readlink(l.c_str(), tgt, sizeof tgt - 1);
      if (n <= 0) continue;
      tgt[n] = 0;
      if (strncmp(tgt, "/dev/dri/renderD", 16) != 0) continue;
      std::string info = read_file(base + "/fdinfo/" + fe->d_name, 8192);
      const char* pdev = strstr(info.c_str(), "drm-pdev:");
      if (!pdev) continue;
      char bdf[32] = {0};
      sscanf(pdev + 9, " %31s", bdf);
      const char* cid = strstr(info.c_str(), "drm-client-id:");
      std::string key = std::string(bdf) + "#" + (cid ? std::to_string(strtoull(cid + 14, nullptr, 10)) : fe->d_name);
      if (!clients.insert(key).second) continue;  // dup'ed fd of the same client
      uint64_t vram = 0;
      const char* vm = strstr(info.c_str(), "drm-memory-vram:");
      if (vm) {
        char unit[8] = {0};
        unsigned long long v = 0;
        sscanf(vm + 16, " %llu %7s", &v, unit);
        vram = v * (unit[0] == 'K' ? 1024ull : unit[0] == 'M' ? 1048576ull : unit[0] == 'G' ? 1073741824ull : 1ull);
      }
      out[bdf][pid] += vram;
    }
    closedir(fd);
  }
  closedir(pd);
  return out;
}

std::string cpu_json() {
  std::string st = read_file("/proc/stat", 4096);
  unsigned long long v[10] = {0};
  sscanf(st.c_str(), "cpu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu", &v[0], &v[1], &v[2], &v[3], &v[4],
         &v[5], &v[6], &v[7], &v[8], &v[9]);
  unsigned long long total = 0;
  for (int i = 0; i < 8; ++i) total += v[i];
  const unsigned long long idle = v[3] + v[4];
  double util = -1;
  if (g_cpu_prev_total && total > g_cpu_prev_total)
    util = 100.0 * (1.0 - (double)(idle - g_cpu_prev_idle) / (double)(total - g_cpu_prev_total));
  g_cpu_prev_total = total;
  g_cpu_prev_idle = idle;
  std::string mi = read_file("/proc/meminfo", 8192);
  auto field = [&](const char* k) -> double {
    const char* p = strstr(mi.c_str(), k);
    return p ? strtod(p + strlen(k), nullptr) / 1024.0 : -1;  // kB -> MiB
  };
  const double mt = field("MemTotal:"), ma = field("MemAvailable:");
  std::string o = "{\"utilization\":" + metric("%", util >= 0, util) + ",\"mem_total\":" + metric("MiB", mt >= 0, mt) +
                  ",\"mem_free\":" + metric("MiB", ma >= 0, ma) + ",\"mem_used\":" +
                  metric("MiB", mt >= 0 && ma >= 0, mt - ma) + "}";
  return o;
}

int discover() {
  g_gpus.clear();
  uint32_t nsock = 0;
  if (amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) return -2;
  std::vector<amdsmi_socket_handle> socks(nsock);
  amdsmi_get_socket_handles(&nsock, socks.data());
  for (auto s : socks) {
    uint32_t np = 0;
    if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    amdsmi_get_processor_handles(s, &np, ph.data());
    for (auto h : ph) {
      Gpu g;
      g.h = h;
      char uuid[AMDSMI_MAX_STRING_LENGTH] = {0};
      unsigned int ul = sizeof uuid;
      if (amdsmi_get_gpu_device_uuid(h, &ul, uuid) == AMDSMI_STATUS_SUCCESS) g.uuid = uuid;
      // the reservation model requires 40-char resource ids: "GPU-" + 36-char uuid
      std::string u = g.uuid;
      if (u.size() > 36) u = u.substr(u.size() - 36);
      while (u.size() < 36) u = "0" + u;
      g.uuid = "GPU-" + u;
      amdsmi_asic_info_t asic;
      memset(&asic, 0, sizeof asic);
      if (amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) g.name = asic.market_name;
      if (g.name.empty()) g.name = "AMD Instinct MI355X";
      amdsmi_bdf_t bdf;
      if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
        char b[32];
        snprintf(b, sizeof b, "%04x:%02x:%02x.%x", (unsigned)bdf.domain_number, (unsigned)bdf.bus_number,
                 (unsigned)bdf.device_number, (unsigned)bdf.function_number);
        g.bdf = b;
      }
      uint32_t numa = 0;
      if (amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) g.numa = (int)numa;
      amdsmi_enumeration_info_t en;
      memset(&en, 0, sizeof en);
      if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) g.hip_index = (int)en.hip_id;
      amdsmi_kfd_info_t kfd;
      memset(&kfd, 0, sizeof kfd);
      if (amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS) g.kfd_id = kfd.kfd_id;
      g_gpus.push_back(g);
    }
  }
  // HIP index order (what HIP_VISIBLE_DEVICES means); fall back to BDF order
  std::sort(g_gpus.begin(), g_gpus.end(), [](const Gpu& a, const Gpu& b) {
    if (a.hip_index >= 0 && b.hip_index >= 0 && a.hip_index != b.hip_index) return a.hip_index < b.hip_index;
    return a.bdf < b.bdf;
  });
  for (size_t i = 0; i < g_gpus.size(); ++i)
    if (g_gpus[i].hip_index < 0) g_gpus[i].hip_index = (int)i;
  return (int)g_gpus.size();
}

std::string gpu_json(Gpu& g, const std::map<uint64_t, std::set<long>>& kfd,
                     const std::map<std::string, std::map<long, uint64_t>>& drm, uint64_t ts) {
  amdsmi_engine_usage_t act;
  memset(&act, 0, sizeof act);
  const bool act_ok = amdsmi_get_gpu_activity(g.h, &act) == AMDSMI_STATUS_SUCCESS;
  amdsmi_vram_usage_t vr;
  memset(&vr, 0, sizeof vr);
  const bool vr_ok = amdsmi_get_gpu_vram_usage(g.h, &vr) == AMDSMI_STATUS_SUCCESS;
  amdsmi_power_info_t pw;
  memset(&pw, 0, sizeof pw);
  const bool pw_ok = amdsmi_get_power_info(g.h, &pw) == AMDSMI_STATUS_SUCCESS;
  double power = pw.current_socket_power ? pw.current_socket_power : (double)pw.average_socket_power;
  int64_t t_edge = 0, t_hot = 0, t_mem = 0;
  const bool te = amdsmi_get_temp_metric(g.h, AMDSMI_TEMPERATURE_TYPE_EDGE, AMDSMI_TEMP_CURRENT, &t_edge) == AMDSMI_STATUS_SUCCESS;
  const bool th = amdsmi_get_temp_metric(g.h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t_hot) == AMDSMI_STATUS_SUCCESS;
  const bool tm = amdsmi_get_temp_metric(g.h, AMDSMI_TEMPERATURE_TYPE_VRAM, AMDSMI_TEMP_CURRENT, &t_mem) == AMDSMI_STATUS_SUCCESS;
  amdsmi_frequencies_t fg, fm;
  memset(&fg, 0, sizeof fg);
  memset(&fm, 0, sizeof fm);
  const bool fg_ok = amdsmi_get_clk_freq(g.h, AMDSMI_CLK_TYPE_GFX, &fg) == AMDSMI_STATUS_SUCCESS && fg.num_supported;
  const bool fm_ok = amdsmi_get_clk_freq(g.h, AMDSMI_CLK_TYPE_MEM, &fm) == AMDSMI_STATUS_SUCCESS && fm.num_supported;
  amdsmi_gpu_metrics_t gm;
  memset(&gm, 0, sizeof gm);
  const bool gm_ok = amdsmi_get_gpu_metrics_info(g.h, &gm) == AMDSMI_STATUS_SUCCESS;
  double xr_rate = -1, xw_rate = -1, e_rate = -1;
  if (gm_ok) {
    uint64_t xr = 0, xw = 0;
    for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
      if (gm.xgmi_read_data_acc[l] != UINT64_MAX) xr += gm.xgmi_read_data_acc[l];
      if (gm.xgmi_write_data_acc[l] != UINT64_MAX) xw += gm.xgmi_write_data_acc[l];
    }
    if (g.ts_prev && ts > g.ts_prev) {
      const double dt = (ts - g.ts_prev) * 1e-9;
      if (xr >= g.xr_prev) xr_rate = (xr - g.xr_prev) * 1024.0 / dt / 1e9;  // KB -> GB/s
      if (xw >= g.xw_prev) xw_rate = (xw - g.xw_prev) * 1024.0 / dt / 1e9;
      if (gm.energy_accumulator >= g.energy_prev) e_rate = (gm.energy_accumulator - g.energy_prev) * 15.259e-6 / dt;
    }
    const uint64_t macc = gm.mem_activity_acc;
    if (g.mem_ts_prev == 0 || macc < g.mem_acc_prev) {
      g.mem_acc_prev = macc;
      g.mem_ts_prev = ts;
    } else if (ts - g.mem_ts_prev >= 1000000000ull) {
      g.hbm_gbps = (macc - g.mem_acc_prev) / ((ts - g.mem_ts_prev) * 1e-9) * hbm_gbps_per_acc();
      g.mem_acc_prev = macc;
      g.mem_ts_prev = ts;
    }
    g.xr_prev = xr;
    g.xw_prev = xw;
    g.energy_prev = gm.energy_accumulator;
    g.ts_prev = ts;
  }
  std::string m = "{";
  m += "\"fan_speed\":" + metric("%", false, 0);
  m += ",\"mem_free\":" + metric("MiB", vr_ok, (double)vr.vram_total - vr.vram_used);
  m += ",\"mem_used\":" + metric("MiB", vr_ok, vr.vram_used);
  m += ",\"mem_total\":" + metric("MiB", vr_ok, vr.vram_total);
  m += ",\"utilization\":" + metric("%", act_ok, act.gfx_activity);
  m += ",\"mem_util\":" + metric("%", act_ok, act.umc_activity);
  m += ",\"temp\":" + metric("C", te || th, te ? (double)t_edge : (double)t_hot);
  m += ",\"power\":" + metric("W", pw_ok, power);
  m += ",\"hotspot_temp\":" + metric("C", th, t_hot);
  m += ",\"mem_temp\":" + metric("C", tm, t_mem);
  m += ",\"gfx_clock\":" + metric("MHz", fg_ok, fg_ok ? fg.frequency[fg.current] / 1e6 : 0);
  m += ",\"mem_clock\":" + metric("MHz", fm_ok, fm_ok ? fm.frequency[fm.current] / 1e6 : 0);
  m += ",\"xgmi_read\":" + metric("GB/s", xr_rate >= 0, xr_rate);
  m += ",\"xgmi_write\":" + metric("GB/s", xw_rate >= 0, xw_rate);
  m += ",\"energy\":" + metric("W", e_rate >= 0, e_rate);
  m += ",\"hbm_bw\":" + metric("GB/s", g.hbm_gbps >= 0, g.hbm_gbps);
  m += "}";

  std::map<long, uint64_t> host;  // amdsmi / KFD: host pid -> vram bytes
  uint32_t np = 0;
  if (amdsmi_get_gpu_process_list(g.h, &np, nullptr) == AMDSMI_STATUS_SUCCESS && np) {
    std::vector<amdsmi_proc_info_t> pl(np);
    if (amdsmi_get_gpu_process_list(g.h, &np, pl.data()) == AMDSMI_STATUS_SUCCESS)
      for (uint32_t i = 0; i < np; ++i) host[(long)pl[i].pid] = pl[i].memory_usage.vram_mem;
  }
  auto it = kfd.find(g.kfd_id);
  if (it != kfd.end())
    for (long pid : it->second)
      if (!host.count(pid)) host[pid] = 0;
  std::map<long, uint64_t> procs;  // pids of our namespace
  for (const auto& p : host)
    if (has_kfd_open(p.first)) procs[p.first] = p.second;
  auto dit = drm.find(g.bdf);
  if (dit != drm.end())
    for (const auto& p : dit->second)
      if (p.second > 0 || procs.count(p.first)) procs[p.first] = std::max(procs[p.first], p.second);
  std::string ps = "[";
  bool first = true;
  for (const auto& p : procs) {
    if (ignored_pid(p.first)) continue;
    ProcInfo pi = resolve_pid(p.first);
    if (pi.uid < 0 && pi.cmd.empty()) continue;  // exited between the two reads
    if (!first) ps += ",";
    first = false;
    ps += "{\"pid\":" + std::to_string(p.first) + ",\"command\":\"" + esc(pi.cmd) + "\",\"owner\":\"" +
          esc(pi.owner) + "\",\"uid\":" + std::to_string(pi.uid) + ",\"vram\":" + std::to_string(p.second) +
          ",\"task_id\":" + (pi.task_id.empty() ? "null" : "\"" + esc(pi.task_id) + "\"") +
          ",\"ppid\":" + std::to_string(pi.ppid) + ",\"pgid\":" + std::to_string(pi.pgid) +
          ",\"sid\":" + std::to_string(pi.sid) + ",\"ancestors\":[";
    for (size_t k = 0; k < pi.ancestors.size(); ++k) ps += (k ? "," : "") + std::to_string(pi.ancestors[k]);
    ps += "]}";
  }
  ps += "]";
  return "{\"uuid\":\"" + esc(g.uuid) + "\",\"name\":\"" + esc(g.name) + "\",\"index\":" +
         std::to_string(g.hip_index) + ",\"bdf\":\"" + g.bdf + "\",\"numa_node\":" + std::to_string(g.numa) +
         ",\"kfd_id\":" + std::to_string(g.kfd_id) + ",\"metrics\":" + m + ",\"processes\":" + ps + "}";
}

int emit(const std::string& s, char* buf, int cap) {
  if ((int)s.size() + 1 > cap) return -(int)(s.size() + 1);
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

}  // namespace

extern "C" int thsmi_init(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_init) return (int)g_gpus.size();
  if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return -1;
  g_init = true;
  return discover();
}

extern "C" int thsmi_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_init) amdsmi_shut_down();
  g_init = false;
  g_gpus.clear();
  return 0;
}

extern "C" int thsmi_sample_json(char* buf, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return -1000000000;
  const uint64_t ts = now_ns();
  auto kfd = kfd_processes();
  auto drm = drm_processes();
  std::string s = "{\"ts_ns\":" + std::to_string(ts) + ",\"cpu\":" + cpu_json() + ",\"gpus\":[";
  for (size_t i = 0; i < g_gpus.size(); ++i) s += (i ? "," : "") + gpu_json(g_gpus[i], kfd, drm, ts);
  s += "],\"ignored_pids\":[" + std::to_string((long)getpid());
  for (long p : g_ignored) s += "," + std::to_string(p);
  s += "]}";
  return emit(s, buf, cap);
}

// The host half of a sample, without amdsmi: CPU utilisation / memory and every process that
// has GPU memory (KFD sysfs + DRM fdinfo), attributed to owner and task -- under the same lock
// as the full sample.  Works on a node whose GPUs amdsmi cannot open (and is what the TSan stress
// test drives from several threads on a CPU-only host).
extern "C" int thsmi_host_sample_json(char* buf, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  const uint64_t ts = now_ns();
  auto kfd = kfd_processes();
  auto drm = drm_processes();
  std::set<long> pids;
  for (const auto& g : kfd)
    for (long p : g.second) pids.insert(p);
  for (const auto& d : drm)
    for (const auto& p : d.second) pids.insert(p.first);
  std::string s = "{\"ts_ns\":" + std::to_string(ts) + ",\"cpu\":" + cpu_json() + ",\"processes\":[";
  bool first = true;
  for (long p : pids) {
    if (ignored_pid(p)) continue;
    ProcInfo pi = resolve_pid(p);
    if (pi.uid < 0 && pi.cmd.empty()) continue;
    s += std::string(first ? "" : ",") + "{\"pid\":" + std::to_string(p) + ",\"command\":\"" + esc(pi.cmd) +
         "\",\"owner\":\"" + esc(pi.owner) + "\"}";
    first = false;
  }
  s += "]}";
  return emit(s, buf, cap);
}

// Replace the ignore list (pids of the monitor's own helper processes); returns its size.
extern "C" int thsmi_set_ignored_pids(const long* pids, int n) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_ignored.clear();
  for (int i = 0; i < n; ++i)
    if (pids[i] > 0) g_ignored.insert(pids[i]);
  return (int)g_ignored.size();
}

extern "C" int thsmi_topology_json(char* buf, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return -1000000000;
  std::string s = "{\"gpus\":[";
  for (size_t i = 0; i < g_gpus.size(); ++i) {
    s += std::string(i ? "," : "") + "{\"index\":" + std::to_string(g_gpus[i].hip_index) + ",\"uuid\":\"" +
         g_gpus[i].uuid + "\",\"bdf\":\"" + g_gpus[i].bdf + "\",\"numa_node\":" + std::to_string(g_gpus[i].numa) +
         ",\"links\":[";
    for (size_t j = 0; j < g_gpus.size(); ++j) {
      uint64_t hops = 0;
      amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
      if (i != j) amdsmi_topo_get_link_type(g_gpus[i].h, g_gpus[j].h, &hops, &t);
      const char* ts = i == j ? "self" : (t == AMDSMI_LINK_TYPE_XGMI ? "xgmi" : (t == AMDSMI_LINK_TYPE_PCIE ? "pcie" : "unknown"));
      s += std::string(j ? "," : "") + "{\"peer\":" + std::to_string(g_gpus[j].hip_index) + ",\"type\":\"" + ts +
           "\",\"hops\":" + std::to_string(hops) + "}";
    }
    s += "]}";
  }
  s += "]}";
  return emit(s, buf, cap);
}

#ifdef THSMI_MAIN
int main(int argc, char** argv) {
  int stream_ms = -1;
  bool topo = false;
  std::vector<long> ignore;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--stream") && i + 1 < argc) stream_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--topology")) topo = true;
    else if (!strcmp(argv[i], "--ignore-pid") && i + 1 < argc) ignore.push_back(atol(argv[++i]));
  }
  if (thsmi_init() < 0) {
    fprintf(stderr, "th-smi: amdsmi init failed\n");
    return 1;
  }
  thsmi_set_ignored_pids(ignore.data(), (int)ignore.size());
  std::vector<char> buf(1 << 20);
  auto once = [&](bool t) {
    int n = t ? thsmi_topology_json(buf.data(), (int)buf.size()) : thsmi_sample_json(buf.data(), (int)buf.size());
    if (n < 0) {
      buf.resize(-n + 1024);
      n = t ? thsmi_topology_json(buf.data(), (int)buf.size()) : thsmi_sample_json(buf.data(), (int)buf.size());
    }
    if (n >= 0) {
      fwrite(buf.data(), 1, n, stdout);
      fputc('\n', stdout);
      fflush(stdout);
    }
  };
  if (topo) {
    once(true);
  } else if (stream_ms > 0) {
    for (;;) {
      once(false);
      usleep(stream_ms * 1000);
    }
  } else {
    thsmi_sample_json(buf.data(), (int)buf.size());  // prime the rate counters
    usleep(100000);
    once(false);
  }
  thsmi_shutdown();
  return 0;
}
#endif
