// th-probe: the per-node device-probe agent.  Runs the gfx950 th-probe kernel
// (ops/csrc/probe.hip) on EVERY GPU of the node at a low duty cycle and streams one JSON line per
// period, which the daemon's GpuProbe turns into per-GPU `mfma_busy` / `hbm_contention`.
//
// It is a process of its own, not code inside the daemon: the daemon never opens /dev/kfd or
// holds a HIP context (so it cannot wedge on a GPU and keeps answering the API), and the agent's
// pid is handed to libthsmi's ignore list so it is never reported as a tenant of the GPUs it
// probes (the reference filtered its own non-tenant processes too:
// tensorhive/core/managers/InfrastructureManager.py:57,70-76).
//
//   th-probe [--period-ms 1000] [--count N (0 = forever)] [--wg 8] [--iters 512]
//            [--slice-kb 1024] [--devices all|0,1,..]
//
// Output, one line per period:
//   {"ts_ns":..,"period_ms":..,"gpus":[{"hip":0,"bdf":"0000:05:00.0","latency_us":..,
//     "wg":[[xcc,mfma_us,hbm_us,hbm_GBps],..]}, ..]}
// Each period launches the probe on every device first and then collects them all, so the
// samples of one line are taken at the same moment.  The agent exits when its parent dies
// (PR_SET_PDEATHSIG), on SIGTERM/SIGINT, or when stdout is closed; every launched probe is
// collected before exit, so no grid is left running.
#include <ctype.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "probe.hip"

namespace {
volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

unsigned long long now_ns() {
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  return (unsigned long long)t.tv_sec * 1000000000ull + t.tv_nsec;
}

std::vector<int> parse_devices(const char* s, int n) {
  std::vector<int> out;
  if (!s || !strcmp(s, "all")) {
    for (int i = 0; i < n; ++i) out.push_back(i);
    return out;
  }
  const std::string str(s);
  size_t i = 0;
  while (i < str.size()) {
    size_t j = str.find(',', i);
    if (j == std::string::npos) j = str.size();
    const int d = atoi(str.substr(i, j - i).c_str());
    if (d >= 0 && d < n) out.push_back(d);
    i = j + 1;
  }
  return out;
}
}  // namespace

int main(int argc, char** argv) {
  int period_ms = 1000, count = 0, wg = 8, iters = 512, slice_kb = 1024;
  const char* devs = "all";
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--period-ms") && i + 1 < argc) period_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--count") && i + 1 < argc) count = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--wg") && i + 1 < argc) wg = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--slice-kb") && i + 1 < argc) slice_kb = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--devices") && i + 1 < argc) devs = argv[++i];
    else {
      fprintf(stderr, "usage: th-probe [--period-ms MS] [--count N] [--wg N] [--iters N] [--slice-kb KB] "
                      "[--devices all|i,j]\n");
      return 2;
    }
  }
  if (wg < 1 || wg > 1024 || iters < 1 || iters > 65536 || slice_kb < 1 || slice_kb > 65536 || period_ms < 1) {
    fprintf(stderr, "th-probe: argument out of range\n");
    return 2;
  }
  prctl(PR_SET_PDEATHSIG, SIGTERM);
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  signal(SIGPIPE, on_signal);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    printf("{\"error\":\"no HIP device\"}\n");
    return 1;
  }
  std::vector<int> devices;
  std::vector<std::string> bdfs;
  for (int d : parse_devices(devs, n)) {
    const int rc = th_probe_init(d, wg, slice_kb);
    if (rc != 0) {
      fprintf(stderr, "th-probe: device %d: init failed (%d)\n", d, rc);
      continue;
    }
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, d) != hipSuccess) bus[0] = 0;
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    devices.push_back(d);
    bdfs.push_back(bus);
  }
  if (devices.empty()) {
    printf("{\"error\":\"no device could be probed\"}\n");
    return 1;
  }
  std::vector<double> out((size_t)wg * 5);
  std::vector<int> launched(devices.size());
  for (int it = 0; !g_stop && (count == 0 || it < count); ++it) {
    const unsigned long long t0 = now_ns();
    for (size_t k = 0; k < devices.size(); ++k) launched[k] = th_probe_launch(devices[k], wg, iters) == 0;
    std::string line = "{\"ts_ns\":" + std::to_string(t0) + ",\"period_ms\":" + std::to_string(period_ms) + ",\"gpus\":[";
    bool first = true;
    for (size_t k = 0; k < devices.size(); ++k) {
      if (!launched[k]) continue;
      const int got = th_probe_collect(devices[k], out.data());
      if (got <= 0) continue;
      char head[160];
      snprintf(head, sizeof head, "%s{\"hip\":%d,\"bdf\":\"%s\",\"latency_us\":%.2f,\"wg\":[", first ? "" : ",",
               devices[k], bdfs[k].c_str(), th_probe_last_latency_us(devices[k]));
      line += head;
      for (int i = 0; i < got; ++i) {
        char row[128];
        snprintf(row, sizeof row, "%s[%d,%.2f,%.2f,%.1f]", i ? "," : "", (int)out[5 * i], out[5 * i + 1],
                 out[5 * i + 2], out[5 * i + 3]);
        line += row;
      }
      line += "]}";
      first = false;
    }
    line += "]}\n";
    if (fputs(line.c_str(), stdout) < 0 || fflush(stdout) != 0) break;
    const long spent_us = (long)((now_ns() - t0) / 1000ull);
    long left_us = (long)period_ms * 1000 - spent_us;
    while (left_us > 0 && !g_stop) {  // short sleeps: a stop request is honoured within 50 ms
      const long s = left_us > 50000 ? 50000 : left_us;
      usleep((useconds_t)s);
      left_us -= s;
    }
  }
  for (int d : devices) th_probe_shutdown(d);
  return 0;
}
