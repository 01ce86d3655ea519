// TSan / ASan stress driver for libthsmi (SURVEY §5 race-detection row; round-2 verdict item 8).
// The daemon calls libthsmi from several threads (monitoring loop, API topology reads, the
// backend updating its ignore list); this driver does the same at a much higher rate:
//   * 2 threads: thsmi_host_sample_json (CPU + KFD/DRM process scan, no GPU needed),
//   * 1 thread:  thsmi_sample_json + thsmi_topology_json (full sample when amdsmi is up),
//   * 1 thread:  thsmi_set_ignored_pids with a changing list.
// Linked straight with thsmi.cpp and built -fsanitize=thread (th-smi-stress-tsan) or
// address,undefined; exits 0 when every call returned and the JSON it got was complete.
//   thsmi-stress [--iters N]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

extern "C" int thsmi_init(void);
extern "C" int thsmi_shutdown(void);
extern "C" int thsmi_sample_json(char* buf, int cap);
extern "C" int thsmi_host_sample_json(char* buf, int cap);
extern "C" int thsmi_topology_json(char* buf, int cap);
extern "C" int thsmi_set_ignored_pids(const long* pids, int n);

namespace {
std::atomic<int> g_bad{0};

void check_json(const char* what, const std::vector<char>& b, int n) {
  if (n < 2 || b[0] != '{' || b[n - 1] != '}') {
    fprintf(stderr, "%s: bad output (%d bytes)\n", what, n);
    g_bad++;
  }
}
}  // namespace

int main(int argc, char** argv) {
  int iters = 200;
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
  const int ngpu = thsmi_init();  // < 0 on a host without usable GPUs: the host half still runs
  std::vector<std::thread> th;
  for (int t = 0; t < 2; ++t)
    th.emplace_back([&] {
      std::vector<char> b(1 << 20);
      for (int i = 0; i < iters; ++i) check_json("host", b, thsmi_host_sample_json(b.data(), (int)b.size()));
    });
  th.emplace_back([&] {
    std::vector<char> b(1 << 20);
    for (int i = 0; i < iters / 4; ++i) {
      if (ngpu < 0) break;
      check_json("sample", b, thsmi_sample_json(b.data(), (int)b.size()));
      check_json("topology", b, thsmi_topology_json(b.data(), (int)b.size()));
    }
  });
  th.emplace_back([&] {
    for (int i = 0; i < iters; ++i) {
      std::vector<long> pids;
      for (int k = 0; k < 1 + i % 7; ++k) pids.push_back(100000 + i + k);
      thsmi_set_ignored_pids(pids.data(), (int)pids.size());
    }
  });
  for (auto& t : th) t.join();
  thsmi_shutdown();
  printf("{\"thsmi_stress\":1,\"gpus\":%d,\"iters\":%d,\"bad\":%d}\n", ngpu, iters, g_bad.load());
  return g_bad.load() == 0 ? 0 : 1;
}
