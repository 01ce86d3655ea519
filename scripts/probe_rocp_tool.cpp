// rocprofiler-sdk tool libraries that isolate where the in-task HBM tool's startup cost comes from
// (scripts/gpu_r05_startup.sh).  PROBE_LEVEL:
//   1  returns a configuration whose init does nothing (rocprofiler-sdk active, no context)
//   2  init creates one context + buffer per GPU agent
//   3  as 2, plus the device counting service configured on each (no counter config yet)
//   4  init only queries the GPU agents
//   5  init queries the agents and creates one context per GPU agent (no buffer)
//   g++ -O2 -std=c++17 -fPIC -shared -DPROBE_LEVEL=N -I/opt/rocm/include scripts/probe_rocp_tool.cpp \
//       -L/opt/rocm/lib -lrocprofiler-sdk -o scripts/libprobetoolN.so
#include <rocprofiler-sdk/agent.h>
#include <rocprofiler-sdk/buffer.h>
#include <rocprofiler-sdk/context.h>
#include <rocprofiler-sdk/device_counting_service.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/registration.h>

#include <stdio.h>
#include <time.h>

#include <vector>

namespace {
double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}
double g_t_configure = 0;
int init(rocprofiler_client_finalize_t, void*) {
  const double t_init = now_s();
  fprintf(stderr, "[probe-tool] configure -> init %.3f s\n", t_init - g_t_configure);
  if (PROBE_LEVEL < 2) return 0;
  constexpr bool kContexts = PROBE_LEVEL != 4, kBuffers = PROBE_LEVEL == 2 || PROBE_LEVEL == 3;
  std::vector<rocprofiler_agent_v0_t> agents;
  rocprofiler_query_available_agents(
      ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
        for (size_t i = 0; i < n; ++i) {
          const auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
          if (a->type == ROCPROFILER_AGENT_TYPE_GPU) static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud)->push_back(*a);
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), &agents);
  fprintf(stderr, "[probe-tool] agent query %.3f s, %zu GPU agents\n", now_s() - t_init, agents.size());
  for (const auto& a : agents) {
    rocprofiler_context_id_t ctx{};
    rocprofiler_buffer_id_t buf{};
    if (!kContexts) continue;
    if (rocprofiler_create_context(&ctx) != ROCPROFILER_STATUS_SUCCESS) continue;
    if (!kBuffers) continue;
    rocprofiler_create_buffer(ctx, 4096, 2048, ROCPROFILER_BUFFER_POLICY_LOSSLESS,
                              [](rocprofiler_context_id_t, rocprofiler_buffer_id_t, rocprofiler_record_header_t**,
                                 size_t, void*, uint64_t) {},
                              nullptr, &buf);
    if (PROBE_LEVEL >= 3)
      rocprofiler_configure_device_counting_service(
          ctx, buf, a.id,
          [](rocprofiler_context_id_t, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t, void*) {},
          nullptr);
  }
  return 0;
}
void fini(void*) {}
}  // namespace

extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                                      rocprofiler_client_id_t* id) {
  id->name = "th-probe-tool";
  g_t_configure = now_s();
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &init, &fini, nullptr};
  return &cfg;
}
