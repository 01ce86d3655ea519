// As probe_rocp_tool.cpp level 4 (init queries the GPU agents), but the tool has no DT_NEEDED entry on
// librocprofiler-sdk: the one API call is resolved with dlsym(RTLD_DEFAULT) from the SDK copy that is already
// loaded when rocprofiler_configure runs.  Does rocprofiler-sdk then skip its scan of every loaded library?
//   g++ -O2 -std=c++17 -fPIC -shared -I/opt/rocm/include scripts/probe_rocp_tool_dl.cpp -ldl -o scripts/libprobetool6.so
#include <dlfcn.h>
#include <rocprofiler-sdk/agent.h>
#include <rocprofiler-sdk/registration.h>
#include <stdio.h>

namespace {
using query_fn = decltype(&rocprofiler_query_available_agents);
int init(rocprofiler_client_finalize_t, void*) {
  auto q = reinterpret_cast<query_fn>(dlsym(RTLD_DEFAULT, "rocprofiler_query_available_agents"));
  size_t n = 0;
  if (q)
    q(ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** arr, size_t k, void* ud) {
        *static_cast<size_t*>(ud) += k;
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), &n);
  fprintf(stderr, "[probe-tool-dl] resolved=%d agents=%zu\n", q != nullptr, n);
  return 0;
}
void fini(void*) {}
}  // namespace

extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                                      rocprofiler_client_id_t* id) {
  id->name = "th-probe-tool-dl";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &init, &fini, nullptr};
  return &cfg;
}
