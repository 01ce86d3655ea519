// A rocprofiler-sdk tool library that registers and does nothing: the floor of what loading any
// tool through ROCP_TOOL_LIBRARIES costs a process (scripts/gpu_r05_startup.sh).
//   g++ -O2 -std=c++17 -fPIC -shared -I/opt/rocm/include scripts/null_rocp_tool.cpp -L/opt/rocm/lib -lrocprofiler-sdk -o scripts/libnulltool.so
#include <rocprofiler-sdk/registration.h>

extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                                      rocprofiler_client_id_t* id) {
  id->name = "th-null";
  return nullptr;
}
