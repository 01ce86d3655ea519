// Which GPU agents the in-task HBM counter tool (th_hbm_tool.cpp) samples.  Header-only and free
// of rocprofiler types so tests/test_hbm_select.py can compile it with the host compiler alone.
//
// The tool sees every GPU ROCr exposes, sorted by KFD node id (= HIP's physical order).  A task
// only drives the GPUs HIP_VISIBLE_DEVICES leaves it (the daemon sets it from the reservation), and
// a torchrun rank drives the LOCAL_RANK-th of those.  Counting a GPU the task never touches would
// report ~0 bytes for it (the counters only see the counting process's own traffic) and hide the
// GPU it really uses.
#pragma once
#include <stdlib.h>

#include <string>
#include <vector>

namespace th_hbm {

// Indices (into the node-id-sorted agent list of size n) that the task can use, in HIP order.
// hip_visible: the HIP_VISIBLE_DEVICES value (nullptr = unset); entries that are not plain indices
// (UUIDs) make the filter unknowable, so every agent is kept.
inline std::vector<int> visible_agents(int n, const char* hip_visible) {
  std::vector<int> all;
  for (int i = 0; i < n; ++i) all.push_back(i);
  if (!hip_visible || !*hip_visible) return all;
  std::vector<int> out;
  const std::string s(hip_visible);
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string tok = s.substr(i, j - i);
    if (!tok.empty()) {
      char* end = nullptr;
      const long v = strtol(tok.c_str(), &end, 10);
      if (end == tok.c_str() || *end != '\0') return all;  // UUID or garbage: cannot map
      if (v >= 0 && v < n) out.push_back((int)v);
    }
    i = j + 1;
  }
  return out;
}

// The agents to sample: the rank's own GPU under torchrun (local_rank set, all_agents false),
// else every GPU visible to the task.
inline std::vector<int> select_agents(int n, const char* hip_visible, const char* local_rank, bool all_agents) {
  std::vector<int> vis = visible_agents(n, hip_visible);
  if (local_rank && *local_rank && !all_agents && !vis.empty()) {
    const int r = atoi(local_rank);
    return {vis[(size_t)(r < 0 ? 0 : r) % vis.size()]};
  }
  return vis;
}

}  // namespace th_hbm
