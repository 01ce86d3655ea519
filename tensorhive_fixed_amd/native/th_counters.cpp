// th-counters: device-wide hardware counter sampler for MI355X nodes.
//
// Uses the rocprofiler-sdk DEVICE COUNTING service: counters are collected for the whole GPU
// (every process's kernels), not per dispatch, so the daemon can show what a reserved GPU is
// really doing -- MFMA activity, HBM traffic, busy cycles -- next to the amdsmi metrics of
// libthsmi.  The reference had nothing comparable (nvidia-smi utilisation only,
// tensorhive/core/monitors/GPUMonitor.py:20-60).
//
// The tool registers itself with rocprofiler (rocprofiler_force_configure) and then initialises
// HSA; every sample starts the per-agent contexts, waits one window, reads the accumulated
// counter records, stops the contexts, and sums the records of each counter over all its
// dimension instances (XCC / SE / channel).  Output: one JSON line per sample,
//   {"ts_ns":..,"window_ms":..,"gpus":[{"kfd_id":..,"bdf":"0000:05:00.0","counters":{NAME:value,..}}]}
//
//   th-counters [--list] [--window MS] [--period MS] [--count N] [--counters A,B,C]
//
// --list prints the counters the device supports (one per line).  Unsupported names given to
// --counters are skipped; if the hardware cannot schedule the whole set in one pass the last
// counters are dropped until it can (reported in "dropped").
#include <hsa/hsa.h>
#include <rocprofiler-sdk/agent.h>
#include <rocprofiler-sdk/buffer.h>
#include <rocprofiler-sdk/context.h>
#include <rocprofiler-sdk/counter_config.h>
#include <rocprofiler-sdk/counters.h>
#include <rocprofiler-sdk/device_counting_service.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/internal_threading.h>
#include <rocprofiler-sdk/registration.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

// declared in rocprofiler.h, whose umbrella includes pull in the HIP/RCCL tracing headers
extern "C" const char* rocprofiler_get_status_string(rocprofiler_status_t status);

namespace {

struct Sampler {
  rocprofiler_agent_v0_t agent{};
  rocprofiler_context_id_t ctx{};
  rocprofiler_buffer_id_t buf{};
  rocprofiler_counter_config_id_t config{.handle = 0};
  size_t n_records = 0;
  std::unordered_map<std::string, rocprofiler_counter_id_t> supported;
  std::map<uint64_t, std::string> id_to_name;
  std::vector<std::string> active, dropped;
  bool ok = false;
};

std::vector<Sampler*> g_samplers;
rocprofiler_client_finalize_t g_fini = nullptr;
rocprofiler_client_id_t* g_client = nullptr;
int g_init_status = 1;  // 1 = pending, 0 = ok, <0 = error

uint64_t now_ns() {
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + t.tv_nsec;
}

std::string bdf_of(const rocprofiler_agent_v0_t& a) {
  char b[32];
  snprintf(b, sizeof b, "%04x:%02x:%02x.%x", a.domain, (a.location_id >> 8) & 0xff, (a.location_id >> 3) & 0x1f,
           a.location_id & 0x7);
  return b;
}

size_t instances_of(rocprofiler_counter_id_t c) {
  rocprofiler_counter_info_v1_t info;
  if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) != ROCPROFILER_STATUS_SUCCESS)
    return 0;
  return info.dimensions_instances_count;
}

void load_supported(Sampler* s) {
  std::vector<rocprofiler_counter_id_t> ids;
  rocprofiler_iterate_agent_supported_counters(
      s->agent.id,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
        v->insert(v->end(), c, c + n);
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &ids);
  for (auto id : ids) {
    rocprofiler_counter_info_v0_t info;
    if (rocprofiler_query_counter_info(id, ROCPROFILER_COUNTER_INFO_VERSION_0, &info) == ROCPROFILER_STATUS_SUCCESS) {
      s->supported.emplace(info.name, id);
      s->id_to_name.emplace(id.handle, info.name);
    }
  }
}

// Build one counter config from `want`, dropping trailing counters the hardware cannot co-schedule.
void configure_counters(Sampler* s, const std::vector<std::string>& want) {
  std::vector<std::string> names;
  for (const auto& w : want) {
    if (s->supported.count(w)) names.push_back(w);
    else s->dropped.push_back(w);
  }
  while (!names.empty()) {
    std::vector<rocprofiler_counter_id_t> ids;
    size_t n = 0;
    for (const auto& nm : names) {
      ids.push_back(s->supported[nm]);
      n += instances_of(s->supported[nm]);
    }
    rocprofiler_counter_config_id_t cfg{};
    if (rocprofiler_create_counter_config(s->agent.id, ids.data(), ids.size(), &cfg) == ROCPROFILER_STATUS_SUCCESS) {
      s->config = cfg;
      s->n_records = n;
      s->active = names;
      return;
    }
    s->dropped.push_back(names.back());
    names.pop_back();
  }
}

int tool_init(rocprofiler_client_finalize_t fini, void*) {
  g_fini = fini;
  std::vector<rocprofiler_agent_v0_t> agents;
  rocprofiler_query_available_agents(
      ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
        for (size_t i = 0; i < n; ++i) {
          const auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
          if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a);
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), &agents);
  for (const auto& a : agents) {
    auto* s = new Sampler();
    s->agent = a;
    if (rocprofiler_create_context(&s->ctx) != ROCPROFILER_STATUS_SUCCESS) continue;
    if (rocprofiler_create_buffer(
            s->ctx, 4096, 2048, ROCPROFILER_BUFFER_POLICY_LOSSLESS,
            [](rocprofiler_context_id_t, rocprofiler_buffer_id_t, rocprofiler_record_header_t**, size_t, void*,
               uint64_t) {},
            nullptr, &s->buf) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    auto st = rocprofiler_configure_device_counting_service(
        s->ctx, s->buf, a.id,
        [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set_config,
           void* ud) {
          auto* smp = static_cast<Sampler*>(ud);
          if (smp->config.handle != 0) set_config(ctx, smp->config);
        },
        s);
    if (st != ROCPROFILER_STATUS_SUCCESS) {
      fprintf(stderr, "th-counters: device counting service unavailable: %s\n", rocprofiler_get_status_string(st));
      continue;
    }
    load_supported(s);
    s->ok = true;
    g_samplers.push_back(s);
  }
  g_init_status = g_samplers.empty() ? -1 : 0;
  return 0;
}

void tool_fini(void*) {
  for (auto* s : g_samplers) rocprofiler_stop_context(s->ctx);
}

extern "C" rocprofiler_tool_configure_result_t* th_configure(uint32_t, const char*, uint32_t,
                                                             rocprofiler_client_id_t* id) {
  id->name = "th-counters";
  g_client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

std::vector<std::string> split(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) out.push_back(s.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

}  // namespace

int main(int argc, char** argv) {
  bool list = false;
  int window_ms = 100, period_ms = 1000, count = 1;
  // default set: the counters that read correctly in device-counting mode on gfx950
  // (profiles/r01_counters: TCC/EA request counters and SQ_WAVES stay ~0 there)
  std::vector<std::string> want = {"GRBM_GUI_ACTIVE", "GRBM_COUNT", "SQ_VALU_MFMA_BUSY_CYCLES",
                                   "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16",
                                   "SQ_INSTS_VALU_MFMA_MOPS_F8", "SQ_INSTS_VALU_MFMA_MOPS_F32"};
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--list")) list = true;
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) window_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--period") && i + 1 < argc) period_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--count") && i + 1 < argc) count = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--counters") && i + 1 < argc) want = split(argv[++i]);
    else {
      fprintf(stderr, "usage: th-counters [--list] [--window MS] [--period MS] [--count N(0=forever)] "
                      "[--counters A,B]\n");
      return 2;
    }
  }
  if (rocprofiler_force_configure(&th_configure) != ROCPROFILER_STATUS_SUCCESS) {
    fprintf(stderr, "th-counters: rocprofiler_force_configure failed\n");
    return 1;
  }
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    fprintf(stderr, "th-counters: hsa_init failed\n");
    return 1;
  }
  if (g_init_status != 0) {
    printf("{\"error\":\"no GPU agent with a usable device counting service\"}\n");
    return 1;
  }
  if (list) {
    for (auto* s : g_samplers) {
      std::vector<std::string> names;
      for (const auto& kv : s->supported) names.push_back(kv.first);
      std::sort(names.begin(), names.end());
      for (const auto& n : names) printf("%s %s\n", bdf_of(s->agent).c_str(), n.c_str());
    }
    return 0;
  }
  for (auto* s : g_samplers) configure_counters(s, want);
  for (int it = 0; count == 0 || it < count; ++it) {
    if (it) usleep((useconds_t)std::max(0, period_ms - window_ms) * 1000);
    for (auto* s : g_samplers)
      if (s->config.handle) rocprofiler_start_context(s->ctx);
    const uint64_t t0 = now_ns();
    usleep((useconds_t)window_ms * 1000);
    std::string line = "{\"ts_ns\":" + std::to_string(t0) + ",\"window_ms\":" + std::to_string(window_ms) +
                       ",\"gpus\":[";
    bool first = true;
    for (auto* s : g_samplers) {
      std::map<std::string, double> sums;
      std::string err;
      if (s->config.handle) {
        std::vector<rocprofiler_counter_record_t> rec(s->n_records + 64);
        size_t n = rec.size();
        auto st = rocprofiler_sample_device_counting_service(s->ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, rec.data(), &n);
        if (st == ROCPROFILER_STATUS_SUCCESS) {
          for (size_t r = 0; r < n; ++r) {
            rocprofiler_counter_id_t cid{};
            rocprofiler_query_record_counter_id(rec[r].id, &cid);
            auto itn = s->id_to_name.find(cid.handle);
            if (itn != s->id_to_name.end()) sums[itn->second] += rec[r].counter_value;
          }
        } else {
          err = rocprofiler_get_status_string(st);
        }
        rocprofiler_stop_context(s->ctx);
      }
      line += std::string(first ? "" : ",") + "{\"kfd_id\":" + std::to_string(s->agent.gpu_id) +
              ",\"bdf\":" + json_str(bdf_of(s->agent)) + ",\"xcc\":" + std::to_string(s->agent.num_xcc) +
              ",\"cu\":" + std::to_string(s->agent.cu_count) + ",\"counters\":{";
      bool f2 = true;
      for (const auto& kv : sums) {
        char v[64];
        snprintf(v, sizeof v, "%.0f", kv.second);
        line += std::string(f2 ? "" : ",") + json_str(kv.first) + ":" + v;
        f2 = false;
      }
      line += "},\"dropped\":[";
      for (size_t d = 0; d < s->dropped.size(); ++d) line += (d ? "," : "") + json_str(s->dropped[d]);
      line += "]";
      if (!err.empty()) line += ",\"error\":" + json_str(err);
      line += "}";
      first = false;
    }
    line += "]}";
    printf("%s\n", line.c_str());
    fflush(stdout);
  }
  if (g_fini && g_client) g_fini(*g_client);
  hsa_shut_down();
  return 0;
}
