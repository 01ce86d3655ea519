// th-probe: low-duty-cycle device probe for MI355X contention telemetry.
//
// One 256-thread workgroup per XCD-slot (grid = 8 by default; the XCD each workgroup actually
// landed on is read from HW_REG_XCC_ID, placement is never assumed).  Each workgroup times
//   (1) a short chain of v_mfma_f32_32x32x16_bf16 on every wave (matrix-pipe availability), and
//   (2) a short non-temporal streaming read of its own HBM slice (memory-path availability)
// with s_memrealtime (100 MHz constant clock, immune to DVFS).  Per-wave timings are reduced
// through LDS (max over waves = the workgroup's phase time) and written to pinned host memory.
// The host compares against an idle-device baseline: mfma_busy ~ 1 - t_idle/t_now and
// hbm_bw_share ~ 1 - bw_now/bw_idle.  A probe costs tens of microseconds; at one probe per
// second the device-time budget is < 0.01 %.
//
// State is per HIP device (th_probe_init/launch/collect take the device index), so one process
// probes every GPU of a node: the `th-probe` agent (native/th_probe.hip) does exactly that, out of
// the daemon's process, and streams one JSON line per period.
#include "th_common.h"

typedef __bf16 bf16x8_p __attribute__((ext_vector_type(8)));
typedef float f32x16_p __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

__global__ __launch_bounds__(256) void th_probe_kernel(const float4v* __restrict__ hbm, long per_wg_vec,
                                                      int mfma_iters, unsigned long long* __restrict__ out,
                                                      float* __restrict__ sink) {
  __shared__ unsigned long long red[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bf16x8_p a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.001f * (lane + j));
    b[j] = (__bf16)(0.002f * (lane - j));
  }
  f32x16_p acc0 = f32x16_p(0.f), acc1 = f32x16_p(0.f);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < mfma_iters; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
  }
  asm volatile("s_nop 15" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const float4v* src = hbm + (long)blockIdx.x * per_wg_vec;
  float4v s = float4v(0.f);
  for (long i = threadIdx.x; i < per_wg_vec; i += blockDim.x) s += __builtin_nontemporal_load(src + i);
  float part = s[0] + s[1] + s[2] + s[3];
  part = wave_sum(part);
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    red[w][0] = t1 - t0;
    red[w][1] = t2 - t1;
  }
  // keep the MFMA chain and the loads alive
  if (acc0[0] + acc1[0] + part == 1234567.0f) sink[0] = acc0[1] + acc1[1] + part;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0, h = 0;
    for (int i = 0; i < 4; ++i) {
      m = red[i][0] > m ? red[i][0] : m;
      h = red[i][1] > h ? red[i][1] : h;
    }
    unsigned long long* o = out + 4 * blockIdx.x;
    o[0] = xcc_id();
    o[1] = m;
    o[2] = h;
    o[3] = (unsigned long long)per_wg_vec * 16ull;
  }
}

namespace {
struct ProbeState {
  int device = -1;
  hipStream_t stream = nullptr;
  float4v* hbm = nullptr;
  float* sink = nullptr;
  unsigned long long* host = nullptr;  // pinned, device-mapped
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_latency_us = 0.f;  // launch-to-completion of the last probe, incl. waiting for a free CU
  int max_wg = 0;
  long per_wg_vec = 0;
  int pending_wg = 0;  // workgroups of a launched, not yet collected probe
};
constexpr int kMaxDevices = 64;
// One independent state per HIP device: every GPU of a node is probed by one process, each on
// its own non-blocking stream (round-2 verdict: the probe used to cover device 0 only).
ProbeState g_probe[kMaxDevices];

ProbeState* state_of(int device) {
  if (device < 0 || device >= kMaxDevices || g_probe[device].device != device) return nullptr;
  return &g_probe[device];
}
}  // namespace

// Allocate the probe's buffers on `device`: `slice_kb` KB of HBM per workgroup, up to `max_wg`.
// Leaves the calling thread's current device unchanged.
extern "C" int th_probe_init(int device, int max_wg, int slice_kb) {
  if (device < 0 || device >= kMaxDevices || max_wg <= 0 || slice_kb <= 0) return -1;
  ProbeState& st = g_probe[device];
  if (st.device == device) return 0;
  int prev = 0;
  hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return 1;
  int rc = 0;
  st.max_wg = max_wg;
  st.per_wg_vec = (long)slice_kb * 1024 / 16;
  const size_t bytes = (size_t)max_wg * st.per_wg_vec * 16;
  if (hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking) != hipSuccess) rc = 2;
  else if (hipMalloc((void**)&st.hbm, bytes) != hipSuccess) rc = 3;
  else if (hipMemsetAsync(st.hbm, 0, bytes, st.stream) != hipSuccess) rc = 3;
  else if (hipMalloc((void**)&st.sink, 64) != hipSuccess) rc = 4;
  else if (hipHostMalloc((void**)&st.host, (size_t)max_wg * 4 * 8, hipHostMallocMapped) != hipSuccess) rc = 5;
  else if (hipEventCreate(&st.ev0) != hipSuccess || hipEventCreate(&st.ev1) != hipSuccess) rc = 6;
  else if (hipStreamSynchronize(st.stream) != hipSuccess) rc = 7;
  if (rc == 0) st.device = device;
  hipSetDevice(prev);
  return rc;
}

// Launch one probe on `device` without waiting (so every GPU of a node is probed at the same
// moment); th_probe_collect() waits for it and decodes the result.
extern "C" int th_probe_launch(int device, int n_wg, int mfma_iters) {
  ProbeState* st = state_of(device);
  if (!st || n_wg <= 0 || n_wg > st->max_wg || mfma_iters <= 0) return -1;
  unsigned long long* dev_host = nullptr;
  if (hipHostGetDevicePointer((void**)&dev_host, st->host, 0) != hipSuccess) return 2;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  hipEventRecord(st->ev0, st->stream);
  th_probe_kernel<<<n_wg, 256, 0, st->stream>>>(st->hbm, st->per_wg_vec, mfma_iters, dev_host, st->sink);
  const hipError_t e = hipGetLastError();
  hipEventRecord(st->ev1, st->stream);
  hipSetDevice(prev);
  if (e != hipSuccess) return 3;
  st->pending_wg = n_wg;
  return 0;
}

// Wait for the launched probe; out[5*i..] = {xcc_id, mfma_us, hbm_us, hbm_GBps, bytes} for
// workgroup i.  Returns the number of workgroups.
extern "C" int th_probe_collect(int device, double* out) {
  ProbeState* st = state_of(device);
  if (!st || st->pending_wg <= 0) return -1;
  const int n_wg = st->pending_wg;
  st->pending_wg = 0;
  if (hipStreamSynchronize(st->stream) != hipSuccess) return -4;
  float ms = 0.f;
  st->last_latency_us = hipEventElapsedTime(&ms, st->ev0, st->ev1) == hipSuccess ? ms * 1e3f : 0.f;
  for (int i = 0; i < n_wg; ++i) {
    const unsigned long long* r = st->host + 4 * i;
    const double mfma_us = r[1] / 100.0, hbm_us = r[2] / 100.0;  // 100 MHz ticks
    out[5 * i + 0] = (double)r[0];
    out[5 * i + 1] = mfma_us;
    out[5 * i + 2] = hbm_us;
    out[5 * i + 3] = hbm_us > 0 ? (double)r[3] / (hbm_us * 1e-6) / 1e9 : 0.0;
    out[5 * i + 4] = (double)r[3];
  }
  return n_wg;
}

// Launch + collect on one device.
extern "C" int th_probe_sample(int device, int n_wg, int mfma_iters, double* out) {
  const int rc = th_probe_launch(device, n_wg, mfma_iters);
  if (rc != 0) return rc < 0 ? rc : -rc;
  return th_probe_collect(device, out);
}

// Queue-to-completion time of the last probe on `device` (us).  A tenant kernel that holds every
// CU's register file (e.g. a 1-wave/SIMD MFMA GEMM) never shares a SIMD with the probe, so it does
// not slow the probe's MFMA chain; it delays the probe's dispatch instead -- this latency rises.
extern "C" double th_probe_last_latency_us(int device) {
  ProbeState* st = state_of(device);
  return st ? (double)st->last_latency_us : -1.0;
}

extern "C" int th_probe_shutdown(int device) {
  ProbeState* st = state_of(device);
  if (!st) return 0;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  hipStreamSynchronize(st->stream);
  hipEventDestroy(st->ev0);
  hipEventDestroy(st->ev1);
  hipFree(st->hbm);
  hipFree(st->sink);
  hipHostFree(st->host);
  hipStreamDestroy(st->stream);
  hipSetDevice(prev);
  *st = ProbeState();
  return 0;
}
