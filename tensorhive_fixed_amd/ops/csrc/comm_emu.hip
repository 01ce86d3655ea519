// One-GPU rehearsal of the CU footprint RCCL's channel kernels leave on the N > 1 step (round-6 item 1).
//
// A ring reduce-scatter / all-gather over xGMI runs as ONE kernel per collective with one workgroup per
// channel; every channel workgroup stays resident for the whole collective (it copies a slice, then spins on
// its peer's flags), so for the collective's lifetime those CUs are not available to the compute stream.
// The step's big MFMA kernels (the TN weight-gradient GEMM, hipBLASLt's 256 x 256 tiles, flash attention)
// run one 128-KB-LDS, full-register-file workgroup per CU and cannot share a CU with any other wave: a CU a
// channel holds is a CU the GEMM loses, and a GEMM whose tiles fill exactly 256 CUs spills into a second round.
//
// comm_channel_kernel reproduces that footprint without a second GPU:
//   * one workgroup per CU (a 96 KB LDS reservation forbids two on one CU, as the GEMM's 128 KB does);
//   * each workgroup streams HBM the way a ring copy does (16-B loads + stores over its own slice,
//     optionally throttled to a copy rate so the HBM share matches a modelled bus bandwidth);
//   * it ends when (a) the step's stop marker reaches its generation (written on the COMPUTE stream at
//     finish_grad_sync, so it is stream-ordered after backward), (b) its byte budget is moved (per-bucket
//     mode: the bytes a ring reduce-scatter of that bucket moves), or (c) its time slice expires -- every
//     wave reaches (c), so the grid always drains even if nothing ever writes the marker.
// Stats (per launch, added with vector atomics): {workgroups, bytes copied, 100 MHz ticks resident}.
#include "th_common.h"

namespace {

constexpr int kEmuLds = 96 * 1024;  // > 160 KB / 2: one channel workgroup per CU

__device__ __forceinline__ unsigned long long rt_now() { return wall_clock64(); }  // 100 MHz constant clock

__global__ __launch_bounds__(256) void comm_channel_kernel(const float4v* __restrict__ src, float4v* __restrict__ dst,
                                                          long slice_vec, long chunk_vec, long budget_vec,
                                                          unsigned long long ticks_per_chunk, const int* stop,
                                                          int gen, unsigned long long slice_ticks,
                                                          unsigned long long* stats) {
  __shared__ float reserve[kEmuLds / 4];
  __shared__ int s_go;
  const int tid = threadIdx.x;
  reserve[tid] = 0.f;  // the reservation is real LDS: the compiler keeps it because it is written and read
  const unsigned long long t0 = rt_now();
  const float4v* s = src + (long)blockIdx.x * slice_vec;
  float4v* d = dst + (long)blockIdx.x * slice_vec;
  long moved = 0, pos = 0, chunks = 0;
  for (;;) {
    if (tid == 0) {
      const int m = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long now = rt_now();
      s_go = (m < gen) && (now - t0 < slice_ticks) && (budget_vec == 0 || moved < budget_vec);
    }
    __syncthreads();
    const int go = s_go;
    __syncthreads();
    if (!go) break;
    if (pos + chunk_vec > slice_vec) pos = 0;
    for (long i = tid; i < chunk_vec; i += 2048) {  // 8 x 16 B in flight per lane (chunk_vec % 2048 == 0)
      float4v v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = s[pos + i + 256 * j];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[pos + i + 256 * j] = v[j];
    }
    pos += chunk_vec;
    moved += chunk_vec;
    ++chunks;
    if (ticks_per_chunk) {  // copy-rate throttle: sleep until this chunk's slot in the modelled stream
      const unsigned long long due = t0 + ticks_per_chunk * (unsigned long long)chunks;
      while (rt_now() < due && rt_now() - t0 < slice_ticks) __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned long long t1 = rt_now();
    atomicAdd(&stats[0], 1ull);
    atomicAdd(&stats[1], (unsigned long long)moved * 16ull);
    atomicAdd(&stats[2], t1 - t0);
    atomicAdd(&stats[3], reserve[gen & 255] == 12345.f ? 1ull : 0ull);  // always 0; keeps the reservation alive
  }
}

// stop marker := gen (one lane, vector atomic store; ordered on the stream it is launched on)
__global__ void comm_stop_kernel(int* stop, int gen) {
  if (threadIdx.x == 0) __hip_atomic_store(stop, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// Launch `nwg` channel workgroups on stream `s`.  src / dst: nwg * slice_vec float4 each.
// chunk_vec: float4 per workgroup per iteration; budget_vec: float4 per workgroup before it exits (0 = none);
// ticks_per_chunk: 100 MHz ticks per chunk (0 = unthrottled); slice_us: hard time limit of the launch.
extern "C" int th_comm_emu_launch(void* src, void* dst, long slice_vec, long chunk_vec, long budget_vec,
                                  long ticks_per_chunk, const int* stop, int gen, long slice_us, int nwg,
                                  unsigned long long* stats, hipStream_t s) {
  if (!src || !dst || !stop || !stats || nwg <= 0 || nwg > 256 || slice_vec <= 0 || chunk_vec <= 0 ||
      chunk_vec > slice_vec || chunk_vec % 2048 || budget_vec < 0 || ticks_per_chunk < 0 || slice_us <= 0 || slice_us > 10000000)
    return -1;
  if ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) return -1;
  comm_channel_kernel<<<nwg, 256, 0, s>>>((const float4v*)src, (float4v*)dst, slice_vec, chunk_vec, budget_vec,
                                         (unsigned long long)ticks_per_chunk, stop, gen,
                                         (unsigned long long)slice_us * 100ull, stats);
  TH_CHECK_LAUNCH();
}

extern "C" int th_comm_emu_stop(int* stop, int gen, hipStream_t s) {
  if (!stop) return -1;
  comm_stop_kernel<<<1, 64, 0, s>>>(stop, gen);
  TH_CHECK_LAUNCH();
}
