// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of tensorhive_fixed_amd.
//
// Conventions used by every kernel in this directory:
//   * wave64 only: lane = threadIdx.x & 63, reductions are 6-step xor shuffles.
//   * bf16 tensors travel as raw `ushort` and are loaded 8 at a time (16 B/lane,
//     `short8`-style) -- hipcc never vectorises scalar bf16 loads on its own.
//   * f32 -> bf16 uses the `__bf16` cast, which lowers to v_cvt_pk_bf16_f32 (RNE,
//     NaN-preserving) at -O3.
//   * Every entry point is `extern "C"` and takes the hipStream_t of the caller, so the
//     Python side (ctypes) launches on torch's current stream without any torch headers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short ushort;
typedef ushort ushort8 __attribute__((ext_vector_type(8)));
typedef ushort ushort4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));

#define TH_WAVE 64

__device__ __forceinline__ float bf2f(ushort u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ ushort f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(ushort, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (<= 16 waves). `scratch` holds >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

// Online (max, sum-exp) pair merge used by the softmax / cross-entropy kernels.
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) { m = mn; s = 0.f; return; }
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

#define TH_CHECK_LAUNCH() return (int)hipGetLastError()
