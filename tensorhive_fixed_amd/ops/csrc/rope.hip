// Rotary position embedding (Llama-3, rotate-half convention) applied IN PLACE to the q and k
// heads of the packed projection output qkv[T, (Hq + 2*Hkv) * Dh] (v heads are untouched).
//
// The cos/sin table [S, Dh/2] (f32) is built once on the host side (theta = 5e5 for Llama-3):
// on-device sin/cos per element would turn this memory-bound op into a VALU-bound one.
// Backward is the inverse rotation, i.e. the same kernel with sign = -1 applied to dqkv.
#include "th_common.h"

__global__ __launch_bounds__(256) void rope_kernel(ushort* __restrict__ qkv,
                                                   const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT, long T, int S,
                                                   int nrot_heads, int row_stride, int Dh,
                                                   float sign) {
  const int half = Dh >> 1;
  const int cph = half >> 3;  // 8-pair chunks per head
  const long total = T * (long)nrot_heads * cph;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cph);
    const long th = i / cph;
    const int h = (int)(th % nrot_heads);
    const long t = th / nrot_heads;
    const int pos = (int)(t % S);
    ushort* base = qkv + t * row_stride + (long)h * Dh + c * 8;
    const ushort8 x1 = *reinterpret_cast<const ushort8*>(base);
    const ushort8 x2 = *reinterpret_cast<const ushort8*>(base + half);
    const float4v* cp = reinterpret_cast<const float4v*>(cosT + (long)pos * half + c * 8);
    const float4v* sp = reinterpret_cast<const float4v*>(sinT + (long)pos * half + c * 8);
    const float4v c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
    const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    ushort8 y1, y2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = bf2f(x1[j]), b = bf2f(x2[j]);
      const float sj = sign * sn[j];
      y1[j] = f2bf(a * cs[j] - b * sj);
      y2[j] = f2bf(b * cs[j] + a * sj);
    }
    *reinterpret_cast<ushort8*>(base) = y1;
    *reinterpret_cast<ushort8*>(base + half) = y2;
  }
}

extern "C" int th_rope_inplace(void* qkv, const float* cosT, const float* sinT, long T, int S,
                               int nrot_heads, int row_stride, int Dh, float sign, hipStream_t s) {
  if (Dh % 16 != 0 || T <= 0 || S <= 0 || row_stride % 8 != 0) return -1;
  const long work = T * (long)nrot_heads * (Dh / 16);
  long g = (work + 255) / 256;
  if (g > 2048) g = 2048;
  rope_kernel<<<(unsigned)g, 256, 0, s>>>((ushort*)qkv, cosT, sinT, T, S, nrot_heads, row_stride,
                                          Dh, sign);
  TH_CHECK_LAUNCH();
}
