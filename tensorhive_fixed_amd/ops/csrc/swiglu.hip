// SwiGLU activation (Llama MLP) forward / backward for gfx950.
//
// Input is the output of the fused gate+up projection, gu[T, 2F] (columns [0,F) = gate,
// [F,2F) = up), so the MLP runs ONE GEMM for both projections.  out[T, F] = silu(g) * u.
// Pure streaming: 16-byte vector loads/stores, grid-stride over (row, 8-column chunk) with
// the grid capped at 8 workgroups per CU.
#include "th_common.h"

__device__ __forceinline__ float sigmoidf_(float g) { return 1.f / (1.f + __expf(-g)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const ushort* __restrict__ gu,
                                                         ushort* __restrict__ out, long T, int F) {
  const int cpr = F >> 3;  // 8-wide chunks per row
  const long total = T * (long)cpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int c = (int)(i - row * cpr);
    const ushort8 g = *reinterpret_cast<const ushort8*>(gu + row * 2 * F + c * 8);
    const ushort8 u = *reinterpret_cast<const ushort8*>(gu + row * 2 * F + F + c * 8);
    ushort8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      o[j] = f2bf(gf * sigmoidf_(gf) * bf2f(u[j]));
    }
    *reinterpret_cast<ushort8*>(out + row * F + c * 8) = o;
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const ushort* __restrict__ dout,
                                                         const ushort* __restrict__ gu,
                                                         ushort* __restrict__ dgu, long T, int F) {
  const int cpr = F >> 3;
  const long total = T * (long)cpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpr;
    const int c = (int)(i - row * cpr);
    const ushort8 g = *reinterpret_cast<const ushort8*>(gu + row * 2 * F + c * 8);
    const ushort8 u = *reinterpret_cast<const ushort8*>(gu + row * 2 * F + F + c * 8);
    const ushort8 d = *reinterpret_cast<const ushort8*>(dout + row * F + c * 8);
    ushort8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      const float sg = sigmoidf_(gf);
      const float silu = gf * sg;
      du[j] = f2bf(df * silu);
      dg[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    *reinterpret_cast<ushort8*>(dgu + row * 2 * F + c * 8) = dg;
    *reinterpret_cast<ushort8*>(dgu + row * 2 * F + F + c * 8) = du;
  }
}

static unsigned grid_for(long work) {
  long g = (work + 255) / 256;
  if (g > 2048) g = 2048;  // 256 CUs x 8 workgroups, grid-stride the rest
  if (g < 1) g = 1;
  return (unsigned)g;
}

extern "C" int th_swiglu_fwd(const void* gu, void* out, long T, int F, hipStream_t s) {
  if (F % 8 != 0 || T <= 0) return -1;
  swiglu_fwd_kernel<<<grid_for(T * (F / 8)), 256, 0, s>>>((const ushort*)gu, (ushort*)out, T, F);
  TH_CHECK_LAUNCH();
}

extern "C" int th_swiglu_bwd(const void* dout, const void* gu, void* dgu, long T, int F,
                             hipStream_t s) {
  if (F % 8 != 0 || T <= 0) return -1;
  swiglu_bwd_kernel<<<grid_for(T * (F / 8)), 256, 0, s>>>((const ushort*)dout, (const ushort*)gu,
                                                          (ushort*)dgu, T, F);
  TH_CHECK_LAUNCH();
}
