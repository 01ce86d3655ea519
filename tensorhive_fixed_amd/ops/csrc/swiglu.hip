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

// Backward that ALSO writes the transposed gradient dguT[2F, T] (the K-contiguous operand of the
// gate|up weight-grad GEMM, see ops/linear.py): one 128-token x 64-feature tile per workgroup,
// gate and up halves staged in LDS (odd-dword pitch) and written out as 256-B row segments.
// Costs one extra 2F*T*2-byte write instead of a separate transpose pass (read + write).
constexpr int ST_R = 128, ST_C = 64, ST_P = ST_C + 2;

__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const ushort* __restrict__ dout,
                                                           const ushort* __restrict__ gu,
                                                           ushort* __restrict__ dgu,
                                                           ushort* __restrict__ dguT, long T, int F) {
  __shared__ ushort tg[ST_R * ST_P];
  __shared__ ushort tu[ST_R * ST_P];
  const int tid = threadIdx.x;
  const long ntc = F / ST_C;
  const long r0 = (blockIdx.x / ntc) * ST_R, c0 = (blockIdx.x % ntc) * ST_C;
  const int lc = (tid & 7) * 8;
  ushort8 g[4], u[4], d[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long row = r0 + (tid >> 3) + 32 * i;
    const long rr = row < T ? row : T - 1;  // clamped: finite data, never stored
    g[i] = *reinterpret_cast<const ushort8*>(gu + rr * 2 * F + c0 + lc);
    u[i] = *reinterpret_cast<const ushort8*>(gu + rr * 2 * F + F + c0 + lc);
    d[i] = *reinterpret_cast<const ushort8*>(dout + rr * F + c0 + lc);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int lr = (tid >> 3) + 32 * i;
    const long row = r0 + lr;
    ushort8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[i][j]), uf = bf2f(u[i][j]), df = bf2f(d[i][j]);
      const float sg = sigmoidf_(gf);
      du[j] = f2bf(df * gf * sg);
      dg[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    if (row < T) {
      *reinterpret_cast<ushort8*>(dgu + row * 2 * F + c0 + lc) = dg;
      *reinterpret_cast<ushort8*>(dgu + row * 2 * F + F + c0 + lc) = du;
    }
    unsigned* pg = reinterpret_cast<unsigned*>(tg + lr * ST_P + lc);
    unsigned* pu = reinterpret_cast<unsigned*>(tu + lr * ST_P + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pg[j] = (unsigned)dg[2 * j] | ((unsigned)dg[2 * j + 1] << 16);
      pu[j] = (unsigned)du[2 * j] | ((unsigned)du[2 * j + 1] << 16);
    }
  }
  __syncthreads();
  // 4 lanes per output row (feature), 32 tokens each
  const int oc = tid >> 2, orr = (tid & 3) * 32;
  ushort* og = dguT + (c0 + oc) * T + r0 + orr;
  ushort* ou = dguT + (F + c0 + oc) * T + r0 + orr;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ushort8 wg, wu;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wg[j] = tg[(orr + 8 * q + j) * ST_P + oc];
      wu[j] = tu[(orr + 8 * q + j) * ST_P + oc];
    }
    if (r0 + orr + 8 * q < T) {
      *reinterpret_cast<ushort8*>(og + 8 * q) = wg;
      *reinterpret_cast<ushort8*>(ou + 8 * q) = wu;
    }
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

extern "C" int th_swiglu_bwd_t(const void* dout, const void* gu, void* dgu, void* dguT, long T, int F,
                               hipStream_t s) {
  if (F % ST_C != 0 || T <= 0 || T % 8 != 0) return -1;
  const long tiles = ((T + ST_R - 1) / ST_R) * (F / ST_C);
  if (tiles > 0x7fffffffL) return -2;
  swiglu_bwd_t_kernel<<<(unsigned)tiles, 256, 0, s>>>((const ushort*)dout, (const ushort*)gu, (ushort*)dgu,
                                                      (ushort*)dguT, T, F);
  TH_CHECK_LAUNCH();
}
