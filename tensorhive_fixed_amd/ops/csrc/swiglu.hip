// SwiGLU activation (Llama MLP) forward / backward for gfx950.
//
// Input is the output of the fused gate+up projection, gu[T, 2F] (columns [0,F) = gate,
// [F,2F) = up), so the MLP runs ONE GEMM for both projections.  out[T, F] = silu(g) * u.
// Pure streaming: 16-byte vector loads/stores; one workgroup per row (row-strided grid).
#include "th_common.h"

__device__ __forceinline__ float sigmoidf_(float g) { return 1.f / (1.f + __expf(-g)); }

// Row-blocked indexing: a workgroup owns whole rows (blockIdx.y strides over rows) and its
// threads stride over the row's 8-wide chunks, so there is no 64-bit division per element chunk
// (the flat grid-stride form spent more VALU on `i / cpr` than on the activation).
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const ushort* __restrict__ gu,
                                                         ushort* __restrict__ out, long T, int F) {
  const int cpr = F >> 3;  // 8-wide chunks per row
  for (long row = blockIdx.x; row < T; row += gridDim.x) {
    const ushort* g_row = gu + row * 2 * F;
    ushort* o_row = out + row * F;
    for (int c = threadIdx.x; c < cpr; c += blockDim.x) {
      const ushort8 g = *reinterpret_cast<const ushort8*>(g_row + c * 8);
      const ushort8 u = *reinterpret_cast<const ushort8*>(g_row + F + c * 8);
      ushort8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gf = bf2f(g[j]);
        o[j] = f2bf(gf * sigmoidf_(gf) * bf2f(u[j]));
      }
      *reinterpret_cast<ushort8*>(o_row + c * 8) = o;
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const ushort* __restrict__ dout,
                                                         const ushort* __restrict__ gu,
                                                         ushort* __restrict__ dgu, long T, int F) {
  const int cpr = F >> 3;
  for (long row = blockIdx.x; row < T; row += gridDim.x) {
    for (int c = threadIdx.x; c < cpr; c += blockDim.x) {
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
}

// Backward that ALSO writes the transposed gradient dguT[2F, T] (the K-contiguous operand of the
// gate|up weight-grad GEMM, see ops/linear.py): one 128-token x 64-feature tile per workgroup.
// Costs one extra 2F*T*2-byte write instead of a separate transpose pass (read + write).
//   * dg / du tiles go to LDS as 128-B token rows (ds_write_b128; an 8-lane write group covers one
//     row: conflict-free) with 16-B chunk c of row r stored at chunk c ^ swz(r);
//   * the transpose is done by the LDS hardware: ds_read_b64_tr_b16 hands each lane 4 consecutive
//     tokens of ONE feature, two of them make a 16-B piece of a dguT row.  A wave writes 16
//     feature rows x 64 contiguous bytes per store instruction;
//   * swz(r) = 2*(((r>>1)&1) | ((r>>3)&1)<<1) puts the 8 token rows a 32-lane half reads
//     ({0-3, 8-11} + 16k or {4-7, 12-15} + 16k) on 8 distinct 32-B bank groups: conflict-free.
// (The previous version gathered the transposed pieces with 64 ds_read_u16 per thread and wrote
// 16-B pieces 64 B apart: 1.71 ms at T 32768, F 14336.)
constexpr int ST_R = 128, ST_C = 64;

__device__ __forceinline__ int st_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }
__device__ __forceinline__ int st_off(int r, int chunk) { return r * 128 + ((chunk ^ st_swz(r)) << 4); }

typedef short i16x4s __attribute__((ext_vector_type(4)));
#define ST_LDS __attribute__((address_space(3)))

__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const ushort* __restrict__ dout,
                                                           const ushort* __restrict__ gu,
                                                           ushort* __restrict__ dgu,
                                                           ushort* __restrict__ dguT, long T, int F) {
  __shared__ __attribute__((aligned(16))) char tile[2 * ST_R * 128];  // [g|u][token][64 features]
  const int tid = threadIdx.x;
  const long ntc = F / ST_C;
  const long r0 = (blockIdx.x / ntc) * ST_R, c0 = (blockIdx.x % ntc) * ST_C;
  const int lch = tid & 7, lc = lch * 8;
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
    *reinterpret_cast<ushort8*>(tile + st_off(lr, lch)) = dg;
    *reinterpret_cast<ushort8*>(tile + ST_R * 128 + st_off(lr, lch)) = du;
  }
  __syncthreads();
  // 2 halves x 4 feature blocks of 16 x 4 token groups of 32 = 32 wave-steps, 8 per wave.  In a
  // wave-step, 16-lane group grp takes tokens tg0 + 8*grp .. +7 of features fb*16 .. +15.
  const int lane = tid & 63, w = tid >> 6, grp = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int step = w * 8 + k;
    const int half = step >> 4, fb = (step >> 2) & 3, tg0 = (step & 3) * 32;
    const int rbase = tg0 + 8 * grp;
    const int col = fb * 16 + 4 * p;  // lane 4q+p: row q, features col .. col+3
    const char* base = tile + half * ST_R * 128 + ((col & 7) << 1);
    const int ch = col >> 3;
    const i16x4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ST_LDS i16x4s*)(base + st_off(rbase + q, ch)));
    const i16x4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ST_LDS i16x4s*)(base + st_off(rbase + 4 + q, ch)));
    ushort8 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = (ushort)lo[e];
      o[4 + e] = (ushort)hi[e];
    }
    const long feat = (long)half * F + c0 + fb * 16 + i16;
    const long tok = r0 + rbase;
    if (tok < T) *reinterpret_cast<ushort8*>(dguT + feat * T + tok) = o;
  }
}

// one workgroup per row, capped at 256 CUs x 16 workgroups (row-stride the rest)
static unsigned grid_for(long rows) {
  long g = rows;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

extern "C" int th_swiglu_fwd(const void* gu, void* out, long T, int F, hipStream_t s) {
  if (F % 8 != 0 || T <= 0) return -1;
  swiglu_fwd_kernel<<<grid_for(T), 256, 0, s>>>((const ushort*)gu, (ushort*)out, T, F);
  TH_CHECK_LAUNCH();
}

extern "C" int th_swiglu_bwd(const void* dout, const void* gu, void* dgu, long T, int F,
                             hipStream_t s) {
  if (F % 8 != 0 || T <= 0) return -1;
  swiglu_bwd_kernel<<<grid_for(T), 256, 0, s>>>((const ushort*)dout, (const ushort*)gu,
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
