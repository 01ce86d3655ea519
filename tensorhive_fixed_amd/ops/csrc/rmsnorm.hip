// RMSNorm forward / backward for gfx950.
//
// Memory-bound (1 read + 1 write of a [T, D] bf16 activation per pass), so the design goal is
// HBM rate: one 256-thread workgroup per row, 16-byte (8 x bf16) loads per lane, the row held
// in registers between the sum-of-squares and the normalise pass (no re-read), wave64 shuffle
// reduction + a 4-entry LDS combine.  The weight gradient is reduced without atomics: each
// workgroup of the backward grid owns a strided set of rows and keeps its dW partial in
// registers, writes one f32 slab, and a second kernel sums the slabs (deterministic).
#include "th_common.h"

// ADD: x + addend is formed (rounded to bf16, as a GEMM epilogue would), written to xsum (the
// residual stream) and normalised -- the residual add of the attention-out / MLP-down projections
// fused into the next norm instead of a copy + beta=1 GEMM epilogue.
template <int MAXV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const ushort* __restrict__ x,
                                                              const ushort* __restrict__ addend,
                                                              ushort* __restrict__ xsum,
                                                              const ushort* __restrict__ w,
                                                              ushort* __restrict__ y,
                                                              float* __restrict__ rstd_out, int D,
                                                              float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = D >> 3;
  const ushort8* xr = reinterpret_cast<const ushort8*>(x + (size_t)row * D);
  ushort8 cache[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = threadIdx.x + i * blockDim.x;
    if (v < nvec) {
      cache[i] = xr[v];
      if (ADD) {
        const ushort8 a = reinterpret_cast<const ushort8*>(addend + (size_t)row * D)[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) cache[i][j] = f2bf(bf2f(cache[i][j]) + bf2f(a[j]));
        reinterpret_cast<ushort8*>(xsum + (size_t)row * D)[v] = cache[i];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(cache[i][j]);
        ss += f * f;
      }
    }
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)D + eps);
  if (threadIdx.x == 0) rstd_out[row] = r;
  const ushort8* wr = reinterpret_cast<const ushort8*>(w);
  ushort8* yr = reinterpret_cast<ushort8*>(y + (size_t)row * D);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = threadIdx.x + i * blockDim.x;
    if (v < nvec) {
      const ushort8 wv = wr[v];
      ushort8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(cache[i][j]) * r * bf2f(wv[j]));
      yr[v] = o;
    }
  }
}

// Backward: dx per row, plus per-workgroup dW partial slab ws[blockIdx.x][D] (f32).
template <int MAXV>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const ushort* __restrict__ dy,
                                                          const ushort* __restrict__ x,
                                                          const ushort* __restrict__ w,
                                                          const float* __restrict__ rstd,
                                                          ushort* __restrict__ dx,
                                                          float* __restrict__ ws, int T, int D,
                                                          const ushort* __restrict__ dres) {
  // dres (optional): gradient arriving through the residual branch of the same x, added into dx
  // here instead of by a separate elementwise pass (ops/rmsnorm.py: rmsnorm_fork)
  __shared__ float red[16];
  const int nvec = D >> 3;
  float dwacc[MAXV][8];
  float wreg[MAXV][8];
  const ushort8* wr = reinterpret_cast<const ushort8*>(w);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = threadIdx.x + i * blockDim.x;
    ushort8 wv = (v < nvec) ? wr[v] : ushort8(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dwacc[i][j] = 0.f;
      wreg[i][j] = bf2f(wv[j]);
    }
  }
  for (int row = blockIdx.x; row < T; row += gridDim.x) {
    const ushort8* xr = reinterpret_cast<const ushort8*>(x + (size_t)row * D);
    const ushort8* gr = reinterpret_cast<const ushort8*>(dy + (size_t)row * D);
    ushort8 xc[MAXV], gc[MAXV], rc[MAXV];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = threadIdx.x + i * blockDim.x;
      if (v < nvec) {
        xc[i] = xr[v];
        gc[i] = gr[v];
        rc[i] = dres ? reinterpret_cast<const ushort8*>(dres + (size_t)row * D)[v] : ushort8(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) dot += bf2f(gc[i][j]) * wreg[i][j] * bf2f(xc[i][j]);
      }
    }
    dot = block_sum(dot, red);
    const float r = rstd[row];
    const float c = dot * r * r * r / (float)D;
    ushort8* dxr = reinterpret_cast<ushort8*>(dx + (size_t)row * D);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = threadIdx.x + i * blockDim.x;
      if (v < nvec) {
        ushort8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = bf2f(xc[i][j]), gf = bf2f(gc[i][j]);
          o[j] = f2bf(r * gf * wreg[i][j] - xf * c + bf2f(rc[i][j]));
          dwacc[i][j] += gf * xf * r;
        }
        dxr[v] = o;
      }
    }
  }
  float* wsr = ws + (size_t)blockIdx.x * D;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = threadIdx.x + i * blockDim.x;
    if (v < nvec) {
      float4v* p = reinterpret_cast<float4v*>(wsr + v * 8);
      p[0] = float4v{dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]};
      p[1] = float4v{dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]};
    }
  }
}

// Sum `nslab` f32 slabs of length D into a bf16 vector (optionally accumulating into it).
// 64 columns per workgroup: 16 column-groups of 4 (float4 loads) x 16 slab-groups, each thread
// summing every 16th slab, then an LDS reduction over the slab-groups.  (One thread per column
// walking all 512 slabs serially took 130 us per call -- latency-bound on 16 workgroups.)
__global__ __launch_bounds__(256) void slab_reduce_bf16_kernel(const float* __restrict__ ws, ushort* __restrict__ out,
                                                               int nslab, int D, int accumulate) {
  __shared__ float4v part[16][16];
  const int cg = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cg * 4;
  float4v acc = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
#pragma unroll 4
    for (int b = sg; b < nslab; b += 16) acc += *reinterpret_cast<const float4v*>(ws + (size_t)b * D + c);
  }
  part[sg][cg] = acc;
  __syncthreads();
  if (sg == 0 && c < D) {
    float4v t = part[0][cg];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += part[k][cg];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = t[j];
      if (accumulate) v += bf2f(out[c + j]);
      out[c + j] = f2bf(v);
    }
  }
}

static int pick_maxv(int D, int threads) { return (D / 8 + threads - 1) / threads; }

extern "C" int th_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int T, int D,
                              float eps, hipStream_t s) {
  if (D % 8 != 0 || T <= 0) return -1;
  const int mv = pick_maxv(D, 256);
  dim3 g(T), b(256);
  if (mv <= 2)
    rmsnorm_fwd_kernel<2, false><<<g, b, 0, s>>>((const ushort*)x, nullptr, nullptr, (const ushort*)w, (ushort*)y, rstd, D, eps);
  else if (mv <= 4)
    rmsnorm_fwd_kernel<4, false><<<g, b, 0, s>>>((const ushort*)x, nullptr, nullptr, (const ushort*)w, (ushort*)y, rstd, D, eps);
  else if (mv <= 8)
    rmsnorm_fwd_kernel<8, false><<<g, b, 0, s>>>((const ushort*)x, nullptr, nullptr, (const ushort*)w, (ushort*)y, rstd, D, eps);
  else
    return -2;
  TH_CHECK_LAUNCH();
}

// xsum = x + addend (bf16), y = rmsnorm(xsum) * w
extern "C" int th_rmsnorm_add_fwd(const void* x, const void* addend, const void* w, void* xsum, void* y,
                                  float* rstd, int T, int D, float eps, hipStream_t s) {
  if (D % 8 != 0 || T <= 0) return -1;
  const int mv = pick_maxv(D, 256);
  dim3 g(T), b(256);
#define TH_RMS_ADD(MV)                                                                                   \
  rmsnorm_fwd_kernel<MV, true><<<g, b, 0, s>>>((const ushort*)x, (const ushort*)addend, (ushort*)xsum, \
                                               (const ushort*)w, (ushort*)y, rstd, D, eps)
  if (mv <= 2)
    TH_RMS_ADD(2);
  else if (mv <= 4)
    TH_RMS_ADD(4);
  else if (mv <= 8)
    TH_RMS_ADD(8);
  else
    return -2;
#undef TH_RMS_ADD
  TH_CHECK_LAUNCH();
}

// Workspace: nblk * D floats; nblk chosen by the caller (<= T), typically 2 * 256 CUs.
extern "C" int th_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                              void* dx, void* dw, float* ws, int nblk, int T, int D,
                              int accumulate, const void* dres, hipStream_t s) {
  if (D % 8 != 0 || T <= 0 || nblk <= 0) return -1;
  const int mv = pick_maxv(D, 256);
  dim3 g(nblk), b(256);
  if (mv <= 2)
    rmsnorm_bwd_kernel<2><<<g, b, 0, s>>>((const ushort*)dy, (const ushort*)x, (const ushort*)w, rstd, (ushort*)dx, ws, T, D, (const ushort*)dres);
  else if (mv <= 4)
    rmsnorm_bwd_kernel<4><<<g, b, 0, s>>>((const ushort*)dy, (const ushort*)x, (const ushort*)w, rstd, (ushort*)dx, ws, T, D, (const ushort*)dres);
  else if (mv <= 8)
    rmsnorm_bwd_kernel<8><<<g, b, 0, s>>>((const ushort*)dy, (const ushort*)x, (const ushort*)w, rstd, (ushort*)dx, ws, T, D, (const ushort*)dres);
  else
    return -2;
  slab_reduce_bf16_kernel<<<dim3((D + 63) / 64), dim3(256), 0, s>>>(ws, (ushort*)dw, nblk, D, accumulate);
  TH_CHECK_LAUNCH();
}
