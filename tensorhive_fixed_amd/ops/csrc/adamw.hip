// Fused AdamW over ONE flat parameter buffer (gfx950).
//
// The training payload keeps every parameter of the model in a single contiguous bf16 buffer
// with matching flat f32 master / exp_avg / exp_avg_sq buffers and a flat bf16 gradient buffer
// (the DDP buckets are views of it).  The whole optimizer step is therefore one streaming
// kernel (28 B/param: 2 B grad + 12 B state read, 12 B state + 2 B param written) instead of a
// multi-tensor-apply over hundreds of tensors.  Global-norm clipping is done on device: a
// sum-of-squares pre-pass writes ||g||^2 into device memory and the step kernel reads it, so
// there is no host synchronisation anywhere in the step (graph-capturable).
#include "th_common.h"

// 8 consecutive gradient values as f32, from the bf16 (default) or the f32 (TH_GRAD_FP32) buffer
__device__ __forceinline__ void load_grad8(const ushort* __restrict__ g, long i, float out[8]) {
  const ushort8 v = reinterpret_cast<const ushort8*>(g)[i];
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bf2f(v[j]);
}
__device__ __forceinline__ void load_grad8(const float* __restrict__ g, long i, float out[8]) {
  const float4v a = reinterpret_cast<const float4v*>(g)[2 * i], b = reinterpret_cast<const float4v*>(g)[2 * i + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[j] = a[j];
    out[4 + j] = b[j];
  }
}

template <typename G>
__global__ __launch_bounds__(256) void sumsq_kernel(const G* __restrict__ g, long n8, float* __restrict__ partial) {
  __shared__ float red[16];
  float acc = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float v[8];
    load_grad8(g, i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ void final_sum_kernel(const float* __restrict__ partial, int np, float* __restrict__ out,
                                 int accumulate) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + acc : acc;
}

template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(
    ushort* __restrict__ p, float* __restrict__ master, float* __restrict__ m,
    float* __restrict__ v, const G* __restrict__ g, long n8, float lr, float b1, float b2,
    float eps, float wd, float bc1, float bc2, float grad_scale, const float* __restrict__ norm_sq,
    float clip) {
  float scale = grad_scale;
  if (norm_sq != nullptr && clip > 0.f) {
    const float tn = sqrtf(norm_sq[0]) * grad_scale;
    scale *= fminf(1.f, clip / (tn + 1e-6f));
  }
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    float gv[8];
    load_grad8(g, i, gv);
    float4v* mp = reinterpret_cast<float4v*>(master) + 2 * i;
    float4v* m1 = reinterpret_cast<float4v*>(m) + 2 * i;
    float4v* v1 = reinterpret_cast<float4v*>(v) + 2 * i;
    float4v pw[2] = {mp[0], mp[1]}, mw[2] = {m1[0], m1[1]}, vw[2] = {v1[0], v1[1]};
    ushort8 po;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int h = j >> 2, k = j & 3;
      const float gr = gv[j] * scale;
      float mm = b1 * mw[h][k] + (1.f - b1) * gr;
      float vv = b2 * vw[h][k] + (1.f - b2) * gr * gr;
      float pp = pw[h][k] * (1.f - lr * wd);
      pp -= step_size * mm / (sqrtf(vv) * inv_sqrt_bc2 + eps);
      mw[h][k] = mm;
      vw[h][k] = vv;
      pw[h][k] = pp;
      po[j] = f2bf(pp);
    }
    mp[0] = pw[0]; mp[1] = pw[1];
    m1[0] = mw[0]; m1[1] = mw[1];
    v1[0] = vw[0]; v1[1] = vw[1];
    reinterpret_cast<ushort8*>(p)[i] = po;
  }
}

static unsigned grid_cap(long work) {
  long gsz = (work + 255) / 256;
  if (gsz > 2048) gsz = 2048;
  if (gsz < 1) gsz = 1;
  return (unsigned)gsz;
}

// ws must hold >= 2048 floats.  Writes ||g||^2 (or adds it, accumulate=1) to out[0].
extern "C" int th_sumsq_bf16(const void* g, long n, float* ws, float* out, int accumulate,
                             hipStream_t s) {
  if (n % 8 != 0 || n <= 0) return -1;
  const unsigned gs = grid_cap(n / 8);
  sumsq_kernel<ushort><<<gs, 256, 0, s>>>((const ushort*)g, n / 8, ws);
  final_sum_kernel<<<1, 1024, 0, s>>>(ws, (int)gs, out, accumulate);
  TH_CHECK_LAUNCH();
}

extern "C" int th_sumsq_f32(const float* g, long n, float* ws, float* out, int accumulate, hipStream_t s) {
  if (n % 8 != 0 || n <= 0) return -1;
  const unsigned gs = grid_cap(n / 8);
  sumsq_kernel<float><<<gs, 256, 0, s>>>(g, n / 8, ws);
  final_sum_kernel<<<1, 1024, 0, s>>>(ws, (int)gs, out, accumulate);
  TH_CHECK_LAUNCH();
}

extern "C" int th_adamw_step(void* p, float* master, float* m, float* v, const void* g, long n,
                             float lr, float b1, float b2, float eps, float wd, int step,
                             float grad_scale, const float* norm_sq, float clip, hipStream_t s) {
  if (n % 8 != 0 || n <= 0 || step < 1) return -1;
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  adamw_kernel<ushort><<<grid_cap(n / 8), 256, 0, s>>>((ushort*)p, master, m, v, (const ushort*)g, n / 8, lr,
                                                       b1, b2, eps, wd, bc1, bc2, grad_scale, norm_sq, clip);
  TH_CHECK_LAUNCH();
}

// Same step reading an f32 gradient buffer (TH_GRAD_FP32): 34 B/param instead of 28.
extern "C" int th_adamw_step_f32g(void* p, float* master, float* m, float* v, const float* g, long n,
                                  float lr, float b1, float b2, float eps, float wd, int step,
                                  float grad_scale, const float* norm_sq, float clip, hipStream_t s) {
  if (n % 8 != 0 || n <= 0 || step < 1) return -1;
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  adamw_kernel<float><<<grid_cap(n / 8), 256, 0, s>>>((ushort*)p, master, m, v, g, n / 8, lr, b1, b2, eps, wd,
                                                      bc1, bc2, grad_scale, norm_sq, clip);
  TH_CHECK_LAUNCH();
}
