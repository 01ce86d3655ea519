// Cross-entropy over a vocab-wide logits chunk, producing the loss AND the logits gradient in
// place (gfx950).  Used by the fused LM-head + CE of the Llama payload: the head GEMM writes a
// [rows, V] bf16 chunk, this kernel turns it into dlogits = (softmax - onehot) * grad_scale,
// and the chunk is immediately consumed by the dX / dW GEMMs -- the full [T, 128256] logits
// tensor never exists.
//
// One 512-thread workgroup per row: pass 1 is an online (max, sum-exp) over 16-byte vectors
// (each thread keeps its own pair, merged by wave shuffles and an LDS combine), pass 2 re-reads
// the row (L2-resident: 256 KB per row) and writes the gradient.
#include "th_common.h"

__global__ __launch_bounds__(512) void ce_fwd_bwd_kernel(ushort* __restrict__ logits, long ld,
                                                         const long* __restrict__ target,
                                                         float* __restrict__ loss,
                                                         float* __restrict__ lse_out, int V,
                                                         float grad_scale, int ignore_index) {
  __shared__ float sm[16], ss[16];
  const long row = blockIdx.x;
  ushort* lr = logits + row * ld;
  const int nvec = (ld & 7) == 0 ? (V >> 3) : 0;  // 16-byte path only on aligned rows
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < nvec; i += blockDim.x) {
    const ushort8 x = reinterpret_cast<const ushort8*>(lr)[i];
    float vmax = -INFINITY;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = bf2f(x[j]);
      vmax = fmaxf(vmax, f[j]);
    }
    float vs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) vs += __expf(f[j] - vmax);
    lse_merge(m, s, vmax, vs);
  }
  for (int i = (nvec << 3) + threadIdx.x; i < V; i += blockDim.x) lse_merge(m, s, bf2f(lr[i]), 1.f);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  m = sm[0]; s = ss[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) lse_merge(m, s, sm[w], ss[w]);
  const float lse = m + __logf(s);
  const long tgt = target[row];
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;  // never read out of the row
  if (threadIdx.x == 0) {
    lse_out[row] = lse;
    loss[row] = valid ? (lse - bf2f(lr[tgt])) : 0.f;
  }
  __syncthreads();  // the target logit is read above before any thread overwrites it
  const float gs = valid ? grad_scale : 0.f;
  for (int i = threadIdx.x; i < nvec; i += blockDim.x) {
    const ushort8 x = reinterpret_cast<const ushort8*>(lr)[i];
    ushort8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(bf2f(x[j]) - lse);
      if (valid && (long)(i * 8 + j) == tgt) p -= 1.f;
      o[j] = f2bf(p * gs);
    }
    reinterpret_cast<ushort8*>(lr)[i] = o;
  }
  for (int i = (nvec << 3) + threadIdx.x; i < V; i += blockDim.x) {
    float p = __expf(bf2f(lr[i]) - lse);
    if (valid && (long)i == tgt) p -= 1.f;
    lr[i] = f2bf(p * gs);
  }
}

extern "C" int th_ce_fwd_bwd(void* logits, long ld, const long* target, float* loss, float* lse,
                             long rows, int V, float grad_scale, int ignore_index, hipStream_t s) {
  if (rows <= 0 || V <= 0 || ld < V) return -1;
  ce_fwd_bwd_kernel<<<(unsigned)rows, 512, 0, s>>>((ushort*)logits, ld, target, loss, lse, V,
                                                  grad_scale, ignore_index);
  TH_CHECK_LAUNCH();
}
