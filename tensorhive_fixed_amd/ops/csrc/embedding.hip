// Token-embedding backward for gfx950: deterministic segment sums, no float atomics.
//
// The caller sorts the token ids once (torch.sort on device) giving sorted ids + the
// permutation.  Workgroup i looks at sorted position i; only the FIRST position of each run of
// equal ids does work: it sums the dX rows of the whole run in f32 (fixed order) and writes the
// bf16 gradient row of that token.  Rows of tokens that never occur are zeroed by the caller
// (a memset of the region) unless gradients are being accumulated.
#include "th_common.h"

template <int MAXV>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const long* __restrict__ sorted_ids,
                                                      const long* __restrict__ perm,
                                                      const ushort* __restrict__ dx,
                                                      ushort* __restrict__ gw, long T, int D,
                                                      int accumulate) {
  const long i = blockIdx.x;
  const long tok = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == tok) return;  // not the head of its run (wave-uniform)
  const int nvec = D >> 3;
  float acc[MAXV][8];
#pragma unroll
  for (int a = 0; a < MAXV; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  for (long r = i; r < T && sorted_ids[r] == tok; ++r) {
    const ushort8* src = reinterpret_cast<const ushort8*>(dx + perm[r] * (long)D);
#pragma unroll
    for (int a = 0; a < MAXV; ++a) {
      const int v = threadIdx.x + a * blockDim.x;
      if (v < nvec) {
        const ushort8 x = src[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[a][j] += bf2f(x[j]);
      }
    }
  }
  ushort8* dst = reinterpret_cast<ushort8*>(gw + tok * (long)D);
#pragma unroll
  for (int a = 0; a < MAXV; ++a) {
    const int v = threadIdx.x + a * blockDim.x;
    if (v < nvec) {
      ushort8 o;
      const ushort8 prev = accumulate ? dst[v] : ushort8(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[a][j] + (accumulate ? bf2f(prev[j]) : 0.f));
      dst[v] = o;
    }
  }
}

extern "C" int th_embedding_bwd(const long* sorted_ids, const long* perm, const void* dx, void* gw,
                                long T, int D, int accumulate, hipStream_t s) {
  if (D % 8 != 0 || T <= 0) return -1;
  const int mv = (D / 8 + 255) / 256;
  if (mv <= 2)
    emb_bwd_kernel<2><<<(unsigned)T, 256, 0, s>>>(sorted_ids, perm, (const ushort*)dx, (ushort*)gw, T, D, accumulate);
  else if (mv <= 4)
    emb_bwd_kernel<4><<<(unsigned)T, 256, 0, s>>>(sorted_ids, perm, (const ushort*)dx, (ushort*)gw, T, D, accumulate);
  else
    return -2;
  TH_CHECK_LAUNCH();
}
