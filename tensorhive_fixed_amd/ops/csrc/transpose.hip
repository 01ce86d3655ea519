// bf16 matrix transpose for gfx950: out[C, R] = in[R, C]^T.
//
// Why it exists: hipBLASLt on gfx950 runs the "both operands K-contiguous" GEMM form ~10-25 %
// faster than the forms whose reduction dim is the outer (row) dim (scripts/gemm_layouts.py,
// profiles/r01_gemm/).  The linear backward therefore transposes W once per step into a
// K-contiguous copy for dX = dY W, and the widest weight-grad GEMM (gate|up) transposes its
// operands so dW = dYᵀX runs in that form; a transpose is only worth it when it moves bytes
// near HBM speed, which torch's generic `.t().contiguous()` (~1 TB/s) does not.
//
// Tile 128 (rows of `in`) x 64 (cols), 256 threads.  Load: each thread moves 4 x 16 B, eight
// lanes cover one 128-B input row segment.  The tile is staged in LDS with a 66-element row
// pitch (33 dwords: a column walk touches 33 distinct banks -> conflict-free).  Store: four
// lanes own one output row and write 4 x 16 B each = 256 B contiguous per output row.
// Edge tiles are guarded; R and C must be multiples of 8 (16-B vectors).
#include "th_common.h"

#define TR 128
#define TC 64
#define PITCH (TC + 2)

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const ushort* __restrict__ in,
                                                             ushort* __restrict__ out, long R, long C,
                                                             long ld_in) {
  __shared__ ushort tile[TR * PITCH];
  const int tid = threadIdx.x;
  const long ntc = (C + TC - 1) / TC;
  const long bt = blockIdx.x;
  const long r0 = (bt / ntc) * TR, c0 = (bt % ntc) * TC;

  const int lc = (tid & 7) * 8;
#pragma unroll
  for (int i = 0; i < TR / 32; ++i) {
    const int lr = (tid >> 3) + 32 * i;
    ushort8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + lr < R && c0 + lc < C) v = *reinterpret_cast<const ushort8*>(in + (r0 + lr) * ld_in + c0 + lc);
    unsigned* dst = reinterpret_cast<unsigned*>(tile + lr * PITCH + lc);  // 4-B aligned: PITCH even
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = (unsigned)v[2 * j] | ((unsigned)v[2 * j + 1] << 16);
  }
  __syncthreads();

  const int oc = tid >> 2;          // output row = input column within the tile
  const int orr = (tid & 3) * 32;   // 32 consecutive input rows per lane
  if (c0 + oc >= C) return;
  ushort* orow = out + (c0 + oc) * R + r0 + orr;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ushort8 w;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = tile[(orr + 8 * q + j) * PITCH + oc];
    if (r0 + orr + 8 * q < R) *reinterpret_cast<ushort8*>(orow + 8 * q) = w;
  }
}

extern "C" int th_transpose_bf16(const void* in, void* out, long R, long C, long ld_in, hipStream_t s) {
  if (R <= 0 || C <= 0 || R % 8 || C % 8 || ld_in % 8 || ld_in < C) return -1;
  const long tiles = ((R + TR - 1) / TR) * ((C + TC - 1) / TC);
  if (tiles > 0x7fffffffL) return -2;
  transpose_bf16_kernel<<<(unsigned)tiles, 256, 0, s>>>((const ushort*)in, (ushort*)out, R, C, ld_in);
  TH_CHECK_LAUNCH();
}
