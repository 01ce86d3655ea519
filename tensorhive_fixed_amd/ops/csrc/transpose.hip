// bf16 matrix transpose for gfx950: out[C, R] = in[R, C]^T.
//
// Why it exists: hipBLASLt on gfx950 runs the "both operands K-contiguous" GEMM form ~10-25 %
// faster than the forms whose reduction dim is the outer (row) dim (scripts/gemm_layouts.py,
// profiles/r01_gemm/).  The linear backward therefore transposes W once per step into a
// K-contiguous copy for dX = dY W, and the widest weight-grad GEMM (gate|up) transposes its
// operands so dW = dYᵀX runs in that form; a transpose is only worth it when it moves bytes
// near HBM speed, which torch's generic `.t().contiguous()` (~1 TB/s) does not.
//
// Tiles TR (rows of `in`) x TC (cols), 256 threads: every thread issues all of its 16-B loads
// before touching LDS; the tile is staged with an odd-dword row pitch (TC + 2 elements: a column
// walk touches distinct banks), then 256/TC lanes own one output row and write TR*2/(256/TC) B
// of it contiguously.  Edge tiles are guarded; R and C must be multiples of 8 (16-B vectors).
#include "th_common.h"

template <int TR, int TC>
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const ushort* __restrict__ in,
                                                             ushort* __restrict__ out, long R, long C,
                                                             long ld_in) {
  constexpr int PITCH = TC + 2;        // odd dword pitch: a column walk hits distinct banks
  constexpr int LPR = TC / 8;          // lanes per input row segment (16 B each)
  constexpr int RPP = 256 / LPR;       // input rows per load pass
  constexpr int OPL = 256 / TC;        // lanes per output row
  constexpr int RPL = TR / OPL;        // input rows (= output elements) per lane
  __shared__ ushort tile[TR * PITCH];
  const int tid = threadIdx.x;
  const long ntc = (C + TC - 1) / TC;
  const long bt = blockIdx.x;
  const long r0 = (bt / ntc) * TR, c0 = (bt % ntc) * TC;

  const int lc = (tid % LPR) * 8;
  ushort8 v[TR / RPP];
#pragma unroll
  for (int i = 0; i < TR / RPP; ++i) {  // all loads first: TR*TC*2/256 bytes in flight per thread
    const int lr = tid / LPR + RPP * i;
    v[i] = ushort8(0);
    if (r0 + lr < R && c0 + lc < C) v[i] = *reinterpret_cast<const ushort8*>(in + (r0 + lr) * ld_in + c0 + lc);
  }
#pragma unroll
  for (int i = 0; i < TR / RPP; ++i) {
    const int lr = tid / LPR + RPP * i;
    unsigned* dst = reinterpret_cast<unsigned*>(tile + lr * PITCH + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = (unsigned)v[i][2 * j] | ((unsigned)v[i][2 * j + 1] << 16);
  }
  __syncthreads();

  const int oc = tid / OPL;            // output row = input column within the tile
  const int orr = (tid % OPL) * RPL;   // RPL consecutive input rows per lane
  if (c0 + oc >= C) return;
  ushort* orow = out + (c0 + oc) * R + r0 + orr;
#pragma unroll
  for (int q = 0; q < RPL / 8; ++q) {
    ushort8 w;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = tile[(orr + 8 * q + j) * PITCH + oc];
    if (r0 + orr + 8 * q < R) *reinterpret_cast<ushort8*>(orow + 8 * q) = w;
  }
}

extern "C" int th_transpose_bf16(const void* in, void* out, long R, long C, long ld_in, int tile, hipStream_t s) {
  if (R <= 0 || C <= 0 || R % 8 || C % 8 || ld_in % 8 || ld_in < C) return -1;
  // tile 1: 128 x 64; 2: 128 x 128; 3: 64 x 128; 0: by shape
  auto launch = [&](auto kern, long tr, long tc) {
    const long tiles = ((R + tr - 1) / tr) * ((C + tc - 1) / tc);
    if (tiles > 0x7fffffffL) return -2;
    kern<<<(unsigned)tiles, 256, 0, s>>>((const ushort*)in, (ushort*)out, R, C, ld_in);
    return (int)hipGetLastError();
  };
  // default: 64 x 128 (4.2-4.7 TB/s on the weight and activation shapes) except very wide inputs,
  // where 128 x 64 keeps more rows in flight (32768 x 28672: 3.7 vs 3.15 TB/s; profiles/r01_gemm)
  if (tile == 0) tile = C > 16384 ? 1 : 3;
  switch (tile) {
    case 2: return launch(transpose_bf16_kernel<128, 128>, 128, 128);
    case 3: return launch(transpose_bf16_kernel<64, 128>, 64, 128);
    default: return launch(transpose_bf16_kernel<128, 64>, 128, 64);
  }
}
