// Weight-gradient GEMM in the layout training produces, for gfx950 (MI355X):
//
//     C[M][N] (+)= sum_k A[k][M] * B[k][N]        (dW = dY^T X, k = tokens)
//
// A = dY [tokens][out] and B = X [tokens][in] are both row-major with the reduction index as
// the SLOW dimension.  hipBLASLt runs this "TN" form at 1.0-1.2 PFLOP/s on the Llama-3-8B
// shapes against 1.4-1.6 for the K-contiguous forms (profiles/r01_gemm/); the K-contiguous form
// needs two transposes of activation-sized operands first.  This kernel reads the operands as
// they are: tiles are staged k-row by k-row with LDS-DMA (global_load_lds_dwordx4) and the MFMA
// operands are gathered column-wise with the hardware transpose read ds_read_b64_tr_b16.
//
//   * tile 256 x 256 x 64, 512 threads = 8 waves as 2 (M) x 4 (N), wave tile 128 x 64,
//     v_mfma_f32_32x32x16_bf16, 128 f32 accumulators per lane;
//   * LDS: per stage an A and a B image of 64 k-rows x 512 B; two stages = 128 KB, one
//     workgroup per CU.  Rows are XOR-swizzled in 64-B chunks by (row & 3) -- applied to the
//     per-lane GLOBAL source address because LDS-DMA writes lane-linearly -- which makes every
//     32-lane half of a transposed read (4 k-rows x 64 B) hit 4 distinct chunks of the 256-B bank
//     row: conflict-free;
//   * pipeline: the DMA of tile t+1 is in flight while tile t is computed; the wait is a counted
//     `s_waitcnt vmcnt(8)` (never 0 inside the loop) + raw s_barrier, so the prefetch survives
//     the barrier (guide §5 "Pipelining across barriers");
//   * XCD-aware grouped tile order: each XCD (own 4 MB L2) works on a compact 8-row band of
//     output tiles so A/B k-panels are re-read from its L2;
//   * optional split-K for grids that would leave CUs idle (f32 slabs + a reduce kernel that
//     also performs the optional C += accumulation and the bf16 conversion).
#include "th_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

#ifndef TH_TN_GM
#define TH_TN_GM 8  // output-tile rows per XCD band in the ping-pong v2 order
#endif
namespace {
constexpr int TM = 256, TN = 256, TK = 64;
constexpr int NTHR = 512;
constexpr int ROWB = TN * 2;              // bytes per LDS k-row (TM == TN)
constexpr int OPB = TK * ROWB;            // 32 KB per operand image
constexpr int STAGEB = 2 * OPB;           // A + B
constexpr int LDSB = 2 * STAGEB;          // two stages = 128 KB
constexpr int GLDS_PER_OP = OPB / (NTHR * 16);  // 4 DMA instructions per lane per operand per stage

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// One 16-B LDS-DMA piece: lane-linear destination (wave-uniform LDS byte address `lds` in M0,
// + 16*lane), source = wave-uniform 64-bit base (SGPRs) + per-lane 32-bit byte offset.  Issued
// through inline asm on purpose: for the builtin, hipcc cannot tell which LDS bytes a DMA writes
// and puts `s_waitcnt vmcnt(0)` in front of every later ds_read, which drains the prefetch each
// k-tile.  The waits are placed by hand instead (counted vmcnt + s_barrier).
__device__ __forceinline__ void glds16(const void* sbase, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
}

__device__ __forceinline__ bf16x8 tr_pair(const char LDS_AS* p0, const char LDS_AS* p1) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)p0);
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)p1);
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N), fully expanded
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_tn(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_tn<I + 1, N>(f);
  }
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Stage k-rows [k0, k0+64) of a [K][ld] operand, columns [c0, c0+256), into a lane-linear LDS
// image whose (row, 64-B chunk c) holds global chunk c ^ (row & 3).  Wave-instruction u writes LDS
// bytes [u*1KB, +1KB) = rows 2u, 2u+1; a lane's byte offset from the wave-uniform row base depends
// on u only through the parity of u (row & 3 = (2(u&1) + (lane>>5)) & 3): two VGPRs per operand.
struct LaneOffs {
  unsigned o[2];
};
__device__ __forceinline__ LaneOffs lane_offs(long ld, long c0, int lane) {
  LaneOffs r;
  const int hi = lane >> 5, slot = lane & 31;
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int chunk = (slot >> 2) ^ ((2 * par + hi) & 3);
    r.o[par] = (unsigned)(2 * ((long)hi * ld + c0 + chunk * 32 + (slot & 3) * 8));
  }
  return r;
}
__device__ __forceinline__ void stage_op(const ushort* __restrict__ g, const LaneOffs& lo, long ld, long k0,
                                         unsigned img, int w, int nw) {
  // nw waves share the 32 wave-instructions of one operand image (8: all waves; 4: one group)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (nw == 8 && j == 1) continue;
      const int u = i * 8 + w + 4 * j;  // nw == 4: waves w and w+4's pieces
      const ushort* base = g + (k0 + 2 * u) * ld;
      glds16(base, lo.o[u & 1], img + u * 1024);
    }
  }
}
}  // namespace

template <bool SPLIT>
__global__ __launch_bounds__(NTHR, 1) void gemm_tn_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk,
    int beta) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDSB];
  char LDS_AS* smem = (char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = SPLIT ? L / splitk : L;
  const int split = SPLIT ? L % splitk : 0;
  // grouped order: bands of GM tile-rows, walked column-major inside a band
  constexpr int GM = 8;
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;        // wave tile: rows wm*128, cols wn*64
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / splitk;
  const long kbeg = (long)split * kper;
  const int nt = kper / TK;

  // transposed-read lane geometry: group g = lane>>4 (h = g>>1 picks k 0-7 / 8-15 of a k-step,
  // g&1 picks the 16-column half of a 32-column block); lane 4q+p addresses row q, cols 4p..4p+3
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lane_base = (8 * (g >> 1) + q) * ROWB + 32 * (g & 1) + 8 * p;
  int a_off[4], b_off[2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) a_off[mb] = lane_base + ((((wm * 128 + 32 * mb) >> 5) ^ q) << 6);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) b_off[nb] = lane_base + ((((wn * 64 + 32 * nb) >> 5) ^ q) << 6);

  f32x16 acc[4][2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16(0.f);

  // prologue: tiles 0 and 1 in flight
  const unsigned lds0 = (unsigned)(uintptr_t)smem;  // LDS byte address of the staging array
  const LaneOffs pa = lane_offs(lda, m0, lane), pb = lane_offs(ldb, n0, lane);
  stage_op(A, pa, lda, kbeg, lds0, w, 8);
  stage_op(B, pb, ldb, kbeg, lds0 + OPB, w, 8);
  if (nt > 1) {
    stage_op(A, pa, lda, kbeg + TK, lds0 + STAGEB, w, 8);
    stage_op(B, pb, ldb, kbeg + TK, lds0 + STAGEB + OPB, w, 8);
  }

  for (int t = 0; t < nt; ++t) {
    // tile t landed (this wave's DMAs), tile t+1 may stay in flight; the barrier publishes all waves'
    // (wait + barrier in ONE asm statement with a memory clobber: no LDS read can be scheduled
    // between them, or above them)
    if (t + 1 < nt) {
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const char LDS_AS* sa = smem + (t & 1) * STAGEB;
    const char LDS_AS* sb = sa + OPB;
#pragma unroll
    for (int ks = 0; ks < TK / 16; ++ks) {
      const int ko = ks * 16 * ROWB;  // k-step: rows 16ks .. 16ks+15
      bf16x8 af[4], bf[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) af[mb] = tr_pair(sa + a_off[mb] + ko, sa + a_off[mb] + ko + 4 * ROWB);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) bf[nb] = tr_pair(sb + b_off[nb] + ko, sb + b_off[nb] + ko + 4 * ROWB);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma(af[mb], bf[nb], acc[mb][nb]);
    }
    // every wave finished reading this stage before anyone restages it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 2 < nt) {
      const unsigned dst = lds0 + (t & 1) * STAGEB;
      stage_op(A, pa, lda, kbeg + (long)(t + 2) * TK, dst, w, 8);
      stage_op(B, pb, ldb, kbeg + (long)(t + 2) * TK, dst + OPB, w, 8);
    }
  }

  // epilogue: D[m][n] of block (mb, nb): n = col on the lane, m = accumulator row
  const int c32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const long n = n0 + wn * 64 + 32 * nb + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (SPLIT) {
          slab[((long)split * M + m) * N + n] = acc[mb][nb][r];
        } else {
          float v = acc[mb][nb][r];
          if (beta) v += bf2f(C[m * ldc + n]);
          C[m * ldc + n] = f2bf(v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong variant: the two wave groups (waves 0-3 = G0: rows 0-127 of the tile, waves 4-7 =
// G1: rows 128-255; each SIMD hosts one wave of each group) alternate roles every slot:
//   slot 2t   : G0 gathers ALL its fragments of k-tile t into registers (48 tr reads) and issues
//               the LDS-DMA of k-tile t+1;       G1 runs its 32 MFMAs of k-tile t-1
//   slot 2t+1 : G0 runs its 32 MFMAs of k-tile t; G1 gathers its fragments of k-tile t
// so each SIMD's matrix pipe is fed by one wave while its partner waits on LDS, instead of both
// waves stalling on the same barrier and the same LDS latency.  Slots end with a workgroup
// barrier; G1 enters one slot late (an extra barrier at the start, G0 one at the end).
//   * buffer reuse: k-tile t+1's DMA (slot 2t) overwrites the stage k-tile t-1 used; its last
//     reader (G1, slot 2t-1) retired its reads (lgkmcnt(0)) before that slot's barrier;
//   * visibility: G0 waits vmcnt(0) at the end of slot 2t+1, so k-tile t+1 is complete before the
//     barrier that opens slot 2t+2 (G0 reads) and slot 2t+3 (G1 reads).
template <bool SPLIT>
__global__ __launch_bounds__(NTHR, 1) void gemm_tn_pp_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk,
    int beta) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDSB];
  char LDS_AS* smem = (char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = SPLIT ? L / splitk : L;
  const int split = SPLIT ? L % splitk : 0;
  constexpr int GM = 8;
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const bool g1 = __builtin_amdgcn_readfirstlane(w) >= 4;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / splitk;
  const long kbeg = (long)split * kper;
  const int nt = kper / TK;

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lane_base = (8 * (g >> 1) + q) * ROWB + 32 * (g & 1) + 8 * p;
  int a_off[4], b_off[2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) a_off[mb] = lane_base + ((((wm * 128 + 32 * mb) >> 5) ^ q) << 6);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) b_off[nb] = lane_base + ((((wn * 64 + 32 * nb) >> 5) ^ q) << 6);

  f32x16 acc[4][2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16(0.f);

  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  const LaneOffs pa = lane_offs(lda, m0, lane), pb = lane_offs(ldb, n0, lane);
  // prologue: k-tile 0 staged by all 8 waves
  stage_op(A, pa, lda, kbeg, lds0, w, 8);
  stage_op(B, pb, ldb, kbeg, lds0 + OPB, w, 8);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (g1) asm volatile("s_barrier" ::: "memory");  // G1 enters one slot late

  bf16x8 af[4][4], bf[2][4];  // [block][k-step]
  for (int t = 0; t < nt; ++t) {
    // ---- gather slot
    if (!g1 && t + 1 < nt) {  // G0 stages k-tile t+1 (4 waves x 16 DMA pieces = 64 KB)
      const unsigned dst = lds0 + ((t + 1) & 1) * STAGEB;
      const long kt = kbeg + (long)(t + 1) * TK;
      stage_op(A, pa, lda, kt, dst, w, 4);
      stage_op(B, pb, ldb, kt, dst + OPB, w, 4);
    }
    const char LDS_AS* sa = smem + (t & 1) * STAGEB;
    const char LDS_AS* sb = sa + OPB;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int ko = ks * 16 * ROWB;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) af[mb][ks] = tr_pair(sa + a_off[mb] + ko, sa + a_off[mb] + ko + 4 * ROWB);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) bf[nb][ks] = tr_pair(sb + b_off[nb] + ko, sb + b_off[nb] + ko + 4 * ROWB);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- compute slot
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma(af[mb][ks], bf[nb][ks], acc[mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (!g1) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_barrier" ::: "memory");
    }
  }
  if (!g1) asm volatile("s_barrier" ::: "memory");  // match G1's extra barrier

  const int c32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const long n = n0 + wn * 64 + 32 * nb + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (SPLIT) {
          slab[((long)split * M + m) * N + n] = acc[mb][nb][r];
        } else {
          float v = acc[mb][nb][r];
          if (beta) v += bf2f(C[m * ldc + n]);
          C[m * ldc + n] = f2bf(v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong v2: k-tiles of 32 in a 4-stage LDS ring (4 x 32 KB).  The deeper ring lets each group
// stage its own operand two k-tiles ahead inside its own gather slot -- G0 the A image, G1 the B
// image -- so the LDS-DMA writes are spread over every slot instead of piling onto one group's
// gather slot (in the 2-stage schedule the even slots carried 96 KB of reads + 64 KB of DMA).
//   G0, iteration t: slot 2t   : DMA A(t+2); gather k-tile t       | barrier
//                    slot 2t+1 : 16 MFMAs of k-tile t; vmcnt -> A(t+1) landed | barrier
//   G1, iteration t: slot 2t+1 : DMA B(t+2); gather k-tile t; vmcnt -> B(t+1) landed | barrier
//                    slot 2t+2 : 16 MFMAs of k-tile t          | barrier
// Stage j%4 is rewritten (tile j+4) only 6 slots after its last reader; each wave's DMAs retire
// in issue order, so vmcnt(4) (one 4-piece DMA still in flight) retires the older tile.
constexpr int TK2 = 32;
constexpr int OPB2 = TK2 * ROWB;        // 16 KB
constexpr int STAGEB2 = 2 * OPB2;       // 32 KB
constexpr int NSTAGE2 = 4;

__device__ __forceinline__ void stage_op2(const ushort* __restrict__ g, const LaneOffs& lo, long ld, long k0,
                                          unsigned img, int w4) {
  // 16 wave-instructions (32 rows x 512 B) over the 4 waves of one group
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = i * 4 + w4;
    const ushort* base = g + (k0 + 2 * u) * ld;
    glds16(base, lo.o[u & 1], img + u * 1024);
  }
}

// SW images: 64-B chunk c of k-row r holds global chunk c ^ S(r), S(r) = (r + (r >> 3)) & 3, so rows 8
// apart (the two 16-lane groups of a half in the 16x16x32 operand read) land on different banks.
// Wave-instruction u = 4i + w4 writes rows 2u, 2u+1: S depends on the lane half, u & 1 (= w4 & 1)
// and i, so a wave needs one offset per i.
__device__ __forceinline__ unsigned lane_off_sw(long ld, long c0, int lane, int w4, int i) {
  const int hi = lane >> 5, slot = lane & 31;
  const int u = 4 * i + w4, row = 2 * u + hi;
  const int chunk = (slot >> 2) ^ ((row + (row >> 3)) & 3);
  return (unsigned)(2 * ((long)hi * ld + c0 + chunk * 32 + (slot & 3) * 8));
}
__device__ __forceinline__ void stage_op2_sw(const ushort* __restrict__ g, const unsigned (&lo)[4], long ld,
                                             long k0, unsigned img, int w4) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = i * 4 + w4;
    glds16(g + (k0 + 2 * u) * ld, lo[i], img + u * 1024);
  }
}

// vmcnt(4 * n) with n in 0..2 (immediate operand)
__device__ __forceinline__ void wait_dma_barrier(int n) {
  if (n >= 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

// AHEAD = how many k-tiles ahead each group's DMA runs (2: two slots of lead time per tile, 3: four;
// with 3 the stage a DMA overwrites was gathered one slot earlier, so G1 retires its reads
// (lgkmcnt(0)) before its gather slot ends)
// MI16: v_mfma_f32_16x16x32_bf16 instead of 32x32x16 (one k-step per 32-deep k-tile, 8 x 4 blocks of
// 16 x 16 per wave).  Operand of lane l: column (l & 15) of a 16-column block, k rows 8 (l >> 4) .. +7,
// one tr_pair (rows 8g + q and 8g + 4 + q of the 16-lane group g, columns 4p .. 4p + 3 of the block).
template <bool SPLIT, int AHEAD, bool MI16 = false, bool SW = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_tn_pp2_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk,
    int beta) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[NSTAGE2 * STAGEB2];
  char LDS_AS* smem = (char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = SPLIT ? L / splitk : L;
  const int split = SPLIT ? L % splitk : 0;
  constexpr int GM = TH_TN_GM;
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3, w4 = w & 3;
  const bool g1 = w >= 4;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / splitk;
  const long kbeg = (long)split * kper;
  const int nt = kper / TK2;

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lane_base = (8 * (g >> 1) + q) * ROWB + 32 * (g & 1) + 8 * p;
  // 32x32 operand rows 16 ks + 8h + q (+4): XOR q, or S = (q + 2 ks + h) & 3 with SW
  int a_off[4][2], b_off[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int x = SW ? (q + 2 * ks + (g >> 1)) & 3 : q;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) a_off[mb][ks] = lane_base + ((((wm * 128 + 32 * mb) >> 5) ^ x) << 6) + ks * 16 * ROWB;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) b_off[nb][ks] = lane_base + ((((wn * 64 + 32 * nb) >> 5) ^ x) << 6) + ks * 16 * ROWB;
  }
  // MI16 offsets: row 8g + q, 64-B chunk (col >> 5) ^ q, byte (col & 31) * 2 + 8p inside it
  const int lane_base16 = (8 * g + q) * ROWB + 8 * p;
  const int x16 = SW ? (q + g) & 3 : q;  // rows 8g + q (+4)
  int a_off16[8], b_off16[4];
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int col = wm * 128 + 16 * mb;
    a_off16[mb] = lane_base16 + (((col >> 5) ^ x16) << 6) + (col & 31) * 2;
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int col = wn * 64 + 16 * nb;
    b_off16[nb] = lane_base16 + (((col >> 5) ^ x16) << 6) + (col & 31) * 2;
  }

  f32x16 acc[MI16 ? 1 : 4][MI16 ? 1 : 2];
  f32x4 acc16[MI16 ? 8 : 1][MI16 ? 4 : 1];
  if constexpr (MI16) {
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc16[mb][nb] = f32x4(0.f);
  } else {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16(0.f);
  }

  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  const LaneOffs pa = lane_offs(lda, m0, lane), pb = lane_offs(ldb, n0, lane);
  unsigned pa_sw[4], pb_sw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pa_sw[i] = SW ? lane_off_sw(lda, m0, lane, w4, i) : 0u;
    pb_sw[i] = SW ? lane_off_sw(ldb, n0, lane, w4, i) : 0u;
  }
  auto stage_a = [&](long k0, unsigned img) {
    if (SW) stage_op2_sw(A, pa_sw, lda, k0, img, w4);
    else stage_op2(A, pa, lda, k0, img, w4);
  };
  auto stage_b = [&](long k0, unsigned img) {
    if (SW) stage_op2_sw(B, pb_sw, ldb, k0, img, w4);
    else stage_op2(B, pb, ldb, k0, img, w4);
  };
  // prologue: k-tiles 0 .. AHEAD-1 (A by G0, B by G1), all landed before the first slot
#pragma unroll
  for (int j = 0; j < AHEAD; ++j) {
    if (j < nt) {
      if (!g1) stage_a(kbeg + j * TK2, lds0 + j * STAGEB2);
      else stage_b(kbeg + j * TK2, lds0 + j * STAGEB2 + OPB2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (g1) asm volatile("s_barrier" ::: "memory");  // G1 enters one slot late

  bf16x8 af[4][2], bf[2][2];
  bf16x8 af16[MI16 ? 8 : 1], bf16[MI16 ? 4 : 1];
  for (int t = 0; t < nt; ++t) {
    // DMAs younger than k-tile t+1's that are in flight at the end of this iteration
    const int younger = min(AHEAD - 1, max(0, nt - 1 - (t + 1)));
    // ---- gather slot (+ this group's DMA AHEAD k-tiles ahead)
    if (t + AHEAD < nt) {
      const unsigned st = lds0 + ((t + AHEAD) & (NSTAGE2 - 1)) * STAGEB2;
      if (!g1) stage_a(kbeg + (long)(t + AHEAD) * TK2, st);
      else stage_b(kbeg + (long)(t + AHEAD) * TK2, st + OPB2);
    }
    const char LDS_AS* sa = smem + (t & (NSTAGE2 - 1)) * STAGEB2;
    const char LDS_AS* sb = sa + OPB2;
    if constexpr (MI16) {
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) af16[mb] = tr_pair(sa + a_off16[mb], sa + a_off16[mb] + 4 * ROWB);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) bf16[nb] = tr_pair(sb + b_off16[nb], sb + b_off16[nb] + 4 * ROWB);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) af[mb][ks] = tr_pair(sa + a_off[mb][ks], sa + a_off[mb][ks] + 4 * ROWB);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) bf[nb][ks] = tr_pair(sb + b_off[nb][ks], sb + b_off[nb][ks] + 4 * ROWB);
      }
    }
    if (g1) {  // G1's B image of k-tile t+1 must land before G0 gathers it (next slot)
      if (AHEAD >= 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_dma_barrier(younger);
    } else {
      asm volatile("s_barrier" ::: "memory");
    }
    // ---- compute slot
    if constexpr (MI16) {
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc16[mb][nb] = mfma16(af16[mb], bf16[nb], acc16[mb][nb]);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma(af[mb][ks], bf[nb][ks], acc[mb][nb]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!g1) {  // G0's A image of k-tile t+1 landed before the barrier that opens its gather
      wait_dma_barrier(younger);
    } else {
      asm volatile("s_barrier" ::: "memory");
    }
  }
  if (!g1) asm volatile("s_barrier" ::: "memory");

  if constexpr (MI16) {  // 16x16 result: lane l holds column (l & 15), rows 4 (l >> 4) + r
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const long n = n0 + wn * 64 + 16 * nb + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long m = m0 + wm * 128 + 16 * mb + 4 * (lane >> 4) + r;
          if (SPLIT) {
            slab[((long)split * M + m) * N + n] = acc16[mb][nb][r];
          } else {
            float v = acc16[mb][nb][r];
            if (beta) v += bf2f(C[m * ldc + n]);
            C[m * ldc + n] = f2bf(v);
          }
        }
      }
    return;
  }
  const int c32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const long n = n0 + wn * 64 + 32 * nb + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (SPLIT) {
          slab[((long)split * M + m) * N + n] = acc[mb][nb][r];
        } else {
          float v = acc[mb][nb][r];
          if (beta) v += bf2f(C[m * ldc + n]);
          C[m * ldc + n] = f2bf(v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// One wave per SIMD, 128 x 128 per wave (the shape hipBLASLt's fast kernels use on gfx950): 4 waves
// as 2 (M) x 2 (N), 256 f32 accumulators per lane (the compiler keeps them in AGPRs: a lone wave per
// SIMD owns the whole 512-entry register file), k-tiles of 32 in the 4-stage ring (DMA two k-tiles
// ahead, 8 pieces per wave per stage).  Twice the MFMAs per fragment of the 8-wave kernels: the
// LDS read traffic per FLOP drops by a third.  With no partner wave on the SIMD, latency is hidden
// inside the wave: the fragments of k-step s+1 are read while the MFMAs of k-step s run, and the
// k-tile boundary (counted vmcnt + barrier) sits between the two halves of the last k-step's MFMAs
// so the first reads of the next k-tile overlap 8 MFMAs already issued.
constexpr int W4_THR = 256;

__device__ __forceinline__ void stage_op_w4(const ushort* __restrict__ g, const LaneOffs& lo, long ld, long k0,
                                            unsigned img, int w) {
  // 16 wave-instructions (32 rows x 512 B) over 4 waves
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = i * 4 + w;
    const ushort* base = g + (k0 + 2 * u) * ld;
    glds16(base, lo.o[u & 1], img + u * 1024);
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(W4_THR, 1) void gemm_tn_w4_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk,
    int beta) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[NSTAGE2 * STAGEB2];
  char LDS_AS* smem = (char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = SPLIT ? L / splitk : L;
  const int split = SPLIT ? L % splitk : 0;
  constexpr int GM = 8;
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;  // wave tile: rows wm*128, cols wn*128
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / splitk;
  const long kbeg = (long)split * kper;
  const int nt = kper / TK2;

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lane_base = (8 * (g >> 1) + q) * ROWB + 32 * (g & 1) + 8 * p;
  int a_off[4], b_off[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a_off[j] = lane_base + ((((wm * 128 + 32 * j) >> 5) ^ q) << 6);
    b_off[j] = lane_base + ((((wn * 128 + 32 * j) >> 5) ^ q) << 6);
  }

  f32x16 acc[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = f32x16(0.f);

  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  const LaneOffs pa = lane_offs(lda, m0, lane), pb = lane_offs(ldb, n0, lane);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < nt) {
      stage_op_w4(A, pa, lda, kbeg + j * TK2, lds0 + j * STAGEB2, w);
      stage_op_w4(B, pb, ldb, kbeg + j * TK2, lds0 + j * STAGEB2 + OPB2, w);
    }
  }
  // k-tile 0 landed (k-tile 1 may stay in flight)
  if (nt > 1) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  auto read_step = [&](const char LDS_AS* st, int ks, bf16x8 (&af)[4], bf16x8 (&bf)[4]) {
    const char LDS_AS* sa = st;
    const char LDS_AS* sb = st + OPB2;
    const int ko = ks * 16 * ROWB;
#pragma unroll
    for (int j = 0; j < 4; ++j) af[j] = tr_pair(sa + a_off[j] + ko, sa + a_off[j] + ko + 4 * ROWB);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = tr_pair(sb + b_off[j] + ko, sb + b_off[j] + ko + 4 * ROWB);
  };

  bf16x8 a0[4], b0[4], a1[4], b1[4];
  read_step(smem, 0, a0, b0);
  for (int t = 0; t < nt; ++t) {
    const char LDS_AS* st = smem + (t & (NSTAGE2 - 1)) * STAGEB2;
    if (t + 2 < nt) {  // DMA two k-tiles ahead into the stage k-tile t-2 used
      const unsigned dst = lds0 + ((t + 2) & (NSTAGE2 - 1)) * STAGEB2;
      stage_op_w4(A, pa, lda, kbeg + (long)(t + 2) * TK2, dst, w);
      stage_op_w4(B, pb, ldb, kbeg + (long)(t + 2) * TK2, dst + OPB2, w);
    }
    // k-step 0 (fragments read before) while k-step 1's fragments are read
    read_step(st, 1, a1, b1);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma(a0[mb], b0[nb], acc[mb][nb]);
    // k-step 1, first half
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma(a1[mb], b1[nb], acc[mb][nb]);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) {
      // k-tile t+1 landed (t+2 may stay in flight); publish, then read its k-step 0 under the
      // second half of this k-step's MFMAs
      if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      read_step(smem + ((t + 1) & (NSTAGE2 - 1)) * STAGEB2, 0, a0, b0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mb = 2; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma(a1[mb], b1[nb], acc[mb][nb]);
  }

  const int c32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      // one 32x32 block at a time: the C loads of the beta path must not be hoisted for all 16
      // blocks at once (256 extra VGPRs next to the 256 accumulators)
      __builtin_amdgcn_sched_barrier(0);
      const long n = n0 + wn * 128 + 32 * nb + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (SPLIT) {
          slab[((long)split * M + m) * N + n] = acc[mb][nb][r];
        } else {
          float v = acc[mb][nb][r];
          if (beta) v += bf2f(C[m * ldc + n]);
          C[m * ldc + n] = f2bf(v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Schedule "hb" (launch flags bit 6): one wave per SIMD, the machine of hipBLASLt's NT kernels and of
// the NT kernel's hb schedule (removed in round 5: profiles/r05_gemm/gemm_nt_removed.patch), on the
// TN operands:
//   * tile 256 x 256 x 64, 4 waves as 2 (M) x 2 (N), wave tile 128 x 128 = 8 x 8 blocks of
//     v_mfma_f32_16x16x32_bf16 -> 64 f32x4 accumulators pinned in the 256 AGPRs by inline-asm MFMAs;
//   * per stage an A and a B image of 64 k-rows x 512 B (2-stage ring, 128 KB), k-row r's 64-B chunk c
//     at c ^ S(r), S(r) = (r + (r >> 3)) & 3 (the pp2 SW swizzle: both transposed reads of a 16x16x32
//     operand, rows 8 apart, conflict-free); an operand is one tr_pair (two ds_read_b64_tr_b16);
//   * DMA as buffer_load ... lds: the k-tile in the descriptor base, one loop-invariant soffset per
//     piece (2 k-rows = 1 KB), the lane's swizzled chunk in the voffset (4 per operand);
//   * one k-tile per iteration, synchronisation split per operand (released per operand, as in hipBLASLt's loop):
//       MFMA   0- 63  k-step 0 (fragments X);  0-15 read A's k-step-1 fragments (16 tr reads) | 20 barrier
//              22- 36 DMA A of tile t+2 (8 pieces);  23-38 read B's k-step-1 fragments       | 44 barrier
//              46- 74 DMA B of tile t+2 (8 pieces, every 4th MFMA)
//       MFMA  64-127  k-step 1 (Y); 88: vmcnt(16) + barrier (tile t+1 landed); 90-121 read X of tile t+1
//   * epilogue: bf16 through LDS with 16-B row stores (beta: C added), or f32x4 stores into the split-K slab.
template <bool SPLIT, bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_tn_hb_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk, int tile0,
    int GM) {
  constexpr int HIMG = 64 * ROWB;     // 32 KB: 64 k-rows x 256 columns
  constexpr int HSTAGE = 2 * HIMG;    // A | B
  __shared__ __attribute__((aligned(1024))) char smem_raw[2 * HSTAGE];
  const char LDS_AS* smem = (const char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = tile0 + (SPLIT ? L / splitk : L);
  const int split = SPLIT ? L % splitk : 0;
  // GM: output-tile rows per XCD band (runtime: launch flags bits 8-11, default TH_TN_GM)
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / splitk;
  const long kbeg = (long)split * kper;
  const int nt = kper / 64;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  // transposed-read offsets (16x16x32 operand of lane l: column l & 15 of a 16-column block, k rows
  // 8 (l >> 4) .. +7 as rows 8g + q and 8g + 4 + q, columns 4p .. 4p + 3 of each b64 half)
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lane_base16 = (8 * g + q) * ROWB + 8 * p;
  const int x16 = (q + g) & 3;
  int a_off[8], b_off[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    const int ca = wm * 128 + 16 * f, cb = wn * 128 + 16 * f;
    a_off[f] = lane_base16 + (((ca >> 5) ^ x16) << 6) + (ca & 31) * 2;
    b_off[f] = lane_base16 + (((cb >> 5) ^ x16) << 6) + (cb & 31) * 2;
  }
  // DMA: piece u = 4 i + w (i = 0..7) of an operand writes k-rows 2u, 2u + 1 (lane half hi); the
  // lane's global chunk is slot ^ S(row), S(row) = (2 w + hi + i) & 3 -> one voffset per i & 3
  const int hi = lane >> 5, slot = lane & 31;
  unsigned va[4], vb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = (slot >> 2) ^ ((2 * w + hi + i) & 3);
    va[i] = (unsigned)(2 * ((long)hi * lda + chunk * 32 + (slot & 3) * 8));
    vb[i] = (unsigned)(2 * ((long)hi * ldb + chunk * 32 + (slot & 3) * 8));
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem_raw;
  const ushort* ga = A + kbeg * lda + m0;
  const ushort* gb = B + kbeg * ldb + n0;
  auto piece = [&](int op, int i, int kt, int st) {
    const long ld = op == 0 ? lda : ldb;
    const ushort* base = (op == 0 ? ga : gb) + (long)kt * 64 * ld;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    const int u = 4 * i + w;
    const unsigned soff = (unsigned)(2L * 2 * u * ld);
    const unsigned voff = op == 0 ? va[i & 3] : vb[i & 3];
    const unsigned lb = __builtin_amdgcn_readfirstlane(lds0 + st * HSTAGE + op * HIMG + u * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(lb), "v"(voff), "s"(r), "s"(soff) : "memory", "m0");
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4(0.f);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4" ::);

#pragma unroll
  for (int i = 0; i < 8; ++i) piece(0, i, 0, 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) piece(1, i, 0, 0);
  const int kt1 = min(1, nt - 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) piece(0, i, kt1, 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) piece(1, i, kt1, 1);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  bf16x8 xa[8], xb[8], ya[8], yb[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    xa[f] = tr_pair(smem + a_off[f], smem + a_off[f] + 4 * ROWB);
    xb[f] = tr_pair(smem + HIMG + b_off[f], smem + HIMG + b_off[f] + 4 * ROWB);
  }
  auto mf = [&](f32x4& c, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  };
  // one transposed b64 half of fragment f (0-7 A, 8-15 B) of k-step ks, stage base sb
  auto rd_half = [&](const char LDS_AS* sb, int f, int ks, int half) -> i16x4 {
    const int off = (f < 8 ? a_off[f] : HIMG + b_off[f - 8]) + ks * 32 * ROWB + half * 4 * ROWB;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(sb + off));
  };
  auto join = [](i16x4 lo, i16x4 hi2) {
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi2[0], hi2[1], hi2[2], hi2[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  i16x4 lo_y = {0, 0, 0, 0}, lo_x = {0, 0, 0, 0};
  for (int t = 0; t < nt; ++t) {
    const int st = t & 1;
    const int kt2 = min(t + 2, nt - 1);  // past the end: re-stage the last tile (nobody reads it)
    const char LDS_AS* s_cur = smem + st * HSTAGE;
    const char LDS_AS* s_nxt = smem + (st ^ 1) * HSTAGE;
    static_for_tn<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      constexpr int mm = m & 63, i = mm >> 3, j = mm & 7;
      if constexpr (m < 64)
        mf(acc[i][j], xb[j], xa[i]);
      else
        mf(acc[i][j], yb[j], ya[i]);
      // Y.a: 16 halves at MFMAs 0-15
      if constexpr (m < 16) {
        if constexpr (!(m & 1)) lo_y = rd_half(s_cur, m >> 1, 1, 0);
        else ya[m >> 1] = join(lo_y, rd_half(s_cur, m >> 1, 1, 1));
      }
      if constexpr (m == 20) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (m >= 22 && m <= 36 && !(m & 1)) piece(0, (m - 22) / 2, kt2, st);
      // Y.b: 16 halves at MFMAs 23-38
      if constexpr (m >= 23 && m <= 38) {
        constexpr int h = m - 23;
        if constexpr (!(h & 1)) lo_y = rd_half(s_cur, 8 + (h >> 1), 1, 0);
        else yb[h >> 1] = join(lo_y, rd_half(s_cur, 8 + (h >> 1), 1, 1));
      }
      if constexpr (m == 44) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (m >= 46 && m <= 74 && ((m - 46) % 4 == 0)) piece(1, (m - 46) / 4, kt2, st);
      if constexpr (m == 88) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
      // X of tile t+1: 32 halves at MFMAs 90-121, A0 B0-B7 A1-A7 (the next iteration starts with row 0)
      if constexpr (m >= 90 && m <= 121) {
        constexpr int h = m - 90;
        constexpr int ord[16] = {0, 8, 9, 10, 11, 12, 13, 14, 15, 1, 2, 3, 4, 5, 6, 7};
        constexpr int f = ord[h >> 1];
        if constexpr (!(h & 1)) {
          lo_x = rd_half(s_nxt, f, 0, 0);
        } else {
          const bf16x8 v = join(lo_x, rd_half(s_nxt, f, 0, 1));
          if constexpr (f < 8) xa[f] = v;
          else xb[f - 8] = v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  // lane holds C[m = 16 i + r16][n = 16 j + 4 g4 .. +3] of the wave tile
  const int r16 = lane & 15, g4 = lane >> 4;
  const long crow0 = m0 + wm * 128, ccol0 = n0 + wn * 128;
  if constexpr (SPLIT) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4*>(slab + ((long)split * M + crow0 + 16 * i + r16) * N + ccol0 + 16 * j + 4 * g4) = acc[i][j];
    return;
  }
  char LDS_AS* ep = (char LDS_AS*)smem_raw + w * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4 v = acc[i][j];
      if constexpr (BETA) {
        const ushort4v old = *reinterpret_cast<const ushort4v*>(C + (crow0 + 16 * i + r16) * ldc + ccol0 + 16 * j + 4 * g4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bf2f(old[e]);
      }
      ushort4v o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      const int row = 16 * i + r16;
      const int blk = (2 * j + (g4 >> 1)) ^ r16;
      *reinterpret_cast<ushort4v LDS_AS*>(ep + row * 256 + blk * 16 + (g4 & 1) * 8) = o;
    }
  }
#pragma unroll
  for (int qq = 0; qq < 32; ++qq) {
    const int row = 4 * qq + g4;
    const ushort8 v = *reinterpret_cast<const ushort8 LDS_AS*>(ep + row * 256 + ((r16 ^ (row & 15)) << 4));
    *reinterpret_cast<ushort8*>(C + (crow0 + row) * ldc + ccol0 + 8 * r16) = v;
  }
}

// C[m][n] (+)= sum over splits of slab[s][m][n], 8 elements per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, ushort* __restrict__ C,
                                                             long ldc, int M, int N, int splitk, int beta) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;
  const long total8 = (long)M * N / 8;
  if (i8 >= total8) return;
  const long e = i8 * 8;
  const long m = e / N, n = e % N;
  float v[8];
  const float4v* s0 = reinterpret_cast<const float4v*>(slab + e);
  float4v x0 = s0[0], x1 = s0[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = x0[j]; v[4 + j] = x1[j]; }
  for (int s = 1; s < splitk; ++s) {
    const float4v* sp = reinterpret_cast<const float4v*>(slab + (long)s * M * N + e);
    x0 = sp[0];
    x1 = sp[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += x0[j]; v[4 + j] += x1[j]; }
  }
  ushort8* cp = reinterpret_cast<ushort8*>(C + m * ldc + n);
  ushort8 o;
  if (beta) {
    const ushort8 c = *cp;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] + bf2f(c[j]));
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  }
  *cp = o;
}

// Split-K remainder of the "data-parallel + split" launch: C tile (+)= sum over splits of its slab
// tiles, for the tiles [tile0, tile0 + gridDim.x) of the band order; one workgroup per tile.
__global__ __launch_bounds__(256) void splitk_reduce_tiles_kernel(const float* __restrict__ slab, ushort* __restrict__ C,
                                                                  long ldc, int M, int N, int splitk, int beta, int tile0,
                                                                  int GM) {
  const int nM = M / TM, nN = N / TN;
  const int tile = tile0 + blockIdx.x;
  const int per_band = GM * nN;
  const int band = tile / per_band, first_m = band * GM, gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const long m0 = (long)(first_m + in_band % gm) * TM, n0 = (long)(in_band / gm) * TN;
  for (int e = threadIdx.x * 8; e < TM * TN; e += 256 * 8) {
    const long m = m0 + e / TN, n = n0 + e % TN;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    for (int sp = 0; sp < splitk; ++sp) {
      const float4v* p = reinterpret_cast<const float4v*>(slab + ((long)sp * M + m) * N + n);
      const float4v x0 = p[0], x1 = p[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += x0[j]; v[4 + j] += x1[j]; }
    }
    ushort8* cp = reinterpret_cast<ushort8*>(C + m * ldc + n);
    ushort8 o;
    const ushort8 c = beta ? *cp : ushort8(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] + (beta ? bf2f(c[j]) : 0.f));
    *cp = o;
  }
}

// C[M][N] (+)= A[K][M]^T B[K][N]; A row stride lda, B ldb, C ldc (elements).  splitk > 1 needs a
// workspace of splitk*M*N floats.  Returns -1 for shapes the kernel does not tile.
// flags: bit0 = ping-pong schedule (gemm_tn_pp_kernel) instead of the lockstep 2-barrier loop;
//        bit1 = ping-pong v2 (k-tiles of 32, 4-stage ring, per-group DMA two k-tiles ahead);
//        bit2 (with bit1) = DMA three k-tiles ahead;
//        bit3 = one wave per SIMD, 128 x 128 per wave (gemm_tn_w4_kernel, 256 threads);
//        bit4 (with bit1) = v_mfma_f32_16x16x32_bf16 fragments in the ping-pong v2 kernel;
//        bit5 (with bit1) = row swizzle S(r) = (r + (r >> 3)) & 3 of the v2 images;
//        bit6 = schedule "hb" (gemm_tn_hb_kernel: one wave per SIMD, 16x16x32 asm MFMAs, per-operand barriers);
//        bit7 (with bit6, splitk > 1) = data-parallel whole tiles + split-K only for the remainder tiles;
//        bits 8-11 (with bit6) = XCD band height in tile rows (0 = TH_TN_GM)
extern "C" int th_gemm_tn(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                          int K, int beta, int splitk, float* ws, int flags, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || splitk < 1 || K % (TK * splitk)) return -1;
  const bool pp2 = flags & 2;
  if (lda < M || ldb < N || ldc < N || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return -1;
  if (splitk > 1 && ws == nullptr) return -1;
  const long tiles = (long)(M / TM) * (N / TN);
  const bool pp = flags & 1;
  const unsigned grid = (unsigned)(tiles * splitk);
  const ushort *a = (const ushort*)A, *b = (const ushort*)B;
  ushort* c = (ushort*)C;
  float* slab = splitk > 1 ? ws : nullptr;
#define TH_TN_LAUNCH(KERNEL)                                                                     \
  do {                                                                                          \
    if (splitk > 1) KERNEL<true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta); \
    else KERNEL<false><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);             \
  } while (0)
#define TH_TN_LAUNCH2(KERNEL, AH)                                                                \
  do {                                                                                          \
    if ((flags & 48) == 48) {                                                                   \
      if (splitk > 1) KERNEL<true, AH, true, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta); \
      else KERNEL<false, AH, true, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);             \
    } else if (flags & 32) {                                                                    \
      if (splitk > 1) KERNEL<true, AH, false, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta); \
      else KERNEL<false, AH, false, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);             \
    } else if (flags & 16) {                                                                    \
      if (splitk > 1) KERNEL<true, AH, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta); \
      else KERNEL<false, AH, true><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);             \
    } else if (splitk > 1) KERNEL<true, AH><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta); \
    else KERNEL<false, AH><<<grid, NTHR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);             \
  } while (0)
  if (flags & 64) {  // schedule "hb": one wave per SIMD, 64-deep k-tiles
    const int gmr = ((flags >> 8) & 15) ? ((flags >> 8) & 15) : TH_TN_GM;  // XCD band height (tile rows)
    if (K / splitk < 64 || (K / splitk) % 64) return -1;
    // buffer descriptors per k-tile: 32-bit offsets over 64 k-rows of one operand
    if (2L * 64 * max(lda, ldb) + 512 >= (1L << 31)) return -1;
    // flags bit7 with splitk > 1: data-parallel rounds of whole tiles on every CU (direct bf16 output),
    // then only the REMAINDER tiles split `splitk` ways (slab + a per-tile reduce): no split-K slab
    // round trip for the bulk of the tiles and no half-empty last round
    const long cus = 256;
    const long full = (flags & 128) && splitk > 1 ? tiles / cus * cus : 0;
    const long rem = tiles - full;
    if (full > 0 && rem * splitk <= cus) {
      if (beta) gemm_tn_hb_kernel<false, true><<<(unsigned)full, 256, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, 0, gmr);
      else gemm_tn_hb_kernel<false, false><<<(unsigned)full, 256, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, 0, gmr);
      if (rem > 0) {
        gemm_tn_hb_kernel<true, false><<<(unsigned)(rem * splitk), 256, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K,
                                                                                splitk, (int)full, gmr);
        splitk_reduce_tiles_kernel<<<(unsigned)rem, 256, 0, s>>>(ws, c, ldc, M, N, splitk, beta, (int)full, gmr);
      }
      TH_CHECK_LAUNCH();
    }
    if (splitk > 1) gemm_tn_hb_kernel<true, false><<<grid, 256, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, 0, gmr);
    else if (beta) gemm_tn_hb_kernel<false, true><<<grid, 256, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, 0, gmr);
    else gemm_tn_hb_kernel<false, false><<<grid, 256, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, 0, gmr);
  } else if (flags & 8) {
    if (splitk > 1) gemm_tn_w4_kernel<true><<<grid, W4_THR, 0, s>>>(a, lda, b, ldb, c, ldc, slab, M, N, K, splitk, beta);
    else gemm_tn_w4_kernel<false><<<grid, W4_THR, 0, s>>>(a, lda, b, ldb, c, ldc, nullptr, M, N, K, 1, beta);
  } else if (pp2 && (flags & 4)) TH_TN_LAUNCH2(gemm_tn_pp2_kernel, 3);
  else if (pp2) TH_TN_LAUNCH2(gemm_tn_pp2_kernel, 2);
  else if (pp) TH_TN_LAUNCH(gemm_tn_pp_kernel);
  else TH_TN_LAUNCH(gemm_tn_kernel);
#undef TH_TN_LAUNCH
#undef TH_TN_LAUNCH2
  if (splitk > 1) {
    const long n8 = (long)M * N / 8;
    splitk_reduce_kernel<<<(unsigned)((n8 + 255) / 256), 256, 0, s>>>(ws, c, ldc, M, N, splitk, beta);
  }
  TH_CHECK_LAUNCH();
}
