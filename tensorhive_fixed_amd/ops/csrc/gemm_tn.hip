// Weight-gradient GEMM in the layout training produces, for gfx950 (MI355X):
//
//     C[M][N] (+)= sum_k A[k][M] * B[k][N]        (dW = dY^T X, k = tokens)
//
// A = dY [tokens][out] and B = X [tokens][in] are both row-major with the reduction index as
// the SLOW dimension.  hipBLASLt runs this "TN" form at 1.0-1.2 PFLOP/s on the Llama-3-8B
// shapes against 1.4-1.6 for the K-contiguous forms (profiles/r01_gemm/); the K-contiguous form
// needs two transposes of activation-sized operands first.  This kernel reads the operands as
// they are: k-rows are staged with LDS-DMA (buffer_load ... lds) and the MFMA operands are gathered
// column-wise with the hardware transpose read ds_read_b64_tr_b16.
//
// One schedule ("hb", gemm_tn_hb_kernel below): 256 x 256 x 64 tiles on one wave per SIMD, the loop shape
// of hipBLASLt's gfx950 MT256x256x64 kernels.  One grid per launch: whole-K tiles first, then split-K
// pieces of the remaining tiles into an f32 slab of those tiles + a per-tile reduce (all whole, all split,
// or the mix ops/gemm_tn.py:tn_plan picks for the CUs the launch may meet).  Output tiles run in XCD bands
// (each XCD's 4 MB L2 re-reads a compact band's k-panels).  The round-1..4 schedules
// (8-wave lockstep / ping-pong, 32-deep ring, 128 x 128 waves) were retired in round 5 after hb beat
// them on every shape: profiles/r05_gemm/ (gemm_tn_old_modes_removed.patch restores them).
#include "th_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

#ifndef TH_TN_GM
#define TH_TN_GM 8  // output-tile rows per XCD band
#endif
#ifndef TH_TN_A0  // DMA piece slots: A's 8 at a0 + as * k (after the barrier at 20), B's at b0 + bs * k (after 44)
#define TH_TN_A0 22
#endif
#ifndef TH_TN_AS
#define TH_TN_AS 4
#endif
#ifndef TH_TN_B0
#define TH_TN_B0 52
#endif
#ifndef TH_TN_BS
#define TH_TN_BS 5
#endif
#ifndef TH_TN_ONEBAR
#define TH_TN_ONEBAR 0  // one WAR barrier per k-tile instead of two (A's and B's stage released together)
#endif
#ifndef TH_TN_RSRC
#define TH_TN_RSRC 1  // main-loop buffer descriptors as raw words advanced in place
#endif
#ifndef TH_TN_M0SPLIT
// main-loop LDS-DMA pieces: M0 written before the gap's MFMA, load after it (307 -> 282 loop instructions;
// wqkv / wo / w2 / w13 1.185 / 0.740 / 2.656 / 5.471 -> 1.168 / 0.732 / 2.614 / 5.417 ms, alternating processes
// on one box: profiles/r06_gemm/tn_m0split/)
#define TH_TN_M0SPLIT 1
#endif

constexpr int TM = 256, TN = 256;
constexpr int ROWB = TN * 2;  // bytes per LDS k-row (TM == TN)

// workgroup id -> launch-order index such that consecutive indices sit on one XCD (blockIdx.x mod 8)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ bf16x8 tr_pair(const char LDS_AS* p0, const char LDS_AS* p1) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)p0);
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)p1);
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N), fully expanded
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_tn(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_tn<I + 1, N>(f);
  }
}
// Diagnostic build only (-DTH_TN_DIAG=1: scripts/build_variant_lib.sh tn_diag -DTH_TN_DIAG=1 gemm_tn,
// scripts/tn_stamps.py): s_memtime stamps around the three waits of each k-tile, summed per wave and added
// into g_tn_stamp = {k-tiles, whole loop, barrier 20, barrier 44, vmcnt + barrier 88} (shader cycles).
// The production libthk.so has none of it.
#ifdef TH_TN_DIAG
__device__ unsigned long long g_tn_stamp[8];
__device__ __forceinline__ unsigned long long tn_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
constexpr bool kTnDiag = true;
#else
__device__ __forceinline__ unsigned long long tn_stamp() { return 0; }
constexpr bool kTnDiag = false;
#endif

// ---------------------------------------------------------------------------------------------
// Schedule "hb": one wave per SIMD, the machine of hipBLASLt's NT kernels (and of the NT kernel's hb
// schedule, removed in round 5: profiles/r05_gemm/gemm_nt_removed.patch), on the TN operands:
//   * tile 256 x 256 x 64, 4 waves as 2 (M) x 2 (N), wave tile 128 x 128 = 8 x 8 blocks of
//     v_mfma_f32_16x16x32_bf16 -> 64 f32x4 accumulators pinned in the 256 AGPRs by inline-asm MFMAs;
//   * per stage an A and a B image of 64 k-rows x 512 B (2-stage ring, 128 KB), k-row r's 64-B chunk c
//     at c ^ S(r), S(r) = (r + (r >> 3)) & 3 (both transposed reads of a 16x16x32 operand, rows 8 apart,
//     conflict-free); an operand is one tr_pair (two ds_read_b64_tr_b16);
//   * DMA as buffer_load ... lds: the k-tile in the descriptor base, one loop-invariant soffset per
//     piece (2 k-rows = 1 KB), the lane's swizzled chunk in the voffset (4 per operand);
//   * one k-tile per iteration, synchronisation split per operand (released per operand, as in hipBLASLt's loop):
//       MFMA   0- 63  k-step 0 (fragments X);  0-15 read A's k-step-1 fragments (16 tr reads) | 20 barrier
//              22- 50 DMA A of tile t+2 (8 pieces, every 4th MFMA);  23-38 read B's k-step-1 fragments
//              | 44 barrier;  52- 87 DMA B of tile t+2 (8 pieces, every 5th MFMA)
//       MFMA  64-127  k-step 1 (Y); 88: vmcnt(16) + barrier (tile t+1 landed); 90-121 read X of tile t+1
//   * epilogue: bf16 through LDS with 16-B row stores (beta: C added), or f32x4 stores into the split-K slab.
//   * one grid holds both kinds of workgroup (round 6): the first `full` workgroups are whole-K tiles
//     0 .. full-1, the rest are `splitk` K-pieces of each remaining tile (into the slab; a reduce follows).
//     The dispatcher starts workgroups in grid order, so on an idle chip the pieces fill the CUs the whole
//     tiles leave free, and with CUs held by RCCL's channels the pieces still trail one short round --
//     instead of the whole-tile round spilling a few tiles into a second full round.  Each part gets its
//     own XCD remap, so consecutive tiles of a part share an XCD's L2.
template <bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_tn_hb_kernel(
    const ushort* __restrict__ A, long lda, const ushort* __restrict__ B, long ldb,
    ushort* __restrict__ C, long ldc, float* __restrict__ slab, int M, int N, int K, int splitk, int full,
    int GM) {
  constexpr int HIMG = 64 * ROWB;     // 32 KB: 64 k-rows x 256 columns
  constexpr int HSTAGE = 2 * HIMG;    // A | B
  __shared__ __attribute__((aligned(1024))) char smem_raw[2 * HSTAGE];
  const char LDS_AS* smem = (const char LDS_AS*)smem_raw;
  const int nM = M / TM, nN = N / TN;
  const int bid = blockIdx.x;
  const bool is_piece = bid >= full;  // uniform per workgroup
  const int L = is_piece ? xcd_remap(bid - full, (int)gridDim.x - full) : xcd_remap(bid, full);
  const int sk = is_piece ? splitk : 1;
  const int tile = is_piece ? full + L / splitk : L;
  const int split = is_piece ? L % splitk : 0;
  // GM: output-tile rows per XCD band (runtime: launch flags bits 8-11, default TH_TN_GM)
  const int per_band = GM * nN;
  const int band = tile / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = tile % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const int kper = K / sk;
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
  // LDS image of operand op (0 A, 1 B) in stage st: A0 | A1 | B0 | B1, 32 KB each, so the stage and operand
  // parts of every read address are compile-time immediates below 64 KB in the two-stage unrolled loop
  auto img = [](int op, int st) { return op * 2 * HIMG + st * HIMG; };
  // piece i of operand op of the k-tile whose first k-row is at `base`, into stage st
  auto piece_at = [&](int op, int i, const ushort* base, int st) {
    const long ld = op == 0 ? lda : ldb;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    const int u = 4 * i + w;
    const unsigned soff = (unsigned)(2L * 2 * u * ld);
    const unsigned voff = op == 0 ? va[i & 3] : vb[i & 3];
    const unsigned lb = __builtin_amdgcn_readfirstlane(lds0 + img(op, st) + u * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(lb), "v"(voff), "s"(r), "s"(soff) : "memory", "m0");
  };
  auto piece = [&](int op, int i, int kt, int st) {
    piece_at(op, i, (op == 0 ? ga : gb) + (long)kt * 64 * (op == 0 ? lda : ldb), st);
  };
  // TH_TN_M0SPLIT: a main-loop piece in two halves -- M0 (this wave's LDS slot of the piece) written by one
  // s_add straight into m0 BEFORE the MFMA of that gap, the buffer_load after it, so the MFMA is the
  // wait state the M0 write needs (no s_mov / s_nop per piece: 32 fewer scalar issues per k-tile)
  const unsigned lds_w = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)w * 1024u);
  // TH_TN_RSRC: the main loop's buffer descriptors kept as raw words (base lo / hi advanced by one 32-bit
  // add with carry per operand and k-tile) instead of a pointer advance + clamp + rebuilt descriptor
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  auto piece_load_w = [&](int op, int i, unsigned long long base) {
    const long ld = op == 0 ? lda : ldb;
    const i32x4 r = {(int)(unsigned)base, (int)(unsigned)(base >> 32), 0x7fffffff, 0x00020000};
    const unsigned soff = (unsigned)(2L * 2 * (4 * i + w) * ld);
    const unsigned voff = op == 0 ? va[i & 3] : vb[i & 3];
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(voff), "s"(r), "s"(soff) : "memory");
  };
  auto piece_load = [&](int op, int i, const ushort* base) {
    const long ld = op == 0 ? lda : ldb;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    const unsigned soff = (unsigned)(2L * 2 * (4 * i + w) * ld);
    const unsigned voff = op == 0 ? va[i & 3] : vb[i & 3];
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(voff), "s"(r), "s"(soff) : "memory");
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
    xa[f] = tr_pair(smem + img(0, 0) + a_off[f], smem + img(0, 0) + a_off[f] + 4 * ROWB);
    xb[f] = tr_pair(smem + img(1, 0) + b_off[f], smem + img(1, 0) + b_off[f] + 4 * ROWB);
  }
  auto mf = [&](f32x4& c, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  };
  // one transposed b64 half of fragment f (0-7 A, 8-15 B) of k-step ks in stage st (a constant in the loop)
  auto rd_half = [&](int st, int f, int ks, int half) -> i16x4 {
    const int off = (f < 8 ? a_off[f] : b_off[f - 8]) + img(f < 8 ? 0 : 1, st) + ks * 32 * ROWB + half * 4 * ROWB;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(smem + off));
  };
  auto join = [](i16x4 lo, i16x4 hi2) {
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi2[0], hi2[1], hi2[2], hi2[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  i16x4 lo_y = {0, 0, 0, 0}, lo_x = {0, 0, 0, 0};
  unsigned long long d_loop = 0, d_w[3] = {0, 0, 0}, d_t = 0;
  if constexpr (kTnDiag) d_loop = tn_stamp();
  // k-tile t+2's first rows, advanced incrementally (no 64-bit multiply per k-tile); past the end the last
  // tile is re-staged (nobody reads it)
  const ushort* pa2 = ga + (long)min(2, nt - 1) * 64 * lda;
  const ushort* pb2 = gb + (long)min(2, nt - 1) * 64 * ldb;
  unsigned long long ra2 = (unsigned long long)(uintptr_t)pa2, rb2 = (unsigned long long)(uintptr_t)pb2;
  const unsigned step_a = 128u * (unsigned)lda, step_b = 128u * (unsigned)ldb;  // bytes per k-tile
  // k-tile t in stage ST = t & 1, unrolled per stage (two k-tiles per trip, plus an even tail tile)
  auto ktile = [&](auto stc) {
    constexpr int ST = decltype(stc)::value;
    static_for_tn<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      constexpr int mm = m & 63, i = mm >> 3, j = mm & 7;
      // DMA pieces spread over the whole k-tile: A's 8 every 4th MFMA from 22 (after the barrier that
      // releases A), B's 8 every 5th from 52 (after B's barrier at 44), the last one before the vmcnt at 88
      // (2 % faster than A every 2nd from 22 and B every 4th from 46: profiles/r05_gemm/tn_pv_sweep*.jsonl)
      // TH_TN_ONEBAR: Y.b read right after Y.a, ONE barrier (34) releases both operands' stage, then the DMA
      constexpr int a0 = TH_TN_ONEBAR ? 36 : TH_TN_A0, as = TH_TN_ONEBAR ? 3 : TH_TN_AS,
                    b0 = TH_TN_ONEBAR ? 59 : TH_TN_B0, bs = TH_TN_ONEBAR ? 4 : TH_TN_BS;
      constexpr int yb0 = TH_TN_ONEBAR ? 16 : 23, bar1 = TH_TN_ONEBAR ? 34 : 20, bar2 = TH_TN_ONEBAR ? -1 : 44;
      static_assert(a0 > bar1 && a0 + 7 * as < b0 && b0 > (TH_TN_ONEBAR ? bar1 : bar2) && b0 + 7 * bs < 88 &&
                    (TH_TN_ONEBAR == 0 || yb0 + 15 < bar1), "TN DMA slots");
      constexpr bool pa = m >= a0 && m < a0 + 8 * as && (m - a0) % as == 0;
      constexpr bool pb = m >= b0 && m < b0 + 8 * bs && (m - b0) % bs == 0;
      constexpr int pi = pa ? (m - a0) / as : (pb ? (m - b0) / bs : 0);
      constexpr int poff = (pb ? 2 * HIMG : 0) + ST * HIMG + 4096 * pi;  // piece 4 pi + w of A / B in stage ST
      if constexpr (TH_TN_M0SPLIT && (pa || pb))
        asm volatile("s_add_i32 m0, %0, %1" :: "s"(lds_w), "n"(poff) : "m0");
      if constexpr (m < 64)
        mf(acc[i][j], xb[j], xa[i]);
      else
        mf(acc[i][j], yb[j], ya[i]);
      // Y.a: 16 halves at MFMAs 0-15
      if constexpr (m < 16) {
        if constexpr (!(m & 1)) lo_y = rd_half(ST, m >> 1, 1, 0);
        else ya[m >> 1] = join(lo_y, rd_half(ST, m >> 1, 1, 1));
      }
      if constexpr (kTnDiag && (m == 20 || m == 44 || m == 88)) d_t = tn_stamp();
      if constexpr (m == bar1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (pa) {
        if constexpr (TH_TN_M0SPLIT && TH_TN_RSRC) piece_load_w(0, pi, ra2);
        else if constexpr (TH_TN_M0SPLIT) piece_load(0, pi, pa2);
        else piece_at(0, pi, pa2, ST);
      }
      // Y.b: 16 halves at MFMAs 23-38
      if constexpr (m >= yb0 && m <= yb0 + 15) {
        constexpr int h = m - yb0;
        if constexpr (!(h & 1)) lo_y = rd_half(ST, 8 + (h >> 1), 1, 0);
        else yb[h >> 1] = join(lo_y, rd_half(ST, 8 + (h >> 1), 1, 1));
      }
      if constexpr (m == bar2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (pb) {
        if constexpr (TH_TN_M0SPLIT && TH_TN_RSRC) piece_load_w(1, pi, rb2);
        else if constexpr (TH_TN_M0SPLIT) piece_load(1, pi, pb2);
        else piece_at(1, pi, pb2, ST);
      }
      if constexpr (m == 88) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
      if constexpr (kTnDiag && (m == 20 || m == 44 || m == 88)) d_w[m == 20 ? 0 : m == 44 ? 1 : 2] += tn_stamp() - d_t;
      // X of tile t+1: 32 halves at MFMAs 90-121, A0 B0-B7 A1-A7 (the next iteration starts with row 0)
      if constexpr (m >= 90 && m <= 121) {
        constexpr int h = m - 90;
        constexpr int ord[16] = {0, 8, 9, 10, 11, 12, 13, 14, 15, 1, 2, 3, 4, 5, 6, 7};
        constexpr int f = ord[h >> 1];
        if constexpr (!(h & 1)) {
          lo_x = rd_half(ST ^ 1, f, 0, 0);
        } else {
          const bf16x8 v = join(lo_x, rd_half(ST ^ 1, f, 0, 1));
          if constexpr (f < 8) xa[f] = v;
          else xb[f - 8] = v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  int t = 0;
  auto advance = [&]() {  // k-tile t+2's first rows for the next k-tile's DMA
    if constexpr (TH_TN_RSRC) {
      const bool more = t + 3 < nt;  // past the end the last k-tile is re-staged (nobody reads it)
      ra2 += more ? step_a : 0u;
      rb2 += more ? step_b : 0u;
    } else if (t + 3 < nt) {
      pa2 += 64 * lda;
      pb2 += 64 * ldb;
    }
    ++t;
  };
  for (; t + 1 < nt;) {
    ktile(std::integral_constant<int, 0>{});
    advance();
    ktile(std::integral_constant<int, 1>{});
    advance();
  }
  if (t < nt) {  // odd k-tile count: the last one sits in stage 0
    ktile(std::integral_constant<int, 0>{});
    advance();
  }
#ifdef TH_TN_DIAG
  if (lane == 0) {
    const unsigned long long loop = tn_stamp() - d_loop;
    atomicAdd(&g_tn_stamp[0], (unsigned long long)nt);
    atomicAdd(&g_tn_stamp[1], loop);
    for (int i = 0; i < 3; ++i) atomicAdd(&g_tn_stamp[2 + i], d_w[i]);
  }
#endif
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  // lane holds C[m = 16 i + r16][n = 16 j + 4 g4 .. +3] of the wave tile
  const int r16 = lane & 15, g4 = lane >> 4;
  const long crow0 = m0 + wm * 128, ccol0 = n0 + wn * 128;
  // (with both epilogues in one kernel the compiler spills 3-4 accumulators around the bf16 path's
  // conversion: 36-68 B of scratch per lane, after the main loop only)
  if (is_piece) {
    // tile-local slab: [split tile][split][256][256] f32, so a launch needs split tiles * splitk * 64 K floats
    float* ts = slab + ((long)(tile - full) * splitk + split) * (TM * TN) + (wm * 128) * TN + wn * 128;
    // stored straight from the AGPRs
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(ts + (16 * i + r16) * TN + 16 * j + 4 * g4),
                     "a"(acc[i][j]) : "memory");
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

// Split-K reduce: C tile (+)= sum over splits of its tile-local slab pieces, for the tiles
// [tile0, tile0 + gridDim.x) of the band order (all tiles, or the remainder of the data-parallel launch);
// one workgroup per tile.
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
      const float4v* p = reinterpret_cast<const float4v*>(slab + ((long)blockIdx.x * splitk + sp) * (TM * TN) + e);
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

// C[M][N] (+)= A[K][M]^T B[K][N]; A row stride lda, B ldb, C ldc (elements).  One launch: the first
// `full` tiles (band order) whole-K, the remaining tiles split `splitk` ways into the f32 workspace
// (ws_floats >= (tiles - full) * splitk * 64 K; ops/gemm_tn.py:tn_plan picks full / splitk for the CUs the
// launch may meet), then one reduce workgroup per split tile.  Returns -1 for shapes the kernel does not
// tile or a workspace that is too small.
// flags: bit6 = schedule "hb" (required; the only schedule since round 5);
//        bits 8-11 = XCD band height in tile rows (0 = TH_TN_GM)
extern "C" int th_gemm_tn(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                          int K, int beta, int splitk, int full, float* ws, long ws_floats, int flags,
                          hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || splitk < 1 || !(flags & 64)) return -1;
  if (K % (64 * splitk)) return -1;
  if (lda < M || ldb < N || ldc < N || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return -1;
  // buffer descriptors per k-tile: 32-bit offsets over 64 k-rows of one operand
  if (2L * 64 * max(lda, ldb) + 512 >= (1L << 31)) return -1;
  const long tiles = (long)(M / TM) * (N / TN);
  if (full < 0 || full > tiles || (splitk == 1 && full != tiles)) return -1;
  const long split_tiles = tiles - full;
  if (split_tiles > 0 && (ws == nullptr || ws_floats < split_tiles * splitk * (long)(TM * TN))) return -1;
  const int gmr = ((flags >> 8) & 15) ? ((flags >> 8) & 15) : TH_TN_GM;  // XCD band height (tile rows)
  const unsigned grid = (unsigned)(full + split_tiles * splitk);
  if (beta)  // whole tiles add C in their epilogue; the pieces never read C (the reduce adds it)
    gemm_tn_hb_kernel<true><<<grid, 256, 0, s>>>((const ushort*)A, lda, (const ushort*)B, ldb, (ushort*)C, ldc, ws,
                                                 M, N, K, splitk, full, gmr);
  else
    gemm_tn_hb_kernel<false><<<grid, 256, 0, s>>>((const ushort*)A, lda, (const ushort*)B, ldb, (ushort*)C, ldc, ws,
                                                  M, N, K, splitk, full, gmr);
  if (split_tiles > 0)
    splitk_reduce_tiles_kernel<<<(unsigned)split_tiles, 256, 0, s>>>(ws, (ushort*)C, ldc, M, N, splitk, beta, full,
                                                                     gmr);
  TH_CHECK_LAUNCH();
}

#ifdef TH_TN_DIAG
// g_tn_stamp -> buf[8]; reset != 0 zeroes it instead
extern "C" int th_tn_stamps(unsigned long long* buf, int reset) {
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tn_stamp), z, sizeof z) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_tn_stamp), 8 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif
