// K-contiguous ("NT") GEMM for gfx950 (MI355X), the layout of the forward and input-gradient
// products of every Llama linear layer:
//
//     C[M][N] (+)= sum_k A[M][k] * B[N][k]        (y = x W^T;  dX = dY (W^T)^T on a W^T copy)
//
// One wave per SIMD, the machine hipBLASLt's MT256x256x64_MI16x16 kernel is (profiles/r03_gemm:
// 83.7 % MFMA busy, one wave per SIMD), with the register allocation taken away from the compiler:
//   * workgroup tile 256 x 256, k-tiles of 64, 4 waves as 2 (M) x 2 (N), wave tile 128 x 128 =
//     8 x 8 blocks of v_mfma_f32_16x16x32_bf16 -> 64 f32x4 accumulators = all 256 AGPRs.  Every
//     MFMA is an inline-asm statement whose accumulator operand is "+a": the accumulators live in
//     the accumulator file for the whole kernel and hipcc has nothing to shuffle (round 3's HIP
//     version of this machine spent 3.2x hipBLASLt's VALU on v_accvgpr moves and ran 0.58-0.67x);
//   * A and B images of a k-tile (256 rows x 128 B each) are staged by LDS-DMA
//     (global_load_lds_dwordx4) into a 2-stage ring (128 KB); 16-B chunk c of image row r lands in
//     slot c ^ ((r >> 1) & 7), applied on the global source because the DMA writes lane-linearly.
//     An MFMA operand is ONE ds_read_b128 (16 rows x 4 chunks); under this swizzle a 16-lane group
//     hits 16 distinct 16-B slots of the bank row: conflict-free;
//   * each k-tile is two phases of 64 MFMAs (k 0-31, k 32-63).  Phase A computes half 0 while it
//     reads half 1's 16 fragments; one barrier (after this wave's DMA of the next tile retired)
//     makes the next tile visible; phase B computes half 1 while it reads the NEXT tile's half 0
//     and issues this wave's 16 DMA pieces of the tile after that into the stage just freed.  So
//     fragments are always one phase ahead, DMA one tile ahead, one barrier per k-tile, and the
//     LDS reads / DMA issues sit in the MFMA shadow (one read per 4 MFMAs);
//   * the MFMA runs with the operands swapped (B block as "A"), so a lane holds 4 consecutive
//     columns of one output row; the epilogue goes through LDS (per wave, no barrier) and leaves
//     as 16-B row stores;
//   * XCD-aware grouped tile order (bands of 8 tile rows per XCD).
// Round 3's ping-pong NT kernel (2 waves per SIMD, 0.77-0.86x hipBLASLt) is in git history.
#include "th_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

namespace {
constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;
constexpr int IMG = BM * BK * 2;   // 32 KB per operand image
constexpr int STAGE = 2 * IMG;     // A | B
constexpr int SMEM = 2 * STAGE;    // 128 KB

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// one LDS-DMA piece: 64 lanes x 16 B from (sbase + voff) into LDS [lds, lds + 1 KB)
template <bool NOP>
__device__ __forceinline__ void glds16(const void* sbase, unsigned voff, unsigned lds) {
  if (NOP)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
}

// acc (accumulator file) += a . b
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ bf16x8 lds_rd(const char LDS_AS* p) { return *reinterpret_cast<const bf16x8 LDS_AS*>(p); }

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N), fully expanded
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_nt(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_nt<I + 1, N>(f);
  }
}

// fragment read order of a phase: the next phase starts with block row 0 (A0 against B0..B7)
__device__ constexpr int RD_ORDER[16] = {0, 8, 9, 10, 11, 12, 13, 14, 15, 1, 2, 3, 4, 5, 6, 7};  // <8: A, else B

struct Ctx {
  // buffer DMA (variant bit 4): one descriptor per operand (this wave's first staged row), a
  // loop-invariant 32-bit lane offset per piece, the k-tile offset as soffset
  __amdgpu_buffer_rsrc_t ra, rb;
  unsigned vpa[8], vpb[8];
  unsigned lds_wave;  // LDS byte address of this wave's first staged A row in stage 0
  const char LDS_AS* smem;
  unsigned lds0;
  int rd[2];          // lane's fragment byte offset in an image row block, per k-half
  int a_wave, b_wave;  // wave's row block offset inside the A / B image
  // DMA: scalar bases of this wave's first A / B piece at k = 0, lane offsets per piece parity
  const ushort* ga;
  const ushort* gb;
  long lda, ldb;
  unsigned va[2], vb[2];
  int dma_row;  // first image row this wave stages
};

// One of the 16 DMA pieces (8 of A, 8 of B) of k-tile `kt` into stage `st`.  The piece's scalar base
// is loop-invariant (hipcc keeps the 16 of them in SGPR pairs); the k-tile offset rides in the
// lane's 32-bit offset (one v_add per operand and parity per tile instead of a 64-bit SALU add per
// piece).
// buffer form: s_add_u32 writes M0 directly (no VGPR or 64-bit address arithmetic per piece)
template <int IMM>
__device__ __forceinline__ void bdma16(unsigned lds_base, unsigned voff, __amdgpu_buffer_rsrc_t r, unsigned soff) {
  asm volatile("s_add_u32 m0, %0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds"
               :: "s"(lds_base), "i"(IMM), "v"(voff), "s"(r), "s"(soff) : "memory", "m0");
}

template <int P, int V>
__device__ __forceinline__ void dma_piece(const Ctx& c, int kt, int st) {
  if (V & 16) {
    const unsigned lb = c.lds_wave + st * STAGE;  // uniform; the piece's constant part is an immediate
    const unsigned soff = (unsigned)kt * (BK * 2);
    if (P < 8)
      bdma16<(P & 7) * 1024>(lb, c.vpa[P & 7], c.ra, soff);
    else
      bdma16<IMG + (P & 7) * 1024>(lb, c.vpb[P & 7], c.rb, soff);
    return;
  }
  const unsigned img = c.lds0 + st * STAGE + (P < 8 ? 0 : IMG) + (c.dma_row + (P & 7) * 8) * 128;
  const unsigned koff = (unsigned)kt * (BK * 2);
  if (P < 8)
    glds16<!(V & 2)>(c.ga + (long)(P & 7) * 8 * c.lda, c.va[P & 1] + koff, img);
  else
    glds16<!(V & 2)>(c.gb + (long)(P & 7) * 8 * c.ldb, c.vb[P & 1] + koff, img);
}

// One phase: acc[i][j] += B_j(.) A_i over the k-half held in (af, bf) -- 64 MFMAs in 16 groups of
// 4, i-major.  RD0 >= 0: the 16 fragment reads of the next half into (an, bn) from stage `rst` /
// k-half `rk`, spread over groups RD0 .. RD0+RDN-1 (RDN 8: two per group, 16: one).  DMA0 >= 0:
// this wave's 16 DMA pieces of k-tile `dkt` into stage `dst`, over groups DMA0 .. DMA0+DMAN-1.
template <int RD0, int RDN, int DMA0, int DMAN, int V>
__device__ __forceinline__ void phase(const Ctx& c, f32x4 (&acc)[8][8], const bf16x8 (&af)[8], const bf16x8 (&bf)[8],
                                      bf16x8 (&an)[8], bf16x8 (&bn)[8], int rst, int rk, int dkt, int dst) {
  const char LDS_AS* sa = c.smem + rst * STAGE + c.a_wave + c.rd[rk];
  const char LDS_AS* sb = c.smem + rst * STAGE + IMG + c.b_wave + c.rd[rk];
  constexpr int RPG = RDN > 0 ? 16 / RDN : 0, DPG = DMAN > 0 ? 16 / DMAN : 0;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = 4 * s + q, i = m >> 3, j = m & 7;
      mfma_acc(acc[i][j], bf[j], af[i]);
    }
    if (RD0 >= 0 && s >= RD0 && s < RD0 + RDN) {
#pragma unroll
      for (int e = 0; e < RPG; ++e) {
        const int f = RD_ORDER[RPG * (s - RD0) + e];
        if (f < 8)
          an[f] = lds_rd(sa + f * 2048);
        else
          bn[f - 8] = lds_rd(sb + (f - 8) * 2048);
      }
    }
    if (DMA0 >= 0 && s >= DMA0 && s < DMA0 + DMAN) {
#pragma unroll
      for (int e = 0; e < DPG; ++e) {
        const int u = DPG * (s - DMA0) + e;  // A0 B0 A1 B1 ... (piece u>>1 of A or B)
        switch (u) {  // constant after unrolling
          case 0: dma_piece<0, V>(c, dkt, dst); break;
          case 1: dma_piece<8, V>(c, dkt, dst); break;
          case 2: dma_piece<1, V>(c, dkt, dst); break;
          case 3: dma_piece<9, V>(c, dkt, dst); break;
          case 4: dma_piece<2, V>(c, dkt, dst); break;
          case 5: dma_piece<10, V>(c, dkt, dst); break;
          case 6: dma_piece<3, V>(c, dkt, dst); break;
          case 7: dma_piece<11, V>(c, dkt, dst); break;
          case 8: dma_piece<4, V>(c, dkt, dst); break;
          case 9: dma_piece<12, V>(c, dkt, dst); break;
          case 10: dma_piece<5, V>(c, dkt, dst); break;
          case 11: dma_piece<13, V>(c, dkt, dst); break;
          case 12: dma_piece<6, V>(c, dkt, dst); break;
          case 13: dma_piece<14, V>(c, dkt, dst); break;
          case 14: dma_piece<7, V>(c, dkt, dst); break;
          default: dma_piece<15, V>(c, dkt, dst); break;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Fine-grained form of `phase` (variant bit 3): the side work is interleaved per MFMA instead of per
// group of 4, so no burst of DMA / read issue outlasts the issue slots an MFMA leaves free (one
// wave per SIMD: an MFMA holds vector issue for 8 of its 16 cycles).  With DMA (phase B): a DMA
// piece after MFMAs 0, 4, .., 60 and a fragment read after MFMAs 2, 6, .., 62; without (phase A):
// a read after MFMAs 0, 3, .., 45.
template <bool RD, bool DMA, int V>
__device__ __forceinline__ void phase_fine(const Ctx& c, f32x4 (&acc)[8][8], const bf16x8 (&af)[8],
                                           const bf16x8 (&bf)[8], bf16x8 (&an)[8], bf16x8 (&bn)[8], int rst, int rk,
                                           int dkt, int dst) {
  const char LDS_AS* sa = c.smem + rst * STAGE + c.a_wave + c.rd[rk];
  const char LDS_AS* sb = c.smem + rst * STAGE + IMG + c.b_wave + c.rd[rk];
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    const int i = m >> 3, j = m & 7;
    mfma_acc(acc[i][j], bf[j], af[i]);
    int r = -1, d = -1;
    if (DMA) {
      if ((m & 3) == 0) d = m >> 2;
      if (RD && (m & 3) == 2) r = m >> 2;
    } else if (RD && m % 3 == 0 && m / 3 < 16) {
      r = m / 3;
    }
    if (r >= 0) {
      const int f = RD_ORDER[r];
      if (f < 8)
        an[f] = lds_rd(sa + f * 2048);
      else
        bn[f - 8] = lds_rd(sb + (f - 8) * 2048);
    }
    if (d >= 0) {
      switch (d) {  // A0 B0 A1 B1 ...; constant after unrolling
        case 0: dma_piece<0, V>(c, dkt, dst); break;
        case 1: dma_piece<8, V>(c, dkt, dst); break;
        case 2: dma_piece<1, V>(c, dkt, dst); break;
        case 3: dma_piece<9, V>(c, dkt, dst); break;
        case 4: dma_piece<2, V>(c, dkt, dst); break;
        case 5: dma_piece<10, V>(c, dkt, dst); break;
        case 6: dma_piece<3, V>(c, dkt, dst); break;
        case 7: dma_piece<11, V>(c, dkt, dst); break;
        case 8: dma_piece<4, V>(c, dkt, dst); break;
        case 9: dma_piece<12, V>(c, dkt, dst); break;
        case 10: dma_piece<5, V>(c, dkt, dst); break;
        case 11: dma_piece<13, V>(c, dkt, dst); break;
        case 12: dma_piece<6, V>(c, dkt, dst); break;
        case 13: dma_piece<14, V>(c, dkt, dst); break;
        case 14: dma_piece<7, V>(c, dkt, dst); break;
        default: dma_piece<15, V>(c, dkt, dst); break;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// this wave's 16 DMA pieces of k-tile kt into stage st, back to back (prologue)
template <int V>
__device__ __forceinline__ void dma_tile(const Ctx& c, int kt, int st) {
  dma_piece<0, V>(c, kt, st); dma_piece<1, V>(c, kt, st); dma_piece<2, V>(c, kt, st); dma_piece<3, V>(c, kt, st);
  dma_piece<4, V>(c, kt, st); dma_piece<5, V>(c, kt, st); dma_piece<6, V>(c, kt, st); dma_piece<7, V>(c, kt, st);
  dma_piece<8, V>(c, kt, st); dma_piece<9, V>(c, kt, st); dma_piece<10, V>(c, kt, st); dma_piece<11, V>(c, kt, st);
  dma_piece<12, V>(c, kt, st); dma_piece<13, V>(c, kt, st); dma_piece<14, V>(c, kt, st); dma_piece<15, V>(c, kt, st);
}

__device__ __forceinline__ void read_half(const Ctx& c, bf16x8 (&af)[8], bf16x8 (&bf)[8], int st, int k) {
  const char LDS_AS* sa = c.smem + st * STAGE + c.a_wave + c.rd[k];
  const char LDS_AS* sb = c.smem + st * STAGE + IMG + c.b_wave + c.rd[k];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int f = RD_ORDER[s];
    if (f < 8)
      af[f] = lds_rd(sa + f * 2048);
    else
      bf[f - 8] = lds_rd(sb + (f - 8) * 2048);
  }
}
}  // namespace

// V (schedule variants, A/B aids): bit0 reads and DMA one per group over all 16 groups (default:
// two per group, reads in one half of the phase, DMA in the other); bit1 no s_nop between the M0
// write and the LDS-DMA; bit2 bands of 16 tile rows instead of 8; bit3 side work interleaved per
// MFMA (phase_fine); bit4 the DMA as buffer_load ... lds with a loop-invariant lane offset per piece,
// the k offset in soffset and M0 written by one s_add (no per-piece VGPR or 64-bit address math).
// Compiled: 0, 1, 8, 16, 17, 20 (8 + 16 loses the AGPR allocation: hipcc moves the accumulators).
template <bool BETA, int V>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_kernel(const ushort* __restrict__ A, long lda,
                                                         const ushort* __restrict__ B, long ldb,
                                                         ushort* __restrict__ C, long ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[SMEM];
  const int nM = M / BM, nN = N / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = (V & 4) ? 16 : 8;  // a band of tile rows walks the tile columns together (A rows stay in L2)
  const int per_band = GM * nN;
  const int band = L / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = L % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int r16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.smem = (const char LDS_AS*)smem_raw;
  c.lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem_raw;
#pragma unroll
  for (int k = 0; k < 2; ++k) c.rd[k] = r16 * 128 + (((4 * k + g) ^ (r16 >> 1)) << 4);
  c.a_wave = wr * 128 * 128;
  c.b_wave = wc * 128 * 128;
  c.dma_row = w * 64;  // wave w stages image rows [64 w, 64 w + 64) of A and of B
  c.lda = lda;
  c.ldb = ldb;
  c.ga = A + (m0 + c.dma_row) * lda;
  c.gb = B + (n0 + c.dma_row) * ldb;
  {
    // piece p covers image rows dma_row + 8p .. +7; lane -> row (lane >> 3), slot (lane & 7), which
    // holds global chunk slot ^ ((row >> 1) & 7) = slot ^ (4 (p & 1) + (lane >> 4))
    const int rr = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int chunk = slot ^ (4 * par + (lane >> 4));
      c.va[par] = (unsigned)(2 * ((long)rr * lda + 8 * chunk));
      c.vb[par] = (unsigned)(2 * ((long)rr * ldb + 8 * chunk));
    }
    if (V & 16) {
      c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)c.ga, 0, 0x7fffffff, 0x00020000);
      c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)c.gb, 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        c.vpa[p] = c.va[p & 1] + (unsigned)(2L * 8 * p * lda);
        c.vpb[p] = c.vb[p & 1] + (unsigned)(2L * 8 * p * ldb);
      }
      c.lds_wave = c.lds0 + c.dma_row * 128;
    }
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4(0.f);
  // Materialise every zero accumulator in the AGPR file here, then pad: hipcc otherwise zeroes an
  // accumulator lazily (v_accvgpr_mov) right before the first MFMA statement that reads it, and it
  // inserts no wait states in front of an asm MFMA, so the MFMA read a stale SrcC (variant 8 returned
  // inf before this).  The empty "+a" statements pin the values; asm volatile keeps them in order.
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4" ::);

  const int nt = K / BK;
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  dma_tile<V>(c, 0, 0);
  if (nt > 1) {
    dma_tile<V>(c, 1, 1);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  read_half(c, a0, b0, 0, 0);
  // phase A(0): half 0 of tile 0, read half 1 of tile 0
  constexpr int RN = (V & 1) ? 16 : 8;
  if (V & 8)
    phase_fine<true, false, V>(c, acc, a0, b0, a1, b1, 0, 1, 0, 0);
  else
    phase<0, RN, -1, 0, V>(c, acc, a0, b0, a1, b1, 0, 1, 0, 0);
  // this wave's DMA of tile 1 retired and every wave's reads of stage 0 done: tile 1 visible, and
  // the next DMA may overwrite stage 0
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // Steady state, one loop iteration = phase B(t) + phase A(t+1) + the barrier, so the loop head sits
  // right after a barrier (hipcc waits lgkmcnt(0) there: nothing is outstanding).  The body is
  // straight-line -- a branch between MFMA statements would give the accumulators phi nodes on
  // several paths, and hipcc then copies them through VGPRs and spills -- so the second-to-last
  // B phase re-stages the last k-tile into the free stage (nobody reads it).
  //   B(t):   half 1 of tile t; DMA tile t+2 -> stage t&1 (groups 0-7, ~2 phases before it is waited
  //           for); read half 0 of tile t+1 (groups 8-15)
  //   A(t+1): half 0 of tile t+1; read half 1 of tile t+1 (groups 0-7)
  for (int t = 0; t < nt - 1; ++t) {
    const int st = t & 1;
    if (V & 8) {
      phase_fine<true, true, V>(c, acc, a1, b1, a0, b0, st ^ 1, 0, min(t + 2, nt - 1), st);
      phase_fine<true, false, V>(c, acc, a0, b0, a1, b1, st ^ 1, 1, 0, 0);
    } else {
      if (V & 1)
        phase<0, 16, 0, 16, V>(c, acc, a1, b1, a0, b0, st ^ 1, 0, min(t + 2, nt - 1), st);
      else
        phase<8, 8, 0, 8, V>(c, acc, a1, b1, a0, b0, st ^ 1, 0, min(t + 2, nt - 1), st);
      phase<0, RN, -1, 0, V>(c, acc, a0, b0, a1, b1, st ^ 1, 1, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  phase<-1, 0, -1, 0, V>(c, acc, a1, b1, a0, b0, 0, 0, 0, 0);  // B(nt-1)
  // MFMA results -> readable (XDL write -> VALU read wait states), then pin every accumulator
  // after the pad so no read of it is scheduled above
  asm volatile("s_nop 15\n\ts_nop 15" ::);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

  // epilogue: lane holds C[m = 16 i + r16][n = 16 j + 4 g .. +3] of the wave tile.  Stage the wave's
  // 128 x 128 bf16 tile in its own 32 KB of LDS (rows of 256 B, 16-B block b of row r at b ^ (r & 15):
  // conflict-free b64 writes and b128 reads), then 16-B row stores.  The last B phase reads and
  // DMAs nothing and the barrier before it drained every wave's reads and DMA: no further barrier.
  char LDS_AS* ep = (char LDS_AS*)smem_raw + w * 32768;
  const long crow0 = m0 + wr * 128, ccol0 = n0 + wc * 128;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4 v = acc[i][j];
      if (BETA) {
        const ushort4v old = *reinterpret_cast<const ushort4v*>(C + (crow0 + 16 * i + r16) * ldc + ccol0 + 16 * j + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bf2f(old[e]);
      }
      ushort4v o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      const int row = 16 * i + r16;
      const int blk = (2 * j + (g >> 1)) ^ r16;
      *reinterpret_cast<ushort4v LDS_AS*>(ep + row * 256 + blk * 16 + (g & 1) * 8) = o;
    }
  }
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int row = 4 * q + g;
    const ushort8 v = *reinterpret_cast<const ushort8 LDS_AS*>(ep + row * 256 + ((r16 ^ (row & 15)) << 4));
    *reinterpret_cast<ushort8*>(C + (crow0 + row) * ldc + ccol0 + 8 * r16) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Schedule "hb" (launch flags bit 5): the same machine (256 x 256 x 64, 4 waves of 128 x 128,
// 16x16x32, 256 AGPR accumulators, 2-stage 128 KB ring) with ONE k-tile per loop iteration and the
// synchronisation split per operand, so the DMA of a tile never has to be waited for with vmcnt(0):
//   MFMA   0- 63  k-step 0 of tile t (fragments X, read at the end of the previous iteration)
//           1- 15  read A's k-step-1 fragments of tile t (Y.a)       | 20: lgkmcnt(0) + barrier: every
//          22- 36  DMA A of tile t+2 into tile t's stage               |     wave is done with A of tile t
//          25- 39  read B's k-step-1 fragments (Y.b)                   | 48: lgkmcnt(0) + barrier
//          50- 66  DMA B pieces 0-4 of tile t+2 (13 pieces issued)
//   MFMA  64-127  k-step 1 of tile t (Y)
//          80      vmcnt(13): the previous iteration's 16 pieces (tile t+1) landed; barrier
//          84-116  DMA B pieces 5-7; 94-124 read tile t+1's k-step-0 fragments (X) from the other stage
// Each DMA has about one iteration of lead time and is waited for by count; the barriers release
// each operand region as soon as its last reader is past it.  DMA pieces are buffer_load ... lds
// with the k-tile in the descriptor base and a loop-invariant soffset per piece (two instructions
// per piece).  SV bit0: reads of X spread one per 3 MFMAs from 82 (with bit1: the tile-(t+1) wait at
// 72 and the reads one per 2 MFMAs from 74);
// SV bit1: B's reads at 17-31, its barrier at 38 and ALL its DMA pieces at 40-68, so the tile-(t+1)
// wait at 88 is vmcnt(16) (every piece has > 1 iteration of lead time).
template <int SV>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_hb_kernel(const ushort* __restrict__ A, long lda,
                                                            const ushort* __restrict__ B, long ldb,
                                                            ushort* __restrict__ C, long ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[SMEM];
  const int nM = M / BM, nN = N / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int per_band = GM * nN;
  const int band = L / per_band;
  const int first_m = band * GM;
  const int gm = min(GM, nM - first_m);
  const int in_band = L % per_band;
  const int tm = first_m + in_band % gm;
  const int tn = in_band / gm;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int r16 = lane & 15, g = lane >> 4;
  const char LDS_AS* smem = (const char LDS_AS*)smem_raw;
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem_raw;
  int rd[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) rd[k] = r16 * 128 + (((4 * k + g) ^ (r16 >> 1)) << 4);
  const int a_wave = wr * 128 * 128, b_wave = wc * 128 * 128;
  const int dma_row = w * 64;  // wave w stages image rows [64 w, 64 w + 64) of A and of B
  const ushort* ga = A + (m0 + dma_row) * lda;
  const ushort* gb = B + (n0 + dma_row) * ldb;
  // lane -> row (lane >> 3) of a piece, slot (lane & 7) holding global chunk slot ^ (4 (p & 1) + (lane >> 4))
  unsigned va[2], vb[2];
  {
    const int rr = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int chunk = slot ^ (4 * par + (lane >> 4));
      va[par] = (unsigned)(2 * ((long)rr * lda + 8 * chunk));
      vb[par] = (unsigned)(2 * ((long)rr * ldb + 8 * chunk));
    }
  }
  const unsigned lds_wave = lds0 + dma_row * 128;
  const unsigned sa_step = (unsigned)(2L * 8 * lda), sb_step = (unsigned)(2L * 8 * ldb);  // bytes per piece (8 rows)
  // piece p of operand X (0 = A, 1 = B) of k-tile kt into stage st
  auto piece = [&](int op, int p, int kt, int st) {
    const ushort* base = (op == 0 ? ga : gb) + (long)kt * BK;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    const unsigned soff = (unsigned)p * (op == 0 ? sa_step : sb_step);
    const unsigned voff = op == 0 ? va[p & 1] : vb[p & 1];
    const unsigned lb = __builtin_amdgcn_readfirstlane(lds_wave + st * STAGE + op * IMG + p * 1024);
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

  const int nt = K / BK;
  bf16x8 xa[8], xb[8], ya[8], yb[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(0, p, 0, 0);
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(1, p, 0, 0);
  const int kt1 = min(1, nt - 1);
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(0, p, kt1, 1);
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(1, p, kt1, 1);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  {
    const char LDS_AS* sa = smem + a_wave + rd[0];
    const char LDS_AS* sb = smem + IMG + b_wave + rd[0];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      xa[f] = lds_rd(sa + f * 2048);
      xb[f] = lds_rd(sb + f * 2048);
    }
  }
  for (int t = 0; t < nt; ++t) {
    const int st = t & 1;
    const int kt2 = min(t + 2, nt - 1);  // past the end: re-stage the last tile (nobody reads it)
    const char LDS_AS* sa1 = smem + st * STAGE + a_wave + rd[1];
    const char LDS_AS* sb1 = smem + st * STAGE + IMG + b_wave + rd[1];
    const char LDS_AS* sa0 = smem + (st ^ 1) * STAGE + a_wave + rd[0];
    const char LDS_AS* sb0 = smem + (st ^ 1) * STAGE + IMG + b_wave + rd[0];
    static_for_nt<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      constexpr int mm = m & 63, i = mm >> 3, j = mm & 7;
      if constexpr (m < 64)
        mfma_acc(acc[i][j], xb[j], xa[i]);
      else
        mfma_acc(acc[i][j], yb[j], ya[i]);
      if constexpr (m >= 1 && m <= 15 && (m & 1)) ya[(m - 1) / 2] = lds_rd(sa1 + ((m - 1) / 2) * 2048);
      if constexpr (m == 20) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (m >= 22 && m <= 36 && !(m & 1)) piece(0, (m - 22) / 2, kt2, st);
      if constexpr (SV & 2) {
        // every B piece before the tile-(t+1) wait, which then lets all 16 of this tile fly (vmcnt(16))
        if constexpr (m >= 17 && m <= 31 && (m & 1)) yb[(m - 17) / 2] = lds_rd(sb1 + ((m - 17) / 2) * 2048);
        if constexpr (m == 38) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if constexpr (m >= 40 && m <= 68 && ((m - 40) % 4 == 0)) piece(1, (m - 40) / 4, kt2, st);
        if constexpr (m == ((SV & 1) ? 72 : 88)) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
      } else {
        if constexpr (m >= 25 && m <= 39 && (m & 1)) yb[(m - 25) / 2] = lds_rd(sb1 + ((m - 25) / 2) * 2048);
        if constexpr (m == 48) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if constexpr (m >= 50 && m <= 66 && ((m - 50) % 4 == 0)) piece(1, (m - 50) / 4, kt2, st);
        if constexpr (m == 80) asm volatile("s_waitcnt vmcnt(13)\n\ts_barrier" ::: "memory");
        if constexpr (m == 84 || m == 100 || m == 116) piece(1, 5 + (m - 84) / 16, kt2, st);
      }
      if constexpr (SV & 1) {
        constexpr int X1 = (SV & 2) ? 74 : 82;
        if constexpr (m >= X1 && m <= 127 && ((m - X1) % 2 == 0) && (m - X1) / 2 < 16 && (SV & 2)) {
          constexpr int f = (m - X1) / 2;
          if constexpr (f < 8) xa[f] = lds_rd(sa0 + f * 2048);
          else xb[f - 8] = lds_rd(sb0 + (f - 8) * 2048);
        }
        if constexpr (m >= 82 && m <= 127 && ((m - 82) % 3 == 0) && (m - 82) / 3 < 16 && !(SV & 2)) {
          constexpr int f = (m - 82) / 3;
          if constexpr (f < 8) xa[f] = lds_rd(sa0 + f * 2048);
          else xb[f - 8] = lds_rd(sb0 + (f - 8) * 2048);
        }
      } else {
        constexpr int X0 = (SV & 2) ? 90 : 94;
        if constexpr (m >= X0 && m <= X0 + 30 && !(m & 1)) {
          constexpr int f = (m - X0) / 2;  // A0 B0..B7 first: the next iteration starts with row 0
          constexpr int ord[16] = {0, 8, 9, 10, 11, 12, 13, 14, 15, 1, 2, 3, 4, 5, 6, 7};
          constexpr int q = ord[f];
          if constexpr (q < 8) xa[q] = lds_rd(sa0 + q * 2048);
          else xb[q - 8] = lds_rd(sb0 + (q - 8) * 2048);
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
  // epilogue (as gemm_nt_kernel): stage the wave's 128 x 128 bf16 tile in LDS, then 16-B row stores
  char LDS_AS* ep = (char LDS_AS*)smem_raw + w * 32768;
  const long crow0 = m0 + wr * 128, ccol0 = n0 + wc * 128;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = acc[i][j];
      ushort4v o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
      const int row = 16 * i + r16;
      const int blk = (2 * j + (g >> 1)) ^ r16;
      *reinterpret_cast<ushort4v LDS_AS*>(ep + row * 256 + blk * 16 + (g & 1) * 8) = o;
    }
  }
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int row = 4 * q + g;
    const ushort8 v = *reinterpret_cast<const ushort8 LDS_AS*>(ep + row * 256 + ((r16 ^ (row & 15)) << 4));
    *reinterpret_cast<ushort8*>(C + (crow0 + row) * ldc + ccol0 + 8 * r16) = v;
  }
}

extern "C" int th_gemm_nt(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                          int beta, int flags, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return -1;
  // per-lane DMA offsets are 32-bit: 8 rows of one piece from the piece's scalar base
  if ((long)8 * lda * 2 >= (1L << 31) || (long)8 * ldb * 2 >= (1L << 31)) return -1;
  const long grid = (long)(M / BM) * (N / BN);
  if (grid > 0x7fffffffL) return -2;
#define TH_NT_LAUNCH(BT, V)                                                                                 \
  gemm_nt_kernel<BT, V><<<(unsigned)grid, NTHR, 0, s>>>((const ushort*)A, lda, (const ushort*)B, ldb, (ushort*)C, ldc, \
                                                       M, N, K)
  if (!beta && (flags & 32)) {  // schedule "hb" (gemm_nt_hb_kernel), sub-variant SV in bits 6-7
    // buffer descriptors address the operands from this workgroup's first staged row: 32-bit offsets
    if ((long)K * 2 + 256L * 2 * max(lda, ldb) >= (1L << 31)) return -1;
#define TH_NT_HB(SV_) \
  gemm_nt_hb_kernel<SV_><<<(unsigned)grid, NTHR, 0, s>>>((const ushort*)A, lda, (const ushort*)B, ldb, (ushort*)C, ldc, M, N, K)
    switch ((flags >> 6) & 3) {
      case 1: TH_NT_HB(1); break;
      case 2: TH_NT_HB(2); break;
      case 3: TH_NT_HB(3); break;
      default: TH_NT_HB(0); break;
    }
#undef TH_NT_HB
    TH_CHECK_LAUNCH();
  }
  // flags bits 0-4: schedule variant (see gemm_nt_kernel); beta = 1 runs the default schedule
  switch (beta ? 64 : (flags & 31)) {
    case 1: TH_NT_LAUNCH(false, 1); break;
    case 8: TH_NT_LAUNCH(false, 8); break;
    case 16: TH_NT_LAUNCH(false, 16); break;
    case 17: TH_NT_LAUNCH(false, 17); break;
    case 20: TH_NT_LAUNCH(false, 20); break;
    case 64: TH_NT_LAUNCH(true, 0); break;
    default: TH_NT_LAUNCH(false, 0); break;
  }
#undef TH_NT_LAUNCH
  TH_CHECK_LAUNCH();
}
