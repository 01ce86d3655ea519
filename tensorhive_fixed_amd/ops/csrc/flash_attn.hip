// Causal GQA flash attention, head_dim 128, bf16 in / f32 accumulate, for gfx950 (MI355X).
//
// All three kernels read q/k/v straight out of the packed QKV projection output
// ([tokens, (Hq + 2*Hkv) * 128], row stride `ld`), so the model never transposes or copies.
// Matrix work is v_mfma_f32_32x32x16_bf16 throughout; the operand orientation is chosen so the
// softmax statistics are lane-local:
//
//   forward  (query-centric, 4 waves x 32 queries per workgroup, 64-key tiles):
//     S^T = K Q^T        A = K rows (LDS, ds_read_b128)    B = Q rows (registers)
//     O^T += V^T P^T     A = V^T    (LDS, ds_read_b64_tr_b16)  B = P^T straight from the S^T
//                        accumulator (query on the lane -> running max / sum need no shuffles
//                        except one lane^32 exchange, and the O^T rescale is per-lane).
//   dQ       (query-centric, same skeleton):  S^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//            dQ^T += K^T dS^T  (K^T via transposed LDS reads).  No atomics: deterministic.
//   dK/dV    (key-centric, loops over the GQA group's query heads):
//            S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS.
//            Default: the paired kernel (dK waves and dV waves of 128 keys share the Q/dO tile,
//            K/V in registers); flags bit3: the fused kernel (8 waves x 32 keys, K/V in LDS).
//
// Every LDS tile uses ONE image that serves both 16-byte row reads and transposed reads
// conflict-free (8-row x 32-column subtiles, see img_off).
// Workgroup ids are remapped so each XCD (own L2) gets a contiguous range of the logical order
// (the GQA query heads that share a K/V head land on one XCD); causal blocks go heaviest first.
// th-build-flags: -fno-slp-vectorize
//   (the SLP vectorizer packs the per-score f32 math into v_pk_mul/add_f32, which cost more issue
//   cycles than two scalar ops beside MFMAs: MI355X_MICROARCH 'price of one filler beside MFMAs')
#include "th_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

namespace {
constexpr int HD = 128;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// 8-row x 32-column subtiles of 512 B.  The 16-byte slot of (row, chunk) inside its 256-B bank
// row is 4*(row&3) + ((ch&3) ^ ((row>>2)&3)): conflict-free for the ds_read_b128 row operands of
// 32x32x16 MFMAs and for ds_read_b64_tr_b16 transposed operands, and the loop-varying parts
// (ch>>2 and row>>3) are pure immediates, so each wave needs only 2 address bases per image.
__device__ __forceinline__ int img_off(int row, int ch) {
  return ((row >> 3) << 11) + ((ch >> 2) << 9) + ((row & 7) << 6) + (((ch & 3) ^ ((row >> 2) & 3)) << 4);
}

__device__ __forceinline__ bf16x8 as_bf(ushort8 u) { return __builtin_bit_cast(bf16x8, u); }

__device__ __forceinline__ bf16x8 lds_row(const char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(img + img_off(row, ch));
}

// Transposed operand (A = X^T with X[row][col] in the image): lane (c = lane&31, h = lane>>5)
// gets X[rbase + 8*(j>>2) + 4h + (j&3)][cbase + c] in element j (the k order the accumulator
// -> operand reuse expects).
__device__ __forceinline__ bf16x8 lds_tr(const char* img, int rbase, int cbase, int lane) {
  const int h = lane >> 5, grp = (lane >> 4) & 1, i = lane & 15;
  const int row = rbase + 4 * h + (i >> 2);
  const int col = cbase + 16 * grp + 4 * (i & 3);
  const char* p0 = img + img_off(row, col >> 3) + ((col & 7) << 1);
  const char* p1 = img + img_off(row + 8, col >> 3) + ((col & 7) << 1);
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(p0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(p1));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Forward: wave priority around the MFMA clusters -- a wave issuing its S or PV block outranks
// its SIMD partner in softmax VALU work, so the matrix pipe is refilled first (fwd 745 -> 684 us
// at B4 S4096; the same hint measured neutral in dQ and +1.7 % in the paired dK|dV kernel).
#ifndef TH_FA_PRIO
#define TH_FA_PRIO 1
#endif
#define FA_PRIO(p)                                  \
  do {                                              \
    if (TH_FA_PRIO) __builtin_amdgcn_s_setprio(p); \
  } while (0)

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[base + j];
  return r;
}

// Epilogue of a transposed 32x32 accumulator set (4 tiles = 128 head dims on the accumulator rows,
// one token per lane column): lane l holds dims 32d + 8g + 0..3 and lane l+32 dims 32d + 8g + 4..7
// of the same token row, so the plain store is 16 dwordx2 per lane.  One v_permlane32_swap per
// dword and group pair (g, g+1) gives lanes 0-31 the 16 contiguous bytes of group g and lanes 32-63
// those of group g+1: 8 dwordx4 stores per lane, same bytes (cdna_hip_programming.md T21: the tail
// is store-issue-bound).  Both lanes of a pair hold the same token, so a token-validity branch
// around the call never splits a pair.
__device__ __forceinline__ void store_row_t21(ushort* row, const f32x16 (&acc)[4], float f, int h) {
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      unsigned a[2], c[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        a[k] = (unsigned)f2bf(acc[d][8 * p + 2 * k] * f) | ((unsigned)f2bf(acc[d][8 * p + 2 * k + 1] * f) << 16);
        c[k] = (unsigned)f2bf(acc[d][8 * p + 4 + 2 * k] * f) | ((unsigned)f2bf(acc[d][8 * p + 5 + 2 * k] * f) << 16);
        const auto r = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
        a[k] = r[0];
        c[k] = r[1];
      }
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = {a[0], a[1], c[0], c[1]};
      *reinterpret_cast<u32x4*>(row + 32 * d + 16 * p + 8 * h) = v;
    }
}

// Rotary-embedding backward folded into a q / k gradient's epilogue (Llama rotate-half pairs (i, i + 64),
// the inverse rotation; tables [S][64] f32 as ops/rope.py builds them): lane (c32, h) holds dims
// 32d + 8g + 4h + e of its row in acc[d][4g + e], so the partner of a dim in blocks 0-1 sits in blocks
// 2-3 of the same lane and the rotation needs no data exchange.  Replaces the separate in-place
// rope pass over dQ and dK after the backward.
__device__ __forceinline__ void rope_bwd_rows(f32x16 (&a)[4], const float* __restrict__ rcos,
                                              const float* __restrict__ rsin, int pos, int h) {
  const float* cr = rcos + (long)pos * 64;
  const float* sr = rsin + (long)pos * 64;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4v c4 = *reinterpret_cast<const float4v*>(cr + 32 * d + 8 * g + 4 * h);
      const float4v s4 = *reinterpret_cast<const float4v*>(sr + 32 * d + 8 * g + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = a[d][4 * g + e], y = a[d + 2][4 * g + e];
        a[d][4 * g + e] = x * c4[e] + y * s4[e];
        a[d + 2][4 * g + e] = y * c4[e] - x * s4[e];
      }
    }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// accumulator row (register r of lane half h) of a 32x32 MFMA tile
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Stage `16*NP` x 128 bf16 rows (global, row stride ld) into registers with 256 threads.
// Thread t covers row 16*i + 2*((t>>3)&7) + ((t>>2)&1), 16-byte chunk 4*(t>>6) + (t&3).  A
// ds_write_b128 is serviced in groups of 8 contiguous lanes with banks (a/4) mod 32, i.e. 128 B:
// each such group writes 2 adjacent rows x 4 chunks = 128 contiguous bytes of the image (the XOR
// only permutes slots inside a row's 64 B) -> conflict-free.  (A 4-rows x 2-chunks group put rows
// r and r+2 on the same banks: 2-way, 20-25 % of the kernels' LDS cycles in SQ_LDS_BANK_CONFLICT.)
// Rows >= limit are clamped to limit-1 (finite data; the consumers mask those keys), so the loads
// are unconditional -- no divergent branch per load.
__device__ __forceinline__ int stage_row(int tid) { return 2 * ((tid >> 3) & 7) + ((tid >> 2) & 1); }
__device__ __forceinline__ int stage_ch(int tid) { return 4 * ((tid >> 6) & 3) + (tid & 3); }
template <int NP>
__device__ __forceinline__ void stage_load(ushort8 (&r)[NP], const ushort* base, long ld, int row0,
                                           int limit, int tid) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int row = min(row0 + 16 * i + stage_row(tid), limit - 1);
    r[i] = *reinterpret_cast<const ushort8*>(base + (long)row * ld + (stage_ch(tid) << 3));
  }
}
template <int NP>
__device__ __forceinline__ void stage_store(char* img, const ushort8 (&r)[NP], int tid) {
#pragma unroll
  for (int i = 0; i < NP; ++i)
    *reinterpret_cast<ushort8*>(img + img_off(16 * i + stage_row(tid), stage_ch(tid))) = r[i];
}

// Logical block -> (batch, q head, q block).  QMAJOR: q blocks heaviest-first across all heads
// (blocks running together on an XCD touch ~16 different K/V heads: 32 MB, far beyond the XCD's
// 4 MB L2).  KVMAJOR: all q blocks x GQA heads of ONE (batch, kv head) are contiguous, so the
// ~64 workgroups resident on an XCD share one 2 MB K/V pair out of its L2.
template <bool KVMAJOR>
__device__ __forceinline__ void q_block_map(int L, int nqb, int B, int Hq, int Hkv, int& b, int& hq, int& qb) {
  if (KVMAJOR) {
    const int G = Hq / Hkv, per = nqb * G;
    const int grp = L / per, r = L % per;
    b = grp / Hkv;
    hq = (grp % Hkv) * G + r % G;
    qb = nqb - 1 - r / G;
  } else {
    const int per = Hq * B;
    qb = nqb - 1 - L / per;
    const int rem = L % per;
    b = rem / Hq;
    hq = rem % Hq;
  }
}

// ------------------------------------------------------------------ LDS-DMA tile staging
// global_load_lds_dwordx4 (inline asm with a scalar base: the builtin makes the compiler drain
// vmcnt before every later ds_read) writes 16 B per lane lane-linearly at M0.  For a 64-row x
// 128-col bf16 tile in the img_off image (16 KB), wave w issues 4 x 1 KB: lane l of instruction u
// fills image byte o = 4096w + 1024u + 16l, so it loads the (row, chunk) that img_off maps to o.
// No staging VGPRs, no ds_write, one barrier per tile (double-buffered images).
__device__ __forceinline__ void glds16(const void* sbase, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
}
// 4 B per lane (a 64-float row: lse / delta of a 64-query tile)
__device__ __forceinline__ void glds4(const void* sbase, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2"
               :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
}
// (row | chunk << 8) of image byte o (inverse of img_off)
__device__ __forceinline__ unsigned img_rc(unsigned o) {
  const unsigned row = ((o >> 11) << 3) | ((o >> 6) & 7);
  const unsigned ch = (((o >> 9) & 3) << 2) | (((o >> 4) & 3) ^ ((row >> 2) & 3));
  return row | (ch << 8);
}
__device__ __forceinline__ void wait_dma_barrier() { asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); }
// K and V rows 64jt .. +63 (clamped to S-1) into image pair jt & 1 at lds0 (pairs of 2 x 16 KB);
// rc[u] = img_rc(4096w + 1024u + 16 lane), wu = wave index (scalar)
__device__ __forceinline__ void dma_kv_tile(const ushort* Kb, const ushort* Vb, long ld, int S, int jt, unsigned lds0,
                                            int wu, const unsigned (&rc)[4]) {
  const unsigned img = lds0 + (jt & 1) * (2 * 64 * 256) + wu * 4096;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = min(jt * 64 + (int)(rc[u] & 255), S - 1);
    const unsigned voff = (unsigned)(row * ld + (rc[u] >> 8) * 8) * 2u;
    glds16(Kb, voff, img + u * 1024);
    glds16(Vb, voff, img + 64 * 256 + u * 1024);
  }
}

// piece p (0-7) of dma_kv_tile: p >> 1 = the 1 KB slice u, p & 1 = K / V
__device__ __forceinline__ void dma_kv_piece(const ushort* Kb, const ushort* Vb, long ld, int S, int jt,
                                             unsigned lds0, int wu, const unsigned (&rc)[4], int p) {
  const unsigned img = lds0 + (jt & 1) * (2 * 64 * 256) + wu * 4096;
  const int u = p >> 1;
  const int row = min(jt * 64 + (int)(rc[u] & 255), S - 1);
  const unsigned voff = (unsigned)(row * ld + (rc[u] >> 8) * 8) * 2u;
  if (p & 1)
    glds16(Vb, voff, img + 64 * 256 + u * 1024);
  else
    glds16(Kb, voff, img + u * 1024);
}

// --------------------------------------------------------------------------------- forward
#ifndef TH_FA_FWD_SPREAD
#define TH_FA_FWD_SPREAD 0
#endif
#ifndef TH_FA_FWD_DEFAULT
#define TH_FA_FWD_DEFAULT 15  // PRESCALE + DEFER + DMA-staged DBUF + KVMAJOR: 937 vs 829 TFLOP/s for 11 (B4 S4096, profiles/r01_flash_v3)
#endif
#ifndef TH_FA_FWD_RDORDER
#define TH_FA_FWD_RDORDER 1
#endif
#ifndef TH_FA_FWD_AHEAD
// K-row operand look-ahead of the forward S chain in k-steps (1 or 2).  2: fwd 1.047 / 1.055 vs 1.057 / 1.066 ms
// (B 8 S 4096, alternating processes, profiles/r06_flash/ahead/), 200 instead of 220 VGPRs
#define TH_FA_FWD_AHEAD 2
#endif
constexpr int F_BM = 128, F_BN = 64;
constexpr float F_DEFER_THR = 8.f;  // log2 units: P may reach 2^8 before O/l are rescaled

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// lane <-> lane^32 combine with v_permlane32_swap (VALU; __shfl_xor(.,32) lowers to ds_bpermute,
// an LDS round trip on the softmax critical path)
__device__ __forceinline__ float half_swap_max(float x) {
  const int xi = __builtin_bit_cast(int, x);
  const auto r = __builtin_amdgcn_permlane32_swap(xi, xi, false, false);
  return fmaxf(__builtin_bit_cast(float, (int)r[0]), __builtin_bit_cast(float, (int)r[1]));
}
__device__ __forceinline__ float half_swap_sum(float x) {
  const int xi = __builtin_bit_cast(int, x);
  const auto r = __builtin_amdgcn_permlane32_swap(xi, xi, false, false);
  return __builtin_bit_cast(float, (int)r[0]) + __builtin_bit_cast(float, (int)r[1]);
}

// Variant knobs (flags of th_flash_attn_fwd):
//   PRESCALE  fold softmax_scale*log2(e) into Q once (no per-score multiply)
//   DEFER     skip the O/l rescale while the running max grows by <= F_DEFER_THR (wave-uniform)
//   DBUF      LDS-DMA staging into double-buffered K/V images: no staging VGPRs / ds_writes, ONE
//             barrier per key tile instead of two
//   SPREAD    (with DBUF) tile j+1's 8 LDS-DMA pieces issued one per MFMA pair of the S chain instead
//             of 8 in a row after the barrier (profiles/r04_flash/)
template <bool PRESCALE, bool DEFER, bool DBUF, bool KVMAJOR, bool SPREAD = false>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    ushort* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale_log2, int causal) {
  constexpr int NBUF = DBUF ? 2 : 1;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * F_BN * 256];
  const int nqb = (S + F_BM - 1) / F_BM;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b, hq, qb;
  q_block_map<KVMAJOR>(L, nqb, B, Hq, Hkv, b, hq, qb);
  const int hk = hq / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
  const int q0 = qb * F_BM + w * 32;
  const int q = q0 + c32;
  const ushort* Qb = Q + b * bs + (long)hq * HD;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;

  bf16x8 qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    ushort8 u = q < S ? *reinterpret_cast<const ushort8*>(Qb + (long)q * ld + 16 * s + 8 * h) : ushort8(0);
    if (PRESCALE) {
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = f2bf(bf2f(u[e]) * scale_log2);
    }
    qf[s] = as_bf(u);
  }
  const float sc = PRESCALE ? 1.f : scale_log2;

  const int kv_end = causal ? min(S, qb * F_BM + F_BM) : S;
  const int ntiles = (kv_end + F_BN - 1) / F_BN;
  ushort8 kr[4], vr[4];
  unsigned rc[4];
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  if (DBUF) {  // LDS-DMA staging (see dma_kv_tile); Q loads retired by a wait the compiler sees
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int u = 0; u < 4; ++u) rc[u] = img_rc(w * 4096 + u * 1024 + lane * 16);
    dma_kv_tile(Kb, Vb, ld, S, 0, lds0, wu, rc);
  } else {
    stage_load<4>(kr, Kb, ld, 0, S, tid);
    stage_load<4>(vr, Vb, ld, 0, S, tid);
  }

  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x16(0.f);
  float m_i = -INFINITY, l_i = 0.f;
  // DEFER + PRESCALE: the S chain starts from -m_base (the max the exponentials are taken against,
  // 0 before the first tile), so a tile that keeps the deferred max needs p = exp2(acc) only --
  // no subtraction per score; a rescale (rare) shifts the tile's scores once and moves m_base.
  constexpr bool SHIFT = DEFER && PRESCALE;
  float m_base = 0.f;
  f32x16 s_init = f32x16(0.f);

  for (int j = 0; j < ntiles; ++j) {
    char* ks = smem + (DBUF ? (j & 1) : 0) * (2 * F_BN * 256);
    char* vs = ks + F_BN * 256;
    if (DBUF) {
      wait_dma_barrier();  // tile j landed (every wave's DMA); everyone is past tile j-1
      if (!SPREAD && j + 1 < ntiles) dma_kv_tile(Kb, Vb, ld, S, j + 1, lds0, wu, rc);
    } else {
      __syncthreads();
      stage_store<4>(ks, kr, tid);
      stage_store<4>(vs, vr, tid);
      __syncthreads();
      if (j + 1 < ntiles) {
        stage_load<4>(kr, Kb, ld, (j + 1) * F_BN, S, tid);
        stage_load<4>(vr, Vb, ld, (j + 1) * F_BN, S, tid);
      }
    }
    const int kbase = j * F_BN;
    // SPREAD: the last tile re-loads itself into the free image pair (no branch around the pieces)
    const int jd = min(j + 1, ntiles - 1);
    if (SPREAD && causal && kbase > q0 + 31) dma_kv_tile(Kb, Vb, ld, S, jd, lds0, wu, rc);  // skipped: still DMA
    if (!(causal && kbase > q0 + 31)) {  // wave-uniform: tile entirely above the diagonal is skipped
      f32x16 sacc[2] = {s_init, s_init};
#if TH_FA_FWD_AHEAD == 2
      {  // K-row operands read two k-steps ahead of the MFMAs that use them (ring of 3)
        FA_PRIO(1);
        bf16x8 ka[3][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          ka[t][0] = lds_row(ks, c32, 2 * t + h);
          ka[t][1] = lds_row(ks, 32 + c32, 2 * t + h);
          if (TH_FA_FWD_RDORDER) __builtin_amdgcn_sched_barrier(0);  // issue order = use order: the first
                                                                     // MFMA waits for its own operand only
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          if (s + 2 < 8) {
            ka[(s + 2) % 3][0] = lds_row(ks, c32, 2 * s + 4 + h);
            ka[(s + 2) % 3][1] = lds_row(ks, 32 + c32, 2 * s + 4 + h);
          }
          __builtin_amdgcn_sched_barrier(0);
          sacc[0] = mfma(ka[s % 3][0], qf[s], sacc[0]);
          if (SPREAD) dma_kv_piece(Kb, Vb, ld, S, jd, lds0, wu, rc, s);
          sacc[1] = mfma(ka[s % 3][1], qf[s], sacc[1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        FA_PRIO(0);
      }
#else
      {  // K-row operands are read one k-step ahead of the MFMAs that use them
        FA_PRIO(1);
        bf16x8 a0 = lds_row(ks, c32, h), a1 = lds_row(ks, 32 + c32, h);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          bf16x8 n0 = a0, n1 = a1;
          if (s < 7) {
            n0 = lds_row(ks, c32, 2 * s + 2 + h);
            n1 = lds_row(ks, 32 + c32, 2 * s + 2 + h);
          }
          __builtin_amdgcn_sched_barrier(0);  // keep the next step's reads ahead of these MFMAs
          sacc[0] = mfma(a0, qf[s], sacc[0]);
          if (SPREAD) dma_kv_piece(Kb, Vb, ld, S, jd, lds0, wu, rc, s);
          sacc[1] = mfma(a1, qf[s], sacc[1]);
          __builtin_amdgcn_sched_barrier(0);
          a0 = n0;
          a1 = n1;
        }
        FA_PRIO(0);
      }
#endif
      const bool need_mask = (causal && kbase + F_BN - 1 > q0) || (kbase + F_BN > S);  // wave-uniform
      if (!PRESCALE) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sacc[kb] *= sc;
      }
      if (need_mask) {
        const int kmax = (causal ? min(q, S - 1) : S - 1) - kbase - 4 * h;  // last visible key, tile-relative
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sacc[kb][r] = (32 * kb + (r & 3) + 8 * (r >> 2) <= kmax) ? sacc[kb][r] : -INFINITY;
      }
      float mt = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mt = fmaxf(mt, sacc[kb][r]);
      mt = half_swap_max(mt);
      float m_use;
      if (SHIFT) {
        // scores are relative to m_base here: mt + m_base is the tile's true max
        if (!__all(mt + m_base - m_i <= F_DEFER_THR)) {
          const float m_new = fmaxf(m_i, mt + m_base);
          const float mu = m_new == -INFINITY ? 0.f : m_new;
          const float alpha = fast_exp2(m_i - mu);
          l_i *= alpha;
#pragma unroll
          for (int d = 0; d < 4; ++d) o[d] *= alpha;
          m_i = m_new;
          const float shift = mu - m_base;  // rebase this tile's scores and the next tiles' chains
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) sacc[kb] -= shift;
          m_base = mu;
          s_init = f32x16(-mu);
        }
        m_use = 0.f;  // sacc already holds s - m_base
      } else if (DEFER) {
        if (!__all(mt - m_i <= F_DEFER_THR)) {  // some query's max moved too far: rescale now
          const float m_new = fmaxf(m_i, mt);
          const float mu = m_new == -INFINITY ? 0.f : m_new;
          const float alpha = fast_exp2(m_i - mu);
          l_i *= alpha;
#pragma unroll
          for (int d = 0; d < 4; ++d) o[d] *= alpha;
          m_i = m_new;
        }
        m_use = m_i == -INFINITY ? 0.f : m_i;
      } else {
        const float m_new = fmaxf(m_i, mt);
        m_use = m_new == -INFINITY ? 0.f : m_new;
        const float alpha = fast_exp2(m_i - m_use);
        l_i *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] *= alpha;
        m_i = m_new;
      }
      float rs4[4] = {0.f, 0.f, 0.f, 0.f};  // 4 partial row sums: no 32-deep dependent add chain
      auto p_of = [&](int kb, int r) {
        const float p = fast_exp2(SHIFT ? sacc[kb][r] : sacc[kb][r] - m_use);
        sacc[kb][r] = p;
        rs4[r & 3] += p;
      };
      // keys 0-31 first: their P feeds the first two PV k-steps, and the exponentials of keys 32-63
      // run two per MFMA gap of those steps instead of ahead of the whole PV chain
#pragma unroll
      for (int r = 0; r < 16; ++r) p_of(0, r);
      bf16x8 pf[4];
      pf[0] = pack8(sacc[0], 0);
      pf[1] = pack8(sacc[0], 8);
      {  // V^T operands read one k-step ahead
        FA_PRIO(1);
        bf16x8 vt[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) vt[d] = lds_tr(vs, 0, 32 * d, lane);
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          if (ks4 == 2) {
            pf[2] = pack8(sacc[1], 0);
            pf[3] = pack8(sacc[1], 8);
          }
          bf16x8 nx[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) nx[d] = ks4 < 3 ? lds_tr(vs, 16 * ks4 + 16, 32 * d, lane) : vt[d];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            o[d] = mfma(vt[d], pf[ks4], o[d]);
            if (ks4 < 2) {
              p_of(1, 8 * ks4 + 2 * d);
              p_of(1, 8 * ks4 + 2 * d + 1);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int d = 0; d < 4; ++d) vt[d] = nx[d];
        }
        FA_PRIO(0);
      }
      const float rs = (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);
      l_i += half_swap_sum(rs);
    }
  }

  if (q < S) {
    const float inv_l = l_i > 0.f ? 1.f / l_i : 0.f;
    store_row_t21(O + b * bso + (long)q * ldo + (long)hq * HD, o, inv_l, h);
    if (h == 0) LSE[((long)b * Hq + hq) * S + q] = (m_i + log2f(l_i)) * LN2;
  }
}

// ------------------------------------------------------------------ ping-pong forward (flags bit 6)
// Diagnostic build only (-DTH_FA_DIAG): measured 9-16 % slower than fa_fwd_kernel at the training shape in
// every configuration tried (profiles/r06_flash/README.md).
#ifdef TH_FA_DIAG
// One workgroup = 8 waves = the same 128 queries of TWO query heads of one GQA group: waves 0-3 head 2p,
// waves 4-7 head 2p + 1 of kv head hk.  Waves w and w + 4 share a SIMD and cover the same 32 query rows, so
// their causal extents and masks are identical, and every K/V tile in LDS serves both heads (half the DMA
// per query of fa_fwd_kernel).  The two halves run one s_barrier apart: while one half issues its MFMA
// segment (S_i = K_i Q^T, then O^T += V_{i-1}^T P_{i-1}^T, 32 MFMAs) its SIMD partner runs its VALU segment
// (softmax of S_i, tile DMA, the next segment's first LDS operands), then they swap, so each SIMD's matrix
// pipe is fed by one of its two waves in every phase (MI355X_MICROARCH 'Two waves per SIMD';
// the free-running two-workgroup pairing of fa_fwd_kernel lets both waves of a SIMD sit in softmax at once).
//
// LDS: a ring of PP_R units of 32 KB; unit u (slot u % PP_R) = K_u (bytes 0-16K, loaded by waves 0-3) and
// V_{u-1} (16-32K, waves 4-7) -- exactly what MFMA segment u reads, so a unit is born and retired as one.
// Phases (A = waves 0-3, B = 4-7): A's MFMA segment i is phase 2i and its VALU segment 2i + 1; B's are
// 2i + 1 and 2i + 2.  Unit u is read from phase 2u - 1 (operand prefetch) to 2u + 1, so it must be
// visible at the barrier ending phase 2u - 2: A waits for it at the end of MFMA segment u - 1, B at the end
// of VALU segment u - 2.  Step i issues unit i + 3 (TH_PP_NMF pieces in the MFMA gaps of its S chain, the
// rest in its VALU segment) into the slot of unit i - 1, last read at phase 2i - 1.
constexpr int PP_R = 4, PP_SLOT = 2 * F_BN * 256;
#ifndef TH_PP_PRIO
#define TH_PP_PRIO 0
#endif
#ifndef TH_PP_SHIFT
#define TH_PP_SHIFT 0
#endif
#ifndef TH_PP_NMF
#define TH_PP_NMF 0  // of a unit's 4 DMA pieces per wave, how many go into the MFMA gaps (the rest: VALU segment)
#endif
#ifndef TH_PP_YPRIO
#define TH_PP_YPRIO 0  // static s_setprio 1 for waves 4-7 (MI355X_MICROARCH 'Two waves per SIMD' item 4)
#endif
#ifdef TH_PP_STAMP
// diagnostic build only: s_memtime at the segment boundaries of workgroup 0 (the heaviest q block),
// kept in spare LDS while the kernel runs (an LDS write does not disturb the counted vmcnt waits)
constexpr int PP_STAMP_STEPS = 72;
__device__ unsigned long long th_pp_stamp_buf[8 * PP_STAMP_STEPS * 5];
#define PP_STAMP(i, k)                                                                                  \
  do {                                                                                                  \
    if (blockIdx.x == 0 && lane == 0 && (i) < PP_STAMP_STEPS)                                           \
      stamp_lds[(wu * PP_STAMP_STEPS + (i)) * 5 + (k)] = __builtin_amdgcn_s_memtime();                  \
  } while (0)
#else
#define PP_STAMP(i, k) \
  do {                 \
  } while (0)
#endif

// does this wave load pieces of unit u (T key tiles -> units 0..T)?
__device__ __forceinline__ bool pp_has(int wu, int u, int T) { return wu < 4 ? u < T : (u >= 1 && u <= T); }
// wait until this wave's pieces of unit `need` have landed, given units up to `last` issued (`part` of
// unit last's 4 pieces so far)
__device__ __forceinline__ void pp_wait(int wu, int need, int last, int part, int T) {
  if (need > T) return;
  int n = 0;
  for (int u = need + 1; u <= last; ++u) n += pp_has(wu, u, T) ? (u == last ? part : 4) : 0;
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void pp_barrier() { asm volatile("s_barrier" ::: "memory"); }

__global__ __launch_bounds__(512, 1) void fa_fwd_pp_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    ushort* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale_log2, int causal) {
  __shared__ __attribute__((aligned(1024))) char smem[PP_R * PP_SLOT];
#ifdef TH_PP_STAMP
  __shared__ unsigned long long stamp_lds[8 * PP_STAMP_STEPS * 5];
#endif
  const int G = Hq / Hkv, P = G >> 1;
  const int nqb = (S + F_BM - 1) / F_BM;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int per = nqb * P, grp = L / per, r = L % per;
  const int b = grp / Hkv, hk = grp % Hkv, qb = nqb - 1 - r / P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const bool half = wu >= 4;
  const int hq = hk * G + 2 * (r % P) + (half ? 1 : 0);
  const int q0 = qb * F_BM + (wu & 3) * 32;  // wave-uniform (scalar branches on it)
  const int q = q0 + c32;
  const ushort* Qb = Q + b * bs + (long)hq * HD;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;

  bf16x8 qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    ushort8 u = q < S ? *reinterpret_cast<const ushort8*>(Qb + (long)q * ld + 16 * s + 8 * h) : ushort8(0);
#pragma unroll
    for (int e = 0; e < 8; ++e) u[e] = f2bf(bf2f(u[e]) * scale_log2);
    qf[s] = as_bf(u);
  }
  const int kv_end = causal ? min(S, qb * F_BM + F_BM) : S;
  const int T = (kv_end + F_BN - 1) / F_BN;
  unsigned rc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) rc[u] = img_rc((w & 3) * 4096 + u * 1024 + lane * 16);
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem + (half ? F_BN * 256 : 0) + (wu & 3) * 4096;
  const ushort* src = half ? Vb : Kb;
  // piece p (of 4) of this wave's share of unit u: K rows of tile u (A) or V rows of tile u - 1 (B)
  auto issue_piece = [&](int u, int p) {
    if (u > T || !pp_has(wu, u, T)) return;
    const int tile = half ? u - 1 : u;
    const int row = min(tile * F_BN + (int)(rc[p] & 255), S - 1);
    glds16(src, (unsigned)(row * ld + (rc[p] >> 8) * 8) * 2u, lds0 + (u % PP_R) * PP_SLOT + p * 1024);
  };
  auto issue = [&](int u) {
#pragma unroll
    for (int p = 0; p < 4; ++p) issue_piece(u, p);
  };
  __builtin_amdgcn_s_waitcnt(0x0F70);  // Q loads retired by a wait the compiler sees (vmcnt(0))
  issue(0);
  issue(1);
  issue(2);
  pp_wait(wu, 0, min(2, T), 4, T);
  pp_barrier();

  auto kimg = [&](int u) { return smem + (u % PP_R) * PP_SLOT; };
  // this wave's key tiles 0 .. Tw - 1 (wave-uniform; the tiles above its diagonal are skipped)
  const int Tw = causal ? min(T, (q0 + 31) / F_BN + 1) : T;
  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x16(0.f);
  float m_i = -INFINITY, l_i = 0.f;
  float m_base = 0.f;  // TH_PP_SHIFT: the S chains start from s_init = -m_base (C = 0 otherwise)
  f32x16 s_init = f32x16(0.f);  // the MFMA reads C from here: no copies
  f32x16 sacc[2];
  bf16x8 pf[4], ka[3][2];
  // first two steps' operands of MFMA segment i's S chain (K_i rows), read in the VALU segment before it;
  // V^T's first k-step is read during the chain's last steps, so 16 operand registers live across the
  // barrier.  Unconditional: a segment without S never reads them.
  auto prefetch = [&](int i) {
    const char* ks = kimg(i);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      ka[t][0] = lds_row(ks, c32, 2 * t + h);
      ka[t][1] = lds_row(ks, 32 + c32, 2 * t + h);
    }
  };
  // MFMA segment i: S_i (DO_S), then PV_{i-1} (DO_PV).  Called with constant flags only, so each loop
  // below has one straight-line body (branches inside a body cost phi copies of the operand registers).
  auto mfma_seg = [&](int i, bool DO_S, bool DO_PV) __attribute__((always_inline)) {
    const char* ks = kimg(i);
    const char* vs = ks + F_BN * 256;
    bf16x8 vt[4];
    if (DO_S) {  // K-row operands two steps ahead of their MFMAs (one step leaves the LDS latency exposed)
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s + 2 < 8) {
          ka[(s + 2) % 3][0] = lds_row(ks, c32, 2 * s + 4 + h);
          ka[(s + 2) % 3][1] = lds_row(ks, 32 + c32, 2 * s + 4 + h);
        } else if (s == 6 && DO_PV) {
#pragma unroll
          for (int d = 0; d < 4; ++d) vt[d] = lds_tr(vs, 0, 32 * d, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        sacc[0] = mfma(ka[s % 3][0], qf[s], s == 0 ? s_init : sacc[0]);
        if ((s & 1) && (s >> 1) < TH_PP_NMF) issue_piece(i + 3, s >> 1);  // DMA pieces in the MFMA gaps
        sacc[1] = mfma(ka[s % 3][1], qf[s], s == 0 ? s_init : sacc[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int p = 0; p < TH_PP_NMF; ++p) issue_piece(i + 3, p);
      if (DO_PV) {
#pragma unroll
        for (int d = 0; d < 4; ++d) vt[d] = lds_tr(vs, 0, 32 * d, lane);
      }
    }
    if (DO_PV) {
#pragma unroll
      for (int ks4 = 0; ks4 < 4; ++ks4) {
        bf16x8 nx[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) nx[d] = ks4 < 3 ? lds_tr(vs, 16 * ks4 + 16, 32 * d, lane) : vt[d];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = mfma(vt[d], pf[ks4], o[d]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int d = 0; d < 4; ++d) vt[d] = nx[d];
      }
    }
  };
  // softmax of S_i -> P_i (bf16 operands pf), running max / sum, O rescale when the max moved past 2^8
  auto softmax = [&](int i) __attribute__((always_inline)) {
    if (TH_PP_PRIO) __builtin_amdgcn_s_setprio(1);  // the VALU segment is the phase's critical path
    const int kbase = i * F_BN;
    const bool need_mask = (causal && kbase + F_BN - 1 > q0) || (kbase + F_BN > S);  // wave-uniform
    if (need_mask) {
      const int kmax = (causal ? min(q, S - 1) : S - 1) - kbase - 4 * h;  // last visible key, tile-relative
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr)
          sacc[kb][rr] = (32 * kb + (rr & 3) + 8 * (rr >> 2) <= kmax) ? sacc[kb][rr] : -INFINITY;
    }
    float mt = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) mt = fmaxf(mt, sacc[kb][rr]);
    mt = half_swap_max(mt);
    if (!__all(mt + m_base - m_i <= F_DEFER_THR)) {  // DEFER of fa_fwd_kernel
      const float m_new = fmaxf(m_i, mt + m_base);
      const float mu = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = fast_exp2(m_i - mu);
      l_i *= alpha;
#pragma unroll
      for (int d = 0; d < 4; ++d) o[d] *= alpha;
      m_i = m_new;
      if (TH_PP_SHIFT) {  // rebase this tile's scores and the next chains' start
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sacc[kb] -= mu - m_base;
        m_base = mu;
        s_init = f32x16(-mu);
      }
    }
    const float m_use = TH_PP_SHIFT ? 0.f : (m_i == -INFINITY ? 0.f : m_i);
    float rs4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const float p = fast_exp2(TH_PP_SHIFT ? sacc[kb][rr] : sacc[kb][rr] - m_use);
        sacc[kb][rr] = p;
        rs4[rr & 3] += p;
      }
    pf[0] = pack8(sacc[0], 0);
    pf[1] = pack8(sacc[0], 8);
    pf[2] = pack8(sacc[1], 0);
    pf[3] = pack8(sacc[1], 8);
    const float rs = (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);
    l_i += half_swap_sum(rs);
    if (TH_PP_PRIO) {
      if (TH_PP_YPRIO && half) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
  };
  // the two barriers of step i around the VALU segment (A waits for unit i + 1 before the first, B for
  // unit i + 2 before the second)
  auto sync_mid = [&](int i) {
    if (!half) pp_wait(wu, i + 1, min(i + 3, T), i + 3 <= T ? TH_PP_NMF : 4, T);
    pp_barrier();
  };
  auto sync_end = [&](int i) {
#pragma unroll
    for (int p = TH_PP_NMF; p < 4; ++p) issue_piece(i + 3, p);
    if (i < T) prefetch(i + 1);
    if (half) pp_wait(wu, i + 2, min(i + 3, T), 4, T);
    pp_barrier();
  };
  prefetch(0);
  if (TH_PP_YPRIO && half) __builtin_amdgcn_s_setprio(1);
  if (half) pp_barrier();  // B sits out A's first MFMA segment

  PP_STAMP(0, 0);
  mfma_seg(0, true, false);
  PP_STAMP(0, 1);
  sync_mid(0);
  PP_STAMP(0, 2);
  softmax(0);
  PP_STAMP(0, 3);
  sync_end(0);
  PP_STAMP(0, 4);
  for (int i = 1; i < Tw; ++i) {
    PP_STAMP(i, 0);
    mfma_seg(i, true, true);
    PP_STAMP(i, 1);
    sync_mid(i);
    PP_STAMP(i, 2);
    softmax(i);
    PP_STAMP(i, 3);
    sync_end(i);
    PP_STAMP(i, 4);
  }
  mfma_seg(Tw, false, true);  // PV of the wave's last tile
  sync_mid(Tw);
  sync_end(Tw);
  for (int i = Tw + 1; i <= T; ++i) {  // tiles above this wave's diagonal: barriers and DMA only
#pragma unroll
    for (int p = 0; p < TH_PP_NMF; ++p) issue_piece(i + 3, p);
    sync_mid(i);
    sync_end(i);
  }
  if (!half) pp_barrier();  // match B's extra barrier
#ifdef TH_PP_STAMP
  if (blockIdx.x == 0) {
    __syncthreads();
    for (int t = tid; t < 8 * PP_STAMP_STEPS * 5; t += 512) th_pp_stamp_buf[t] = stamp_lds[t];
  }
#endif

  if (q < S) {
    const float inv_l = l_i > 0.f ? 1.f / l_i : 0.f;
    store_row_t21(O + b * bso + (long)q * ldo + (long)hq * HD, o, inv_l, h);
    if (h == 0) LSE[((long)b * Hq + hq) * S + q] = (m_i + log2f(l_i)) * LN2;
  }
}
#endif  // TH_FA_DIAG (ping-pong forward)

// ------------------------------------------------------------------------------- dQ kernel
// dQ: wave priority around the MFMA chains (round 1 measured it neutral on the older dQ body)
#ifndef TH_DQ_PRIO_ON
#define TH_DQ_PRIO_ON 1
#endif
#define TH_DQ_PRIO(p)                                     \
  do {                                                    \
    if (TH_DQ_PRIO_ON) __builtin_amdgcn_s_setprio(p);    \
  } while (0)
#ifndef TH_DQ_AHEAD
#define TH_DQ_AHEAD 1  // 0: reads issued right before their MFMA (compiler order)
#endif
#ifndef TH_DQ_PREKB
#define TH_DQ_PREKB 1
#endif
#ifndef TH_DQ_TR_AHEAD
#define TH_DQ_TR_AHEAD 1  // K^T operand look-ahead of the dQ chain in d-steps (1 or 2)
#endif
// SPREAD (with DMA): tile j+1's 8 LDS-DMA pieces issued one per MFMA pair of the first S|dP chain
// (no VALU there) instead of 8 in a row after the barrier -- the kf lesson: a piece costs the issuing
// wave 60-185 cycles (profiles/r04_flash/)
// L2OUT: also write -lse * log2(e) of each query into Dl[B*Hq*S + ...] (the second half of the
// delta buffer), so kf VAR bit12 starts its S' chain from it without a multiply per element
template <bool KVMAJOR, bool DMA, bool SPREAD = false, bool L2OUT = false>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    const ushort* __restrict__ dO, const ushort* __restrict__ O, const float* __restrict__ LSE,
    float* __restrict__ Dl, ushort* __restrict__ dQ, int B, int S, int Hq, int Hkv, long ld, long bs, long ldo,
    long bso, float scale, float scale_log2, int causal, const float* __restrict__ rcos,
    const float* __restrict__ rsin) {
  // DMA: two K|V image pairs (64 KB), else one pair staged through registers
  __shared__ __attribute__((aligned(1024))) char smem_dq[(DMA ? 2 : 1) * 2 * F_BN * 256];
  const int nqb = (S + F_BM - 1) / F_BM;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b, hq, qb;
  q_block_map<KVMAJOR>(L, nqb, B, Hq, Hkv, b, hq, qb);
  const int hk = hq / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
  const int q0 = qb * F_BM + w * 32;
  const int q = q0 + c32;
  const ushort* Qb = Q + b * bs + (long)hq * HD;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;
  const ushort* dOb = dO + b * bso + (long)hq * HD;
  const ushort* Ob = O + b * bso + (long)hq * HD;

  bf16x8 qf[8], gf[8];
  ushort8 qraw[8];
  // delta = rowsum(dO * O) of this lane's query, formed here from the dO row the kernel loads anyway
  // (the two half-waves hold the two halves of the row) and written for the dK|dV kernel -- no
  // separate delta pass over dO and O
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qraw[s] = q < S ? *reinterpret_cast<const ushort8*>(Qb + (long)q * ld + 16 * s + 8 * h) : ushort8(0);
    const ushort8 graw = q < S ? *reinterpret_cast<const ushort8*>(dOb + (long)q * ldo + 16 * s + 8 * h) : ushort8(0);
    const ushort8 oraw = q < S ? *reinterpret_cast<const ushort8*>(Ob + (long)q * ldo + 16 * s + 8 * h) : ushort8(0);
    gf[s] = as_bf(graw);
#pragma unroll
    for (int e = 0; e < 8; ++e) dpart += bf2f(oraw[e]) * bf2f(graw[e]);
  }
  const long st = ((long)b * Hq + hq) * S;
  const float lse2 = q < S ? LSE[st + q] * LOG2E : INFINITY;
  const float dsum = half_swap_sum(dpart);
  if (q < S && h == 0) Dl[st + q] = dsum;
  if (L2OUT && q < S && h == 0) Dl[(long)B * Hq * S + st + q] = -lse2;
  const float dlt = q < S ? dsum : 0.f;
  // Row constants as the initial accumulators (the query is this lane's for the whole kernel): Q is
  // prescaled by softmax_scale * log2(e) once (as the forward's PRESCALE variant does), the S chain
  // starts from -lse2 and the dP chain from -delta, so p = exp2(acc) and dS = p * acc' -- two VALU
  // per score instead of four (fma, exp, sub, mul).
#pragma unroll
  for (int s = 0; s < 8; ++s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) qraw[s][e] = f2bf(bf2f(qraw[s][e]) * scale_log2);
    qf[s] = as_bf(qraw[s]);
  }
  const f32x16 s_init = f32x16(-lse2), p_init = f32x16(-dlt);

  const int kv_end = causal ? min(S, qb * F_BM + F_BM) : S;
  const int ntiles = (kv_end + F_BN - 1) / F_BN;
  ushort8 kr[4], vr[4];
  unsigned rc[4];
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem_dq;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto dma_tile = [&](int jt) { dma_kv_tile(Kb, Vb, ld, S, jt, lds0, wu, rc); };
  if (DMA) {
    // retire the Q / dO / LSE / delta loads HERE with a real s_waitcnt (vmcnt(0)) the compiler's
    // wait insertion sees: otherwise it places the waits for them at their first use inside the
    // loop, where each iteration would also wait for the tile DMA it has just issued
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int u = 0; u < 4; ++u) rc[u] = img_rc(w * 4096 + u * 1024 + lane * 16);
    dma_tile(0);
  } else {
    stage_load<4>(kr, Kb, ld, 0, S, tid);
    stage_load<4>(vr, Vb, ld, 0, S, tid);
  }
  f32x16 dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dq[d] = f32x16(0.f);

  for (int j = 0; j < ntiles; ++j) {
    char* ks = smem_dq + (DMA ? (j & 1) * (2 * F_BN * 256) : 0);
    char* vs = ks + F_BN * 256;
    if (DMA) {
      wait_dma_barrier();  // tile j landed (every wave's DMA); everyone is past tile j-1
      if (!SPREAD && j + 1 < ntiles) dma_tile(j + 1);
    } else {
      __syncthreads();
      stage_store<4>(ks, kr, tid);
      stage_store<4>(vs, vr, tid);
      __syncthreads();
      if (j + 1 < ntiles) {
        stage_load<4>(kr, Kb, ld, (j + 1) * F_BN, S, tid);
        stage_load<4>(vr, Vb, ld, (j + 1) * F_BN, S, tid);
      }
    }
    const int kbase = j * F_BN;
    // SPREAD: the tile DMA'd this iteration (the last tile re-loads itself into the free image pair,
    // which nobody reads again: no branch around the pieces)
    const int jd = min(j + 1, ntiles - 1);
    if (causal && kbase > q0 + 31) {
      if (SPREAD) dma_tile(jd);  // this wave skips the tile but still owes its DMA share
      continue;
    }
    const bool need_mask = (causal && kbase + F_BN - 1 > q0) || (kbase + F_BN > S);
    // TH_DQ_PREKB: the second key half's first S|dP operands are read during the first half's dQ chain
    bf16x8 pka[2], pva[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {  // 32-key halves: keeps only one S^T / dP^T pair live
      f32x16 sacc = s_init, pacc = p_init;
#if TH_DQ_AHEAD
      {  // K/V row operands read two k-steps ahead of the MFMAs that use them (2 gaps of latency cover)
        bf16x8 ka[2], va[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (TH_DQ_PREKB && DMA && kb == 1) {
            ka[s] = pka[s];
            va[s] = pva[s];
          } else {
            ka[s] = lds_row(ks, 32 * kb + c32, 2 * s + h);
            va[s] = lds_row(vs, 32 * kb + c32, 2 * s + h);
          }
        }
        TH_DQ_PRIO(1);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          bf16x8 kn = ka[s & 1], vn = va[s & 1];
          if (s + 2 < 8) {
            kn = lds_row(ks, 32 * kb + c32, 2 * s + 4 + h);
            vn = lds_row(vs, 32 * kb + c32, 2 * s + 4 + h);
          }
          __builtin_amdgcn_sched_barrier(0);
          sacc = mfma(ka[s & 1], qf[s], sacc);
          if (SPREAD && kb == 0) dma_kv_piece(Kb, Vb, ld, S, jd, lds0, wu, rc, s);
          pacc = mfma(va[s & 1], gf[s], pacc);
          __builtin_amdgcn_sched_barrier(0);
          ka[s & 1] = kn;
          va[s & 1] = vn;
        }
        TH_DQ_PRIO(0);
      }
#else
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        sacc = mfma(lds_row(ks, 32 * kb + c32, 2 * s + h), qf[s], sacc);
        pacc = mfma(lds_row(vs, 32 * kb + c32, 2 * s + h), gf[s], pacc);
      }
#endif
      // Only diagonal / ragged tiles are masked: a wave-uniform branch keeps the v_cmp + v_cndmask
      // pair per score (a third of this VALU block) off every other tile.
      if (need_mask) {
        // tile-relative last visible key of this lane's query
        const int kmax = (causal ? min(q, S - 1) : S - 1) - kbase - 32 * kb - 4 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fast_exp2(sacc[r]);
          p = ((r & 3) + 8 * (r >> 2) <= kmax) ? p : 0.f;
          sacc[r] = p * pacc[r];  // dS^T = P (dP - delta)
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[r] = fast_exp2(sacc[r]) * pacc[r];
      }
      const bf16x8 s0 = pack8(sacc, 0), s1 = pack8(sacc, 8);
#if TH_DQ_AHEAD
#if TH_DQ_TR_AHEAD == 2
      {  // K^T operands two d-steps ahead (ring of 3)
        bf16x8 kt[3][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          kt[t][0] = lds_tr(ks, 32 * kb, 32 * t, lane);
          kt[t][1] = lds_tr(ks, 32 * kb + 16, 32 * t, lane);
        }
        TH_DQ_PRIO(1);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (d + 2 < 4) {
            kt[(d + 2) % 3][0] = lds_tr(ks, 32 * kb, 32 * d + 64, lane);
            kt[(d + 2) % 3][1] = lds_tr(ks, 32 * kb + 16, 32 * d + 64, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
          dq[d] = mfma(kt[d % 3][0], s0, dq[d]);
          dq[d] = mfma(kt[d % 3][1], s1, dq[d]);
          __builtin_amdgcn_sched_barrier(0);
        }
        TH_DQ_PRIO(0);
      }
#else
      {  // K^T operands one d-step ahead
        bf16x8 t0 = lds_tr(ks, 32 * kb, 0, lane), t1 = lds_tr(ks, 32 * kb + 16, 0, lane);
        TH_DQ_PRIO(1);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16x8 n0 = t0, n1 = t1;
          if (d < 3) {
            n0 = lds_tr(ks, 32 * kb, 32 * d + 32, lane);
            n1 = lds_tr(ks, 32 * kb + 16, 32 * d + 32, lane);
          }
          if (TH_DQ_PREKB && DMA && kb == 0 && d == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              pka[s] = lds_row(ks, 32 + c32, 2 * s + h);
              pva[s] = lds_row(vs, 32 + c32, 2 * s + h);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          dq[d] = mfma(t0, s0, dq[d]);
          dq[d] = mfma(t1, s1, dq[d]);
          __builtin_amdgcn_sched_barrier(0);
          t0 = n0;
          t1 = n1;
        }
        TH_DQ_PRIO(0);
      }
#endif
#else
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        dq[d] = mfma(lds_tr(ks, 32 * kb, 32 * d, lane), s0, dq[d]);
        dq[d] = mfma(lds_tr(ks, 32 * kb + 16, 32 * d, lane), s1, dq[d]);
      }
#endif
    }
  }
  if (q < S) {
    if (rcos != nullptr) {  // rotary backward in the epilogue (position = the query's index in its sequence)
      rope_bwd_rows(dq, rcos, rsin, q, h);
    }
    store_row_t21(dQ + b * bs + (long)q * ld + (long)hq * HD, dq, scale, h);
  }
}

// ---------------------------------------------------------------------------- dK/dV kernel
// 8 waves x 32 keys = 256 keys of one (batch, kv head) per workgroup; the K/V block lives in
// LDS (128 KB) and is re-read every query tile (the reads are kept in the loop on purpose:
// hoisting them would cost 64 VGPRs and drop the kernel to one wave per SIMD).
constexpr int B_BK = 256, B_BQ = 32, B_THREADS = 512;

template <bool KVMAJOR>
__global__ __launch_bounds__(B_THREADS, 2) void fa_bwd_dkv_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    const ushort* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Dl,
    ushort* __restrict__ dK, ushort* __restrict__ dV, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale, float scale_log2, int causal, int young_prio) {
  // K image 64 KB | V image 64 KB | Q tile 8 KB | dO tile 8 KB | lse 128 B | delta 128 B
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ks = smem;
  char* vs = ks + B_BK * 256;
  char* qs = vs + B_BK * 256;
  char* gs = qs + B_BQ * 256;
  float* ls = reinterpret_cast<float*>(gs + B_BQ * 256);
  float* ds = ls + B_BQ;
  const int nkb = (S + B_BK - 1) / B_BK;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b, hk, kblk;
  if (KVMAJOR) {  // the key blocks of one (batch, kv head) together: they stream the same Q/dO
    const int grp = L / nkb, r = L % nkb;
    b = grp / Hkv;
    hk = grp % Hkv;
    kblk = causal ? r : nkb - 1 - r;  // causal: low key blocks are heaviest
  } else {
    const int per = Hkv * B;
    kblk = causal ? L / per : nkb - 1 - L / per;
    const int rem = L % per;
    b = rem / Hkv;
    hk = rem % Hkv;
  }
  const int G = Hq / Hkv;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
  const int kblk0 = kblk * B_BK;
  const int k0 = kblk0 + 32 * w;
  const int key = k0 + c32;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;
  {
    // 256 rows x 16 chunks = 4096 chunks per tensor, 8 per thread; every 8-lane write group
    // covers 2 rows x 4 chunks = 128 contiguous bytes (conflict-free ds_write_b128, see stage_load)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 32 * i + 2 * ((tid >> 3) & 15) + ((tid >> 2) & 1), ch = 4 * (tid >> 7) + (tid & 3);
      const bool ok = kblk0 + row < S;
      const long go = (long)(kblk0 + row) * ld + (ch << 3);
      *reinterpret_cast<ushort8*>(ks + img_off(row, ch)) = ok ? *reinterpret_cast<const ushort8*>(Kb + go) : ushort8(0);
      *reinterpret_cast<ushort8*>(vs + img_off(row, ch)) = ok ? *reinterpret_cast<const ushort8*>(Vb + go) : ushort8(0);
    }
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) { dk[d] = f32x16(0.f); dv[d] = f32x16(0.f); }

  const int nqt = (S + B_BQ - 1) / B_BQ;
  const int qt0 = causal ? kblk0 / B_BQ : 0;
  const int per_head = nqt - qt0;
  const int total = G * per_head;
  // Q/dO tile: 32 rows x 16 chunks = 512 chunks -> one per thread per tensor (conflict-free map:
  // 8-lane write groups cover 2 rows x 4 chunks)
  const int srow = 2 * ((tid >> 3) & 15) + ((tid >> 2) & 1), sch = 4 * (tid >> 7) + (tid & 3);
  ushort8 qr, gr;
  float lr = 0.f, dr = 0.f;
  // (head, query tile) of the prefetch and of the current iteration, advanced incrementally (a
  // runtime division per iteration cost ~80 scalar instructions per wave)
  int pf_h = 0, pf_t = 0, cur_t = 0;
  auto prefetch = [&](int h_i, int t_i) {
    const int hq = hk * G + h_i;
    const int qq0 = (qt0 + t_i) * B_BQ;
    // rows past S are clamped to S-1 (finite data; their lse = +inf makes P and dS exactly 0), so
    // the loads are unconditional: no exec-mask branch around them
    const int row = min(qq0 + srow, S - 1);
    qr = *reinterpret_cast<const ushort8*>(Q + b * bs + (long)hq * HD + (long)row * ld + (sch << 3));
    gr = *reinterpret_cast<const ushort8*>(dO + b * bso + (long)hq * HD + (long)row * ldo + (sch << 3));
    if (tid < B_BQ) {
      const int qq = qq0 + tid;
      const long st = ((long)b * Hq + hq) * S;
      const int qc = min(qq, S - 1);
      lr = LSE[st + qc];  // scaled by log2(e) when stored: no use right after the load
      dr = Dl[st + qc];
      lr = qq < S ? lr : INFINITY;
      dr = qq < S ? dr : 0.f;
    }
  };
  if (total > 0) prefetch(0, 0);
  int krow = 32 * w + c32;
  // static priority for the second-dispatched half (waves 4-7): it otherwise loses VALU
  // arbitration to its SIMD partner on every segment (guide T5, static form)
  if (young_prio && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  for (int it = 0; it < total; ++it) {
    __syncthreads();
    *reinterpret_cast<ushort8*>(qs + img_off(srow, sch)) = qr;
    *reinterpret_cast<ushort8*>(gs + img_off(srow, sch)) = gr;
    if (tid < B_BQ) { ls[tid] = lr * LOG2E; ds[tid] = dr; }
    __syncthreads();
    const int qbase = (qt0 + cur_t) * B_BQ;
    if (++cur_t == per_head) cur_t = 0;
    if (++pf_t == per_head) { pf_t = 0; ++pf_h; }
    if (it + 1 < total) prefetch(pf_h, pf_t);
    if (causal && qbase + B_BQ - 1 < k0) continue;  // all queries of the tile precede our keys
    asm volatile("" : "+v"(krow));  // keep the K/V row reads inside the loop (see header)
    f32x16 sacc = f32x16(0.f), pacc = f32x16(0.f);
#pragma unroll
    for (int s = 0; s < 8; ++s) sacc = mfma(lds_row(qs, c32, 2 * s + h), lds_row(ks, krow, 2 * s + h), sacc);
#pragma unroll
    for (int s = 0; s < 8; ++s) pacc = mfma(lds_row(gs, c32, 2 * s + h), lds_row(vs, krow, 2 * s + h), pacc);
    // Masking is branch-free inside the tile: a wave-uniform test decides whether this tile needs
    // it at all, then every element is a select.  (Written as `if (need_mask && (key >= S || ...))`
    // the short-circuit logic compiled to three exec-mask branches PER ELEMENT -- 45 saveexec
    // blocks per iteration.)  Query row ro + 4h sees this key iff key - qbase - 4h <= ro.
    const bool tile_mask = (causal && qbase < k0 + 31) || (k0 + 31 >= S);  // wave-uniform
    const int kq = causal ? key - qbase - 4 * h : -0x40000000;
    // one per-lane threshold: the element (row ro) is zeroed iff mthr > ro (no per-element SALU
    // mask algebra: a v_cmp + v_cndmask each)
    const int mthr = tile_mask ? (key >= S ? 0x7fffffff : kq) : -0x7fffffff;
    // lse / delta of the accumulator rows (4h + (r&3) + 8(r>>2)): four 16-byte reads each
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4v lv = *reinterpret_cast<const float4v*>(ls + 4 * h + 8 * g);
      const float4v dv4 = *reinterpret_cast<const float4v*>(ds + 4 * h + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e, ro = e + 8 * g;
        float p = fast_exp2(sacc[r] * scale_log2 - lv[e]);
        p = mthr > ro ? 0.f : p;
        sacc[r] = p;
        pacc[r] = p * (pacc[r] - dv4[e]);
      }
    }
    const bf16x8 p0 = pack8(sacc, 0), p1 = pack8(sacc, 8);
    const bf16x8 s0 = pack8(pacc, 0), s1 = pack8(pacc, 8);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dv[d] = mfma(lds_tr(gs, 0, 32 * d, lane), p0, dv[d]);
      dv[d] = mfma(lds_tr(gs, 16, 32 * d, lane), p1, dv[d]);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dk[d] = mfma(lds_tr(qs, 0, 32 * d, lane), s0, dk[d]);
      dk[d] = mfma(lds_tr(qs, 16, 32 * d, lane), s1, dk[d]);
    }
  }
  if (key < S) {
    ushort* krow_o = dK + b * bs + (long)key * ld + (long)hk * HD;
    ushort* vrow_o = dV + b * bs + (long)key * ld + (long)hk * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ushort4v ok, ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ok[e] = f2bf(dk[d][4 * g + e] * scale);
          ov[e] = f2bf(dv[d][4 * g + e]);
        }
        *reinterpret_cast<ushort4v*>(krow_o + 32 * d + 8 * g + 4 * h) = ok;
        *reinterpret_cast<ushort4v*>(vrow_o + 32 * d + 8 * g + 4 * h) = ov;
      }
  }
}
// ------------------------------------------------------------ paired key-centric dK | dV kernel
// The fused dK/dV kernel above needs 128 accumulator VGPRs (dK and dV) and so cannot keep its
// K/V operands in registers: every S / dP MFMA reads BOTH operands from LDS, and the K/V block
// costs 128 KB of LDS.  In the paired kernels each 32-key slice is owned by a PAIR of waves with
// one accumulator each:
//   dV wave:  phase 1  S = Q K^T -> P (registers + LDS exchange)   phase 2  dV^T += dO^T P
//   dK wave:  phase 1  dP = dO V^T                                 phase 2  dS = P (dP - delta),
//                                                                           dK^T += Q^T dS
// Both roles run 16 + 16 MFMAs per 64-query tile (balanced, no GEMM recomputed), hold only 64
// accumulator VGPRs, keep their K (dV wave) or V (dK wave) fragments in registers for the whole
// kernel, and read one MFMA operand per instruction from LDS (like the dQ kernel).  P crosses
// from the dV wave to its partner through a lane-linear LDS slot (conflict-free wide
// ds_write/read), one barrier between the phases.  The pair shares one staged Q/dO tile
// (the dK waves stage Q + lse + delta, the dV waves dO).
// B4 S4096 32/8 heads: backward 2.64 -> 2.29 ms against the fused kernel (profiles/r01_flash_v3).
// (Measured on the way: one role per workgroup streaming the tile twice = no faster than the
// fused kernel; paired roles that each recompute S = -9 %; LDS double-buffering = no change.)
constexpr int C_BQ = 64, KC_TILE = 2 * C_BQ * 256 + 2 * C_BQ * 4;  // one staged Q|dO|lse|delta tile

// ------------------------------------ paired dK | dV kernel, half width: two workgroups per CU
// The paired roles above in workgroups of 4 waves over 64 keys: one dK wave and one dV wave per
// 32-key slice, two slices.  The retired 8-wave kernel (kc, one workgroup per CU; its code and the
// one-barrier kc3 variant: profiles/r03_flash/retired_kc_kernels.patch) held one workgroup per
// CU, so its 8 waves pass the same two barriers per tile together and every phase boundary
// (barrier, first LDS operands, MFMA -> exp) is exposed on all of them at once (39.8 % MFMA busy,
// profiles/r02_flash).  With two independent workgroups per CU the waves of one SIMD belong to
// different barrier domains, as in the dQ kernel (60.5 % busy).  LDS per workgroup: two Q|dO
// tiles (DMA double buffer) + the P exchange of the two pairs, as bf16 (the value the dV MFMA
// consumes): 2 x 33 KB + 8 KB = 73 KB, two workgroups = 146 KB of the 160 KB.
constexpr int KH_BK = 64, KH_LDS = 2 * KC_TILE + 2 * 4096;

template <bool DK>
__device__ __forceinline__ void kh_body(const ushort* __restrict__ Q, const ushort* __restrict__ dO,
                                        const float* __restrict__ LSE, const float* __restrict__ Dl,
                                        const ushort* Kb, const ushort* Vb, ushort* __restrict__ out,
                                        char* smem, int b, int hk, int kblk0, int S, int Hq, int G, long ld,
                                        long bs, long ldo, long bso, float scale, float scale_log2, int causal,
                                        const float* __restrict__ rcos, const float* __restrict__ rsin) {
  // role-local ids: waves 0-1 are the dK role, 2-3 the dV role of the same 64 keys
  const int tid = threadIdx.x & 127, lane = tid & 63, w = tid >> 6, h = lane >> 5, c32 = lane & 31;
  // P exchange of pair w: [half][s0 | s1][lane] bf16x8, 4 KB
  bf16x8* pbuf = reinterpret_cast<bf16x8*>(smem + 2 * KC_TILE + w * 4096);
  const int k0 = kblk0 + 32 * w;
  const int key = k0 + c32;
  const ushort* fb = DK ? Vb : Kb;
  bf16x8 kf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    ushort8 u = key < S ? *reinterpret_cast<const ushort8*>(fb + (long)key * ld + 16 * s + 8 * h) : ushort8(0);
    if (!DK) {
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = f2bf(bf2f(u[e]) * scale_log2);
    }
    kf[s] = as_bf(u);
  }
  f32x16 acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x16(0.f);

  const int nqt = (S + C_BQ - 1) / C_BQ;
  const int qt0 = causal ? kblk0 / C_BQ : 0;
  const int per_head = nqt - qt0;
  const int total = G * per_head;
  // each role's 2 waves DMA its 16 KB image (Q for dK, dO for dV): 8 x 1 KB per wave
  unsigned rc[8];
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto dma_tile = [&](int h_i, int t_i, int buf) {
    const int hq = hk * G + h_i;
    const int qq0 = (qt0 + t_i) * C_BQ;
    const ushort* base = DK ? Q + b * bs + (long)hq * HD : dO + b * bso + (long)hq * HD;
    const long ldx = DK ? ld : ldo;
    const unsigned img = lds0 + buf * KC_TILE + (DK ? 0 : C_BQ * 256) + wu * 8192;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = min(qq0 + (int)(rc[u] & 255), S - 1);
      glds16(base, (unsigned)(row * ldx + (rc[u] >> 8) * 8) * 2u, img + u * 1024);
    }
  };
  float lr = 0.f, dr = 0.f;
  int lq = 0;
  auto load_ld = [&](int h_i, int t_i) {
    if (DK && tid < C_BQ) {
      const int hq = hk * G + h_i;
      lq = (qt0 + t_i) * C_BQ + tid;
      const long st = ((long)b * Hq + hq) * S;
      const int qc = min(lq, S - 1);
      lr = LSE[st + qc];
      dr = Dl[st + qc];
    }
  };
  auto write_ld = [&](int buf) {
    if (DK && tid < C_BQ) {
      float* l = reinterpret_cast<float*>(smem + buf * KC_TILE + 2 * C_BQ * 256);
      l[tid] = lq < S ? -lr * LOG2E : -INFINITY;  // negated (initial accumulators); past S: P = 0
      l[C_BQ + tid] = lq < S ? -dr : 0.f;
    }
  };
  int pf_h = 0, pf_t = 0, lh = 0, lt = 0, cur_t = 0;
  auto adv = [&](int& hh, int& tt) {
    if (++tt == per_head) { tt = 0; ++hh; }
  };
  __builtin_amdgcn_s_waitcnt(0x0F70);  // K/V fragment loads retired (a wait the compiler sees)
#pragma unroll
  for (int u = 0; u < 8; ++u) rc[u] = img_rc(wu * 8192 + u * 1024 + lane * 16);
  if (total > 0) {
    load_ld(0, 0);
    write_ld(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    dma_tile(0, 0, 0);
    adv(lh, lt);
    if (total > 1) load_ld(lh, lt);
  }
  for (int it = 0; it < total; ++it) {
    char* cur = smem + (it & 1) * KC_TILE;
    wait_dma_barrier();  // tile it landed; every wave is past tile it-1 (its buffer is free)
    if (it + 1 < total) {
      write_ld((it + 1) & 1);
      adv(pf_h, pf_t);
      dma_tile(pf_h, pf_t, (it + 1) & 1);
      adv(lh, lt);
      if (it + 2 < total) load_ld(lh, lt);
    }
    const char* qs = cur;
    const char* gs = cur + C_BQ * 256;
    const float* ls = reinterpret_cast<const float*>(cur + 2 * C_BQ * 256);
    const float* ds = ls + C_BQ;
    const int qbase = (qt0 + cur_t) * C_BQ;
    if (++cur_t == per_head) cur_t = 0;
    // phase 1: dK role dP' = dO V^T - delta, dV role S' = Q K^T - lse2 -> P (bf16, kept + to LDS)
    f32x16 c[2];
    bf16x8 sp[2][2];
    auto init_c = [&](int kb) {  // -delta (dK role) / -lse2 (dV role) of the half's 32 query rows
      const float* rowc = (DK ? ds : ls) + 32 * kb + 4 * h;
      const float4v r0 = *reinterpret_cast<const float4v*>(rowc), r1 = *reinterpret_cast<const float4v*>(rowc + 8),
                    r2 = *reinterpret_cast<const float4v*>(rowc + 16), r3 = *reinterpret_cast<const float4v*>(rowc + 24);
      c[kb] = __builtin_shufflevector(__builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7),
                                      __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3, 4, 5, 6, 7,
                                      8, 9, 10, 11, 12, 13, 14, 15);
    };
    // the half's 8-MFMA chain, row operands read two k-steps ahead; fill(s) runs in MFMA gap s
    auto chain1 = [&](int kb, auto&& fill) {
      const char* img = DK ? gs : qs;
      bf16x8 xa[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) xa[s] = lds_row(img, 32 * kb + c32, 2 * s + h);
      FA_PRIO(1);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        bf16x8 xn = xa[s & 1];
        if (s + 2 < 8) xn = lds_row(img, 32 * kb + c32, 2 * s + 4 + h);
        __builtin_amdgcn_sched_barrier(0);
        c[kb] = mfma(xa[s & 1], kf[s], c[kb]);
        fill(s);
        __builtin_amdgcn_sched_barrier(0);
        xa[s & 1] = xn;
      }
      FA_PRIO(0);
    };
    auto no_fill = [](int) {};
    auto publish_p = [&](int kb) {
      sp[kb][0] = pack8(c[kb], 0);
      sp[kb][1] = pack8(c[kb], 8);
      pbuf[(2 * kb) * 64 + lane] = sp[kb][0];
      pbuf[(2 * kb + 1) * 64 + lane] = sp[kb][1];
    };
    // Interleaved dV schedule (both halves live, neither on the diagonal): half 0's exponentials run
    // two per MFMA gap of half 1's chain instead of between the chains (MI355X_MICROARCH issue
    // costs: a gap runs ~max(32, sum of its issue costs), the MFMA's own 8 included, and a v_exp
    // costs 8, so two fit).  Diagonal / partly-skipped tiles keep the plain order.
    const bool fast1 = !DK && !(causal && qbase < k0 + 31);
    if (fast1) {
      init_c(0);
      init_c(1);
      chain1(0, no_fill);
      chain1(1, [&](int s) {
        c[0][2 * s] = fast_exp2(c[0][2 * s]);
        c[0][2 * s + 1] = fast_exp2(c[0][2 * s + 1]);
      });
      publish_p(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) c[1][r] = fast_exp2(c[1][r]);
      publish_p(1);
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int q0 = qbase + 32 * kb;
        if (causal && q0 + 31 < k0) continue;  // every query of the half precedes our keys
        init_c(kb);
        chain1(kb, no_fill);
        if (!DK) {
          const bool tile_mask = causal && q0 < k0 + 31;  // wave-uniform: only diagonal tiles pay the mask
          if (tile_mask) {
            asm volatile("" ::: "memory");
            const int mthr = key - q0 - 4 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float p = fast_exp2(c[kb][r]);
              c[kb][r] = mthr > (r & 3) + 8 * (r >> 2) ? 0.f : p;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) c[kb][r] = fast_exp2(c[kb][r]);
          }
          publish_p(kb);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // P of both pairs visible
    // phase 2: dK role dS = P (dP - delta), dK^T += Q^T dS; dV role dV^T += dO^T P
    const char* op = DK ? qs : gs;
    auto chain2 = [&](int kb, const bf16x8& s0, const bf16x8& s1, auto&& fill) {
      bf16x8 t0 = lds_tr(op, 32 * kb, 0, lane), t1 = lds_tr(op, 32 * kb + 16, 0, lane);
      FA_PRIO(1);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        bf16x8 n0 = t0, n1 = t1;
        if (d < 3) {
          n0 = lds_tr(op, 32 * kb, 32 * d + 32, lane);
          n1 = lds_tr(op, 32 * kb + 16, 32 * d + 32, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        acc[d] = mfma(t0, s0, acc[d]);
        acc[d] = mfma(t1, s1, acc[d]);
        fill(d);
        __builtin_amdgcn_sched_barrier(0);
        t0 = n0;
        t1 = n1;
      }
      FA_PRIO(0);
    };
    auto ds_part = [&](int kb, const ushort8& p0, const ushort8& p1, int j0, int j1) {
#pragma unroll
      for (int j = j0; j < j1; ++j) {
        c[kb][j] = bf2f(p0[j]) * c[kb][j];
        c[kb][8 + j] = bf2f(p1[j]) * c[kb][8 + j];
      }
    };
    if (DK && !(causal && qbase + 31 < k0)) {
      // both halves live: half 1's dS = P (dP - delta) runs in the MFMA gaps of half 0's dK chain
      const ushort8 p00 = __builtin_bit_cast(ushort8, pbuf[lane]), p01 = __builtin_bit_cast(ushort8, pbuf[64 + lane]);
      const ushort8 p10 = __builtin_bit_cast(ushort8, pbuf[128 + lane]), p11 = __builtin_bit_cast(ushort8, pbuf[192 + lane]);
      ds_part(0, p00, p01, 0, 8);
      const bf16x8 a0 = pack8(c[0], 0), a1 = pack8(c[0], 8);
      chain2(0, a0, a1, [&](int d) { ds_part(1, p10, p11, 2 * d, 2 * d + 2); });
      chain2(1, pack8(c[1], 0), pack8(c[1], 8), no_fill);
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int q0 = qbase + 32 * kb;
        if (causal && q0 + 31 < k0) continue;
        if (DK) {
          const ushort8 p0 = __builtin_bit_cast(ushort8, pbuf[(2 * kb) * 64 + lane]);
          const ushort8 p1 = __builtin_bit_cast(ushort8, pbuf[(2 * kb + 1) * 64 + lane]);
          ds_part(kb, p0, p1, 0, 8);
          chain2(kb, pack8(c[kb], 0), pack8(c[kb], 8), no_fill);
        } else {
          chain2(kb, sp[kb][0], sp[kb][1], no_fill);
        }
      }
    }
  }
  if (key < S) {
    if (DK && rcos != nullptr) rope_bwd_rows(acc, rcos, rsin, key, h);  // dK rows: rotary backward
    store_row_t21(out + b * bs + (long)key * ld + (long)hk * HD, acc, DK ? scale : 1.f, h);
  }
}

__global__ __launch_bounds__(256, 2) void fa_bwd_kh_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    const ushort* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Dl,
    ushort* __restrict__ dK, ushort* __restrict__ dV, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale, float scale_log2, int causal, const float* __restrict__ rcos,
    const float* __restrict__ rsin) {
  __shared__ __attribute__((aligned(1024))) char smem[KH_LDS];
  const int nkb = (S + KH_BK - 1) / KH_BK;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = L / nkb, kb_i = L % nkb;  // (batch, kv head)-major, heaviest key block first
  const int b = grp / Hkv, hk = grp % Hkv;
  const int kblk = causal ? kb_i : nkb - 1 - kb_i;
  const int G = Hq / Hkv;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;
  if (threadIdx.x >= 128)
    kh_body<false>(Q, dO, LSE, Dl, Kb, Vb, dV, smem, b, hk, kblk * KH_BK, S, Hq, G, ld, bs, ldo, bso, scale,
                   scale_log2, causal, nullptr, nullptr);
  else
    kh_body<true>(Q, dO, LSE, Dl, Kb, Vb, dK, smem, b, hk, kblk * KH_BK, S, Hq, G, ld, bs, ldo, bso, scale,
                  scale_log2, causal, rcos, rsin);
}

// ------------------------------ fused dK | dV kernel, one wave per SIMD, both roles per wave (kf)
// kh splits each 32-key slice between a dK and a dV wave because one wave cannot hold both
// accumulator sets beside its operands in 256 registers.  Here the dK^T and dV^T accumulators
// (8 x f32x16 = 128 registers) sit in the AGPR half of the 512-entry file, pinned there by
// inline-asm MFMAs ("+a" operands, as in gemm_tn.hip's hb kernel), so ONE wave computes S, P, dP, dS,
// dV^T and dK^T of its 32 keys:
//   * no P exchange through LDS and one barrier per tile (kh: two);
//   * 4 waves cover 128 keys per staged Q|dO tile (kh: 64), so half the LDS-DMA bytes per MFMA;
//   * a 3-slot Q|dO ring with the DMA two tiles ahead, so the next tile's first operands are read
//     before this tile's MFMAs run out (one barrier per tile, at its start in the default variant).
// Per 64-query tile a wave issues 64 MFMAs (32x32x16) in one fixed order -- S|dP chains of query
// half 0 (i = 0-15) and half 1 (16-31), then dV^T|dK^T of half 0 (32-47) and half 1 (48-63) -- with
// each MFMA's LDS operand read three MFMAs ahead and the softmax-gradient VALU of one half spread
// one element per MFMA gap over the next 16 MFMAs (half 0 in 16-31, half 1 in 32-47; the next
// tile's -lse / -delta accumulator init in 48-63).  Every MFMA is inline asm: the S|dP accumulators
// stay in VGPRs ("+v", no v_accvgpr_read before the exponentials), the dV|dK ones in AGPRs.
// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N), fully expanded (a 64-step
// #pragma unroll body exceeds clang's unroll size threshold and stays a runtime loop)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}
// ring slot: Q | dO | lse | delta as in KC_TILE + 512 B where waves 2-3 drop their copy of the lse /
// delta load (every wave issues the same DMA sequence: no branch in the loop body)
constexpr int KF_BK = 128, KF_STAGES = 3, KF_TILE = KC_TILE + 512, KF_LDS = KF_STAGES * KF_TILE;

// s_nop 1: A/B/C may be fresh VALU results (packed P / dS, the -lse init); hipcc pads nothing in
// front of an asm statement (cdna_hip_programming.md 5.7 item 2).  D -> next MFMA as C: 0 states.
template <bool PAD>
__device__ __forceinline__ void mfma_a(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (PAD)
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
template <bool PAD>
__device__ __forceinline__ void mfma_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (PAD)
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// Variant bits (VAR; launch flags bits 6-18 = VAR; measured in profiles/r04_flash/README.md, the
// rejected ones -- operands 6 MFMAs ahead, a per-half mask branch, a sub-major phase 2, per-pair
// bf16 packing -- are kept as profiles/r04_flash/rejected_kf_variants*.patch):
//   bit0  the next tile's lse / delta read from LDS right after the barrier, converted 4-8 gaps later
//   bit1  the causal mask applied to the S' chain's initial C (-inf where key > query) in the nearly
//         idle gaps 48-63 instead of to P in the softmax gaps (exp2(-inf + finite) = 0, dS = 0 * dP')
//   bit2  the 9 DMA pieces of tile it+2 issued one per MFMA gap instead of all in one (a piece costs
//         the issuing wave ~60-185 cycles, MI355X_MICROARCH 'LDS-DMA piece issue cost')
//   bit3  the 2-state VALU -> MFMA pad only in front of the MFMAs whose B / C a recent gap wrote
//   bit5  each workgroup takes the key-block pair (i, nkb-1-i): uniform causal work per workgroup
//   bit6  the barrier and the DMA pieces at the start of the tile, in the gaps of half 0's S|dP
//         chains, which carry no softmax VALU (default: step 48)
//   bit7  s_memtime stamps per tile phase (diagnostic build only, scripts/kf_stamps.py)
//   bit8  V fragments negated once per block, so the dP' chain starts from +delta loaded straight
//         into its C registers (no per-tile negation) and yields -dS; the dK epilogue takes the sign back
//   bit10 (with bit1) the init unmasked, and one scalar branch per tile masks the next tile's initial
//         C when it crosses this wave's diagonal (around VALU only: a branch around the asm MFMAs
//         gives the AGPR accumulators phi copies)
//   bit11 the paired blocks run by one copy of the block code in a loop
//   bit12 the lse row DMA'd from -lse * log2(e), which the dQ kernel writes (L2OUT) into the second
//         half of the delta buffer: the S' chain's initial C loads straight from LDS, no multiply
// bit7 builds sum their stamps over all waves into g_kf_stamp = {barrier + DMA wait, MFMA 0-15,
// 16-31, 32-47, 48-63, wave-tiles, wave-blocks, whole-block cycles} (s_memtime ticks = shader cycles)
// Only the diagnostic build (-DTH_KF_DIAG=1, scripts/build_variant_lib.sh kf_diag, used by
// scripts/kf_stamps.py) has the stamped variants, the accumulators and th_kf_stamps: the production
// libthk.so carries none of them (tests/test_flash_flags.py checks its exports).
#ifdef TH_KF_DIAG
__device__ unsigned long long g_kf_stamp[8];
// one stamp: s_memtime with its own lgkmcnt(0) in the same statement (cdna_hip_programming.md
// 'In-kernel stamps'; read the SHARES of a stamped build, not its length)
__device__ __forceinline__ unsigned long long kf_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void kf_stamp_add(int i, unsigned long long v) { atomicAdd(&g_kf_stamp[i], v); }
#else
__device__ __forceinline__ unsigned long long kf_stamp() { return 0; }
__device__ __forceinline__ void kf_stamp_add(int, unsigned long long) {}
#endif
#define BAR_OF(V) (((V) & 64) ? 0 : 48)
#ifndef TH_KF_M0SPLIT
#define TH_KF_M0SPLIT 1
#endif
#ifndef TH_KF_WAIT2
#define TH_KF_WAIT2 1
#endif

// one 128-key block (keys kblk0 ..) of (batch b, kv head hk)
template <int VAR>
__device__ __forceinline__ void kf_block(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    const ushort* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Dl,
    ushort* __restrict__ dK, ushort* __restrict__ dV, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale, float scale_log2, int causal, const float* __restrict__ rcos,
    const float* __restrict__ rsin, char* smem, int b, int hk, int kblk0) {
  const int G = Hq / Hkv;
  const ushort* Kb = K + b * bs + (long)hk * HD;
  const ushort* Vb = V + b * bs + (long)hk * HD;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k0 = kblk0 + 32 * w;
  const int key = k0 + c32;
  // K (prescaled by softmax_scale * log2 e: S' = Q K'^T - lse2 is a log2-domain score) and V
  // fragments of this wave's 32 keys, for the whole kernel
  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    ushort8 u = key < S ? *reinterpret_cast<const ushort8*>(Kb + (long)key * ld + 16 * s + 8 * h) : ushort8(0);
#pragma unroll
    for (int e = 0; e < 8; ++e) u[e] = f2bf(bf2f(u[e]) * scale_log2);
    kf[s] = as_bf(u);
    ushort8 vv = key < S ? *reinterpret_cast<const ushort8*>(Vb + (long)key * ld + 16 * s + 8 * h) : ushort8(0);
    if constexpr (VAR & 256) vv ^= (ushort)0x8000;  // -V: dP' = delta - dO V^T, see init_c
    vf[s] = as_bf(vv);
  }
  f32x16 ak[4], av[4];  // dK^T, dV^T: 128 head dims (4 x 32 accumulator rows) x 32 keys (lanes)
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    ak[d] = f32x16(0.f);
    av[d] = f32x16(0.f);
  }
  // the zeros materialised in the AGPRs here, with a pad before the first asm MFMA reads them
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    asm volatile("" : "+a"(ak[d]));
    asm volatile("" : "+a"(av[d]));
  }
  asm volatile("s_nop 4" ::);

  const int nqt = S / C_BQ;  // host: S % 64 == 0
  const int qt0 = causal ? kblk0 / C_BQ : 0;
  const int per_head = nqt - qt0;
  const int total = G * per_head;
  // Tile DMA into a ring slot: waves 0-1 stage Q, waves 2-3 dO (8 x 1 KB per wave); wave 0 also
  // the tile's 64 lse, wave 1 its 64 delta (raw; waves 2-3 the same into the spare), issued FIRST, so one vmcnt(9) per wave means "my
  // pieces of the older tile landed" on every wave.  Tile index clamped (branch-free loop body):
  // a DMA past the last tile re-loads it into a slot nobody reads again.
  unsigned rc[8];
  const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem;
  // DMA of one tile in pieces: dma_prep(j, slot) picks the source rows, dma_piece(u) issues piece u
  // (u = 0: the lse / delta row, 1-8: the 1 KB Q or dO pieces)
  const ushort* d_base = Q;
  const float* d_lb = LSE;
  unsigned d_slot0 = 0, d_img = 0;
  int d_qq0 = 0;
  long d_ldx = ld;
  int dh_i = 0, dt_i = 0;  // (head, tile) of the next dma_prep, clamped at the last tile
  auto dma_prep = [&](int j, int slot) {
    (void)j;
    const int h_i = __builtin_amdgcn_readfirstlane(dh_i), t_i = __builtin_amdgcn_readfirstlane(dt_i);
    if (dh_i * per_head + dt_i < total - 1) {
      if (++dt_i == per_head) {
        dt_i = 0;
        ++dh_i;
      }
    }
    const int hq = hk * G + h_i;
    d_qq0 = (qt0 + t_i) * C_BQ;
    const bool isq = w < 2;
    d_base = isq ? Q + b * bs + (long)hq * HD : dO + b * bso + (long)hq * HD;
    d_ldx = isq ? ld : ldo;
    d_slot0 = __builtin_amdgcn_readfirstlane(lds0 + slot * KF_TILE);
    d_lb = ((w & 1) ? Dl : ((VAR & 4096) ? Dl + (long)B * Hq * S : LSE)) + ((long)b * Hq + hq) * S + d_qq0;
    d_img = d_slot0 + (isq ? 0 : C_BQ * 256) + (w & 1) * 8192;
  };
  auto dma_piece = [&](int u) {
    if (u == 0) {
      glds4(d_lb, (unsigned)lane * 4u, d_slot0 + 2 * C_BQ * 256 + w * (C_BQ * 4));
    } else {
      const unsigned r = rc[u - 1];
      const int row = d_qq0 + (int)(r & 255);
      glds16(d_base, (unsigned)(row * d_ldx + (r >> 8) * 8) * 2u, d_img + (u - 1) * 1024);
    }
  };
  // TH_KF_M0SPLIT: a gap's piece in two halves -- M0 before the gap's MFMA, the load after it, so the MFMA
  // is the wait state the M0 write needs (no s_nop per piece; the TN kernel's round-6 cut)
  auto dma_m0 = [&](int u) {
    const unsigned lds = u == 0 ? d_slot0 + 2 * C_BQ * 256 + w * (C_BQ * 4) : d_img + (u - 1) * 1024;
    asm volatile("s_mov_b32 m0, %0" :: "s"(lds) : "m0");
  };
  auto dma_load = [&](int u) {
    if (u == 0) {
      asm volatile("global_load_lds_dword %0, %1" :: "v"((unsigned)lane * 4u), "s"(d_lb) : "memory");
    } else {
      const unsigned r = rc[u - 1];
      const int row = d_qq0 + (int)(r & 255);
      asm volatile("global_load_lds_dwordx4 %0, %1" :: "v"((unsigned)(row * d_ldx + (r >> 8) * 8) * 2u), "s"(d_base)
                   : "memory");
    }
  };
  auto dma_tile = [&](int j, int slot) {
    dma_prep(j, slot);
#pragma unroll
    for (int u = 0; u < 9; ++u) dma_piece(u);
  };
  __builtin_amdgcn_s_waitcnt(0x0F70);  // K/V fragment loads retired (a wait the compiler sees)
  {
    const int wq = w & 1;
#pragma unroll
    for (int u = 0; u < 8; ++u) rc[u] = img_rc(wq * 8192 + u * 1024 + lane * 16);
  }
  dma_tile(0, 0);
  dma_tile(1, 1);
  asm volatile("s_waitcnt vmcnt(9)\n\ts_barrier" ::: "memory");  // tile 0 landed everywhere

  // operand of MFMA i (0-63) of the tile staged at `slot`
  auto opnd = [&](int i, const char* qs) -> bf16x8 {
    const char* gs = qs + C_BQ * 256;
    if (i < 32) {
      const int kb = i >> 4, j = (i & 15) >> 1;
      return lds_row((i & 1) ? gs : qs, 32 * kb + c32, 2 * j + h);
    }
    const int r = (i - 32) & 15, kb = (i - 32) >> 4, d = r >> 2, sub = r & 3;
    return lds_tr(sub < 2 ? gs : qs, 32 * kb + 16 * (sub & 1), 32 * d, lane);
  };
  // -lse2 / -delta of query half kb (accumulator row order) as the S' / dP' chains' initial C
  f32x16 cs[2], cp[2];
  // (VAR bit1) -inf where key > query: mt = key - (first query of the tile) - 4h, or < -64
  auto masked = [&](float x, int mt, int kb, int g, int e) {
    return (VAR & 2) && mt - 32 * kb > e + 8 * g ? -INFINITY : x;
  };
  auto init_c = [&](int kb, const char* qs, int mt) {
    const float* rl = reinterpret_cast<const float*>(qs + 2 * C_BQ * 256) + 32 * kb + 4 * h;
    const float* rd = rl + C_BQ;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4v l = *reinterpret_cast<const float4v*>(rl + 8 * g);
      const float4v dl = *reinterpret_cast<const float4v*>(rd + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // scalar: packed f32 VALU is an anti-lever beside MFMAs
        cs[kb][4 * g + e] = masked((VAR & 4096) ? l[e] : l[e] * -LOG2E, mt, kb, g, e);
        cp[kb][4 * g + e] = (VAR & 256) ? dl[e] : -dl[e];
      }
    }
  };
  float4v lraw[2][4], draw[2][4];
  auto load_c = [&](int kb, const char* qs) {
    const float* rl = reinterpret_cast<const float*>(qs + 2 * C_BQ * 256) + 32 * kb + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      lraw[kb][g] = *reinterpret_cast<const float4v*>(rl + 8 * g);
      draw[kb][g] = *reinterpret_cast<const float4v*>(rl + C_BQ + 8 * g);
      if constexpr (VAR & 256) {  // +delta is the C the -V chain wants: straight from LDS
#pragma unroll
        for (int e = 0; e < 4; ++e) cp[kb][4 * g + e] = draw[kb][g][e];
      }
      if constexpr (VAR & 4096) {  // -lse2 precomputed by the dQ kernel: straight from LDS too
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[kb][4 * g + e] = lraw[kb][g][e];
      }
    }
  };
  auto conv_c = [&](int kb, int g, int mt) {
    if constexpr (VAR & 1024) {  // unmasked here; the fix-up after the conversion masks the rare diagonal tiles
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[kb][4 * g + e] = lraw[kb][g][e] * -LOG2E;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[kb][4 * g + e] = masked(lraw[kb][g][e] * -LOG2E, mt, kb, g, e);
    }
    if constexpr (!(VAR & 256)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) cp[kb][4 * g + e] = -draw[kb][g][e];
    }
  };
  // P = exp2(S') (0 where key > query), dS = P dP', packed to the bf16 B operands of the dV / dK
  // chains: element r of half kb
  bf16x8 pp[2][2], sp[2][2];
  int mthr = 0;
  auto softmax_elem = [&](int kb, int r) {
    const float pv = !(VAR & 2) && mthr - 32 * kb > (r & 3) + 8 * (r >> 2) ? 0.f : fast_exp2(cs[kb][r]);
    const float dsv = pv * cp[kb][r];
    pp[kb][r >> 3][r & 7] = (__bf16)pv;
    sp[kb][r >> 3][r & 7] = (__bf16)dsv;
  };

  // key - first query of tile t - 4h (causal), or a value no row constant exceeds
  // t = tile index within its head (0 .. per_head-1), kept incrementally (no integer division)
  auto mt_of = [&](int t) { return causal ? key - (qt0 + t) * C_BQ - 4 * h : -128; };
  auto diag_of = [&](int t, int kb) { return causal && k0 + 31 > (qt0 + t) * C_BQ + 32 * kb; };
  int tc = 0;
  constexpr bool STAMP = (VAR & 128) != 0;
  unsigned long long st_t0 = 0, st_prev = 0;
  unsigned st_acc[5] = {0, 0, 0, 0, 0};
  unsigned long long st_ts[4] = {0, 0, 0, 0};
  static_assert(!STAMP || BAR_OF(VAR) == 0, "stamps assume the barrier at the tile start");
  if constexpr (STAMP) st_t0 = kf_stamp();
  const char* cur = smem;
  init_c(0, cur, mt_of(0));
  init_c(1, cur, mt_of(0));
  constexpr int PD = 3, NR = 4;  // operand read distance (MFMAs), operand ring (6: neutral, profiles/r04_flash)
  constexpr int BAR = BAR_OF(VAR);  // MFMA step of the per-tile barrier + tile it+2's DMA
  bf16x8 opr[NR];
#pragma unroll
  for (int i = 0; i < PD; ++i) opr[i] = opnd(i, cur);
  for (int it = 0; it < total; ++it) {
    const char* nxt = smem + ((it + 1) % KF_STAGES) * KF_TILE;
    const int tn = tc + 1 == per_head ? 0 : tc + 1;
    mthr = mt_of(tc);  // causal: mask where key > query
    const int mnext = mt_of(tn);
    const bool dn0 = diag_of(tn, 0), dn1 = diag_of(tn, 1);
    static_for<0, 64>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (STAMP && i == 0) st_prev = kf_stamp();
      if constexpr (STAMP && (i == 16 || i == 32 || i == 48)) st_ts[i / 16] = kf_stamp();
      if constexpr (i == BAR) {
        // this wave's DMA of tile it+1 landed, the barrier makes every wave's visible and puts
        // everyone past tile it-1, whose slot (it+2) % 3 takes tile it+2
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if constexpr (STAMP) st_ts[0] = kf_stamp();  // after the barrier
        if constexpr (VAR & 4)
          dma_prep(it + 2, (it + 2) % KF_STAGES);
        else
          dma_tile(it + 2, (it + 2) % KF_STAGES);
      }
      if constexpr ((VAR & 4) && i >= BAR && i < BAR + 9) {
        if constexpr (TH_KF_M0SPLIT) dma_m0(i - BAR);
        else dma_piece(i - BAR);
      }
      constexpr int ni = i + PD;
      const bf16x8 nx = ni < 64 ? opnd(ni, cur) : opnd(ni - 64, nxt);
      __builtin_amdgcn_sched_barrier(0);
      // TH_KF_WAIT2: one lgkmcnt(2) per MFMA pair (a wait the compiler's waitcnt pass sees) instead of one
      // per MFMA: the pair's operands, read 3 and 2 MFMAs ahead, are older than the two newest reads
      if constexpr (TH_KF_WAIT2 && (i & 1) == 0) __builtin_amdgcn_s_waitcnt(0xC27F);
      const bf16x8 a = opr[i % NR];
      constexpr bool pad = !(VAR & 8) || i == 0 || i == 16 || i == 32 || i == 33 || i == 48 || i == 49;
      if constexpr (i < 32) {
        constexpr int kb = i >> 4, j = (i & 15) >> 1;
        if constexpr (i & 1) mfma_v<pad>(cp[kb], a, vf[j]);
        else mfma_v<pad>(cs[kb], a, kf[j]);
      } else {
        constexpr int r = (i - 32) & 15, kb = (i - 32) >> 4, d = r >> 2, sub = r & 3;
        if constexpr (sub < 2) mfma_a<pad>(av[d], a, pp[kb][sub]);
        else mfma_a<pad>(ak[d], a, sp[kb][sub & 1]);
      }
      if constexpr (TH_KF_M0SPLIT && (VAR & 4) && i >= BAR && i < BAR + 9) {
        __builtin_amdgcn_sched_barrier(0);  // the MFMA stays between the M0 write and the load
        dma_load(i - BAR);
      }
      // VALU of the gap
      if constexpr (i == 16 || i == 32) {
        // the S' / dP' chain of the half just finished: its last MFMA's D -> VALU read (8-pass XDL)
        const int kb = (i >> 4) - 1;
        asm volatile("s_nop 7\n\ts_nop 3" : "+v"(cs[kb]), "+v"(cp[kb]));
      }
      if constexpr (i >= 16 && i < 48) softmax_elem((i >> 4) - 1, i & 15);
      if constexpr (VAR & 1) {
        if constexpr (i == 48) load_c(0, nxt);
        if constexpr (i == 50) load_c(1, nxt);
        if constexpr (!(VAR & 4096) && i >= 54 && i < 62) conv_c((i - 54) >> 2, (i - 54) & 3, mnext);
        if constexpr ((VAR & 1024) && i == 63) {
          // one scalar branch per tile, around VALU only (a branch around the asm MFMAs would give
          // the AGPR accumulators phi copies): -inf where key > query, on the tiles that need it
          if (dn0 || dn1) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                cs[kb][r] = masked(cs[kb][r], mnext, kb, r >> 2, r & 3);
          }
        }
      } else {
        if constexpr (i == 48) init_c(0, nxt, mnext);
        if constexpr (i == 52) init_c(1, nxt, mnext);
      }
      __builtin_amdgcn_sched_barrier(0);
      opr[(i + PD) % NR] = nx;
    });
    if constexpr (STAMP) {
      // BAR == 0 layout: tile start, barrier done (ts0), 16, 32, 48, end
      const unsigned long long t = kf_stamp();
      st_acc[4] += (unsigned)(st_ts[0] - st_prev);
      st_acc[1] += (unsigned)(st_ts[1] - st_ts[0]);
      st_acc[2] += (unsigned)(st_ts[2] - st_ts[1]);
      st_acc[3] += (unsigned)(st_ts[3] - st_ts[2]);
      st_acc[0] += (unsigned)(t - st_ts[3]);
    }
    cur = nxt;
    tc = tn;
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      // the order of g_kf_stamp: barrier, 0-15, 16-31, 32-47, 48-63, tiles, blocks, whole block
      const unsigned long long t = kf_stamp();
      kf_stamp_add(0, (unsigned long long)st_acc[4]);
      kf_stamp_add(1, (unsigned long long)st_acc[1]);
      kf_stamp_add(2, (unsigned long long)st_acc[2]);
      kf_stamp_add(3, (unsigned long long)st_acc[3]);
      kf_stamp_add(4, (unsigned long long)st_acc[0]);
      kf_stamp_add(5, (unsigned long long)total);
      kf_stamp_add(6, 1ull);
      kf_stamp_add(7, t - st_t0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    asm volatile("" : "+a"(ak[d]));
    asm volatile("" : "+a"(av[d]));
  }
  if (key < S) {
    if (rcos != nullptr) rope_bwd_rows(ak, rcos, rsin, key, h);  // dK rows: rotary backward
    // (VAR bit8: the chain computed -dS, so dK^T accumulated -dK^T)
    store_row_t21(dK + b * bs + (long)key * ld + (long)hk * HD, ak, (VAR & 256) ? -scale : scale, h);
    store_row_t21(dV + b * bs + (long)key * ld + (long)hk * HD, av, 1.f, h);
  }
}


// VAR bit5: each workgroup takes the key-block pair (i, nkb-1-i) one after the other -- under a
// causal mask every pair carries the same number of tiles, so the grid is one uniform size
// instead of a 32:1 spread whose heavy blocks may start last on a CU
template <int VAR>
__global__ __launch_bounds__(256, 1) void fa_bwd_kf_kernel(
    const ushort* __restrict__ Q, const ushort* __restrict__ K, const ushort* __restrict__ V,
    const ushort* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Dl,
    ushort* __restrict__ dK, ushort* __restrict__ dV, int B, int S, int Hq, int Hkv, long ld,
    long bs, long ldo, long bso, float scale, float scale_log2, int causal, const float* __restrict__ rcos,
    const float* __restrict__ rsin) {
  __shared__ __attribute__((aligned(1024))) char smem[KF_LDS];
  const int nkb = (S + KF_BK - 1) / KF_BK;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if constexpr (VAR & 32) {
    const int np = (nkb + 1) / 2;
    const int grp = L / np, kb_i = L % np;
    const int b = grp / Hkv, hk = grp % Hkv;
    const int kb2 = nkb - 1 - kb_i;
    if constexpr (VAR & 2048) {
      // one copy of the block code, run once or twice (the two inlined copies below double the
      // kernel's instruction footprint)
      const int npass = kb2 != kb_i ? 2 : 1;
#pragma nounroll
      for (int pass = 0; pass < npass; ++pass) {
        if (pass) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        kf_block<VAR>(Q, K, V, dO, LSE, Dl, dK, dV, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale_log2, causal,
                      rcos, rsin, smem, b, hk, (pass ? kb2 : kb_i) * KF_BK);
      }
      return;
    }
    kf_block<VAR>(Q, K, V, dO, LSE, Dl, dK, dV, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale_log2, causal, rcos,
                  rsin, smem, b, hk, kb_i * KF_BK);
    if (kb2 != kb_i) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done with the ring
      kf_block<VAR>(Q, K, V, dO, LSE, Dl, dK, dV, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale_log2, causal,
                    rcos, rsin, smem, b, hk, kb2 * KF_BK);
    }
  } else {
    const int grp = L / nkb, kb_i = L % nkb;  // (batch, kv head)-major, heaviest key block first
    const int b = grp / Hkv, hk = grp % Hkv;
    kf_block<VAR>(Q, K, V, dO, LSE, Dl, dK, dV, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale_log2, causal, rcos,
                  rsin, smem, b, hk, (causal ? kb_i : nkb - 1 - kb_i) * KF_BK);
  }
}

constexpr int B_LDS = 2 * B_BK * 256 + 2 * B_BQ * 256 + 2 * B_BQ * 4;
}  // namespace

static int check_geom(int B, int S, int Hq, int Hkv, int D, long ld, long ldo) {
  if (B <= 0 || S <= 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv != 0 || D != HD) return -1;
  if (ld % 8 != 0 || ldo % 8 != 0) return -1;
  return 0;
}

extern "C" int th_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                                 int B, int S, int Hq, int Hkv, int D, int causal, long ld, long bs,
                                 long ldo, long bso, float scale, int flags, hipStream_t s) {
  if (check_geom(B, S, Hq, Hkv, D, ld, ldo)) return -1;
  const long nblk = (long)((S + F_BM - 1) / F_BM) * Hq * B;
  // flags: 0 = default variant; 16 + v = explicit v (bit0 PRESCALE, bit1 DEFER, bit2 DBUF,
  // bit3 KVMAJOR block order)
  // flags bit5 (with 16 + v): SPREAD on the DMA variants (default: TH_FA_FWD_SPREAD)
  if (flags & 64) {  // ping-pong kernel (diagnostic build): two query heads per workgroup, 32-bit DMA offsets
#ifdef TH_FA_DIAG
    if ((Hq / Hkv) % 2 != 0 || (long)S * ld * 2 >= (1L << 31)) return -3;
    const long npp = (long)((S + F_BM - 1) / F_BM) * (Hq / 2) * B;
    fa_fwd_pp_kernel<<<(unsigned)npp, 512, 0, s>>>((const ushort*)q, (const ushort*)k, (const ushort*)v,
                                                    (ushort*)o, lse, B, S, Hq, Hkv, ld, bs, ldo, bso,
                                                    scale * LOG2E, causal);
    TH_CHECK_LAUNCH();
#else
    return -3;
#endif
  }
  int var = flags >= 16 ? (flags & 15) : TH_FA_FWD_DEFAULT;
  bool spread = flags >= 16 ? ((flags >> 5) & 1) : TH_FA_FWD_SPREAD;
  if ((long)S * ld * 2 >= (1L << 31)) var &= ~4;  // DMA staging uses 32-bit row offsets
#define TH_FWD(P, Dd, Db, Km)                                                                      \
  fa_fwd_kernel<P, Dd, Db, Km><<<(unsigned)nblk, 256, 0, s>>>((const ushort*)q, (const ushort*)k,  \
                                                             (const ushort*)v, (ushort*)o, lse, B,  \
                                                             S, Hq, Hkv, ld, bs, ldo, bso,          \
                                                             scale * LOG2E, causal)
#ifdef TH_FA_DIAG
  // experiment matrix (diagnostic library only: scripts/build_variant_lib.sh fa_diag -DTH_FA_DIAG=1)
  if (var == 15 && spread) {
    fa_fwd_kernel<true, true, true, true, true><<<(unsigned)nblk, 256, 0, s>>>(
        (const ushort*)q, (const ushort*)k, (const ushort*)v, (ushort*)o, lse, B, S, Hq, Hkv, ld, bs, ldo, bso,
        scale * LOG2E, causal);
    TH_CHECK_LAUNCH();
  }
  switch (var) {
    case 0: TH_FWD(false, false, false, false); break;
    case 1: TH_FWD(true, false, false, false); break;
    case 2: TH_FWD(false, true, false, false); break;
    case 3: TH_FWD(true, true, false, false); break;
    case 4: TH_FWD(false, false, true, false); break;
    case 5: TH_FWD(true, false, true, false); break;
    case 6: TH_FWD(false, true, true, false); break;
    case 7: TH_FWD(true, true, true, false); break;
    case 8: TH_FWD(false, false, false, true); break;
    case 11: TH_FWD(true, true, false, true); break;
    case 15: TH_FWD(true, true, true, true); break;
    default: TH_FWD(true, true, true, true); break;
  }
#else
  // production: the default (15: PRESCALE + DEFER + LDS-DMA DBUF + KVMAJOR) and, when the DMA staging's
  // 32-bit row offsets would overflow, the same kernel with register-staged tiles (11)
  if (spread || (var != 15 && var != 11)) return -3;
  if (var == 15) TH_FWD(true, true, true, true);
  else TH_FWD(true, true, false, true);
#endif
#undef TH_FWD
  TH_CHECK_LAUNCH();
}

#ifdef TH_PP_STAMP
extern "C" int th_pp_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(th_pp_stamp_buf), sizeof(th_pp_stamp_buf));
}
#endif

// rcos / rsin (the [S][64] rotary tables, or null): the rotary backward of dQ and dK is applied in the
// dQ and dK|dV kernels' epilogues (default dK|dV kernel only: other flags return -3 with tables given)
// kf variant: flags bits 6-18
static int kf_var_of(int flags) { return (flags >> 6) & 8191; }
static bool kf_variant_known(int v) {
  return v == 7535
#ifdef TH_FA_DIAG
         || v == 0 || v == 111 || v == 3439  // earlier kf variants (profiles/r04_flash)
#endif
#ifdef TH_KF_DIAG
         || v == 3567 || v == 7663  // s_memtime-stamped builds (diagnostic library only)
#endif
      ;
}

// The launch flags the production library serves (ops/attention.py): the default kf path (bit4, kf 7535,
// bit19), the paired kh kernel (bit19; also the automatic fallback for S % 64 != 0), the fused
// register-staged dK|dV kernel with the DMA dQ kernel (bit3 + bit19), and register-staged tiles throughout
// (bit5; also the automatic fallback when 32-bit DMA offsets overflow).  The q-major dQ order, the dQ kernel
// without the spread DMA, the old dK/dV block order / priority bits and the earlier kf variants exist only in
// the diagnostic build (-DTH_FA_DIAG).
static bool flags_shipped(int flags) {
#ifdef TH_FA_DIAG
  (void)flags;
  return true;
#else
  const int known = 8 | 16 | 32 | (8191 << 6) | (1 << 19);
  if (flags & ~known) return false;
  if (flags & 32) return !(flags & 16);
  if (!((flags >> 19) & 1)) return false;
  if (flags & 16) return !(flags & 8) && kf_variant_known(kf_var_of(flags));
  return kf_var_of(flags) == 0;
#endif
}

static int flash_bwd_impl(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq,
                          int Hkv, int D, int causal, long ld, long bs, long ldo, long bso, float scale,
                          const float* rcos, const float* rsin, int flags, hipStream_t s) {
  if (check_geom(B, S, Hq, Hkv, D, ld, ldo)) return -1;
  if (rcos != nullptr && ((flags & (8 | 32)) || (long)S * ld * 2 >= (1L << 31) || rsin == nullptr))
    return -3;
  if ((flags & 16) && !kf_variant_known(kf_var_of(flags))) return -3;  // before any launch
  if (!flags_shipped(flags)) return -3;
  if ((flags & 16) && S % C_BQ != 0) flags &= ~16;  // kf assumes whole 64-query tiles: kh instead
  const long nq = (long)((S + F_BM - 1) / F_BM) * Hq * B;
  // flags bit0: q-major block order for the dQ kernel (default: KV-major, see q_block_map);
  // bit5: register-staged K/V tiles instead of LDS-DMA (also used when 32-bit offsets overflow)
  const bool dq_dma = !(flags & 32) && (long)S * ld * 2 < (1L << 31);
  // bit19: the dQ kernel's tile DMA spread over its first S|dP chain (SPREAD)
  const bool dq_spread = (flags >> 19) & 1;
  // kf VAR bit12 reads -lse2 from the dQ kernel (L2OUT) in the second half of the delta buffer
  const bool dq_l2 = (flags & 16) && !(flags & 8) && dq_dma && (kf_var_of(flags) & 4096);
  if (dq_l2 && !(dq_spread && !(flags & 1))) return -3;  // instantiated for the default order + spread only
  if (dq_l2) {
    fa_bwd_dq_kernel<true, true, true, true><<<(unsigned)nq, 256, 0, s>>>(
        (const ushort*)q, (const ushort*)k, (const ushort*)v, (const ushort*)dout, (const ushort*)o, lse, delta,
        (ushort*)dq, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale * LOG2E, causal, rcos, rsin);
  } else {
#define TH_DQ_LAUNCH(KVM, DMA_, SP_)                                                                         \
  fa_bwd_dq_kernel<KVM, DMA_, SP_><<<(unsigned)nq, 256, 0, s>>>((const ushort*)q, (const ushort*)k, (const ushort*)v, \
                                                               (const ushort*)dout, (const ushort*)o, lse, delta,     \
                                                               (ushort*)dq, B, S, Hq, Hkv, ld, bs, ldo, bso, scale,   \
                                                               scale * LOG2E, causal, rcos, rsin)
#ifdef TH_FA_DIAG
  if (flags & 1) {
    if (dq_dma) {
      if (dq_spread) TH_DQ_LAUNCH(false, true, true); else TH_DQ_LAUNCH(false, true, false);
    } else {
      TH_DQ_LAUNCH(false, false, false);
    }
  } else {
    if (dq_dma) {
      if (dq_spread) TH_DQ_LAUNCH(true, true, true); else TH_DQ_LAUNCH(true, true, false);
    } else {
      TH_DQ_LAUNCH(true, false, false);
    }
  }
#else
  if (dq_dma) TH_DQ_LAUNCH(true, true, true);  // flags_shipped: bit19 is set on every DMA path
  else TH_DQ_LAUNCH(true, false, false);
#endif
#undef TH_DQ_LAUNCH
  }
  // bit4 (ops/attention.py's default, with a kf variant in bits 6-12): the one-wave-per-SIMD kf
  // kernel (profiles/r04_flash); flags 0: the half-width paired dK|dV kernel kh (two workgroups per
  // CU, profiles/r03_flash); bit3, bit5 or 32-bit LDS-DMA offsets that overflow: the fused
  // register-staged dK/dV kernel below
  if ((flags & 16) && !(flags & 8) && dq_dma) {  // bit4: the fused one-wave-per-SIMD kernel (kf)
    const int kvar = kf_var_of(flags);
    const int nkb_f = (S + KF_BK - 1) / KF_BK;
    const long nkf = (long)((kvar & 32) ? (nkb_f + 1) / 2 : nkb_f) * Hkv * B;
#define TH_KF_LAUNCH(V_)                                                                                      \
  fa_bwd_kf_kernel<V_><<<(unsigned)nkf, 256, 0, s>>>((const ushort*)q, (const ushort*)k, (const ushort*)v,        \
                                                     (const ushort*)dout, lse, delta, (ushort*)dk, (ushort*)dv,   \
                                                     B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale * LOG2E, causal, \
                                                     rcos, rsin)
    // the instantiated variants (profiles/r04_flash/README.md has the measured ones; others are
    // rejected up front by kf_variant_known)
    switch (kvar) {
#ifdef TH_FA_DIAG
      case 0: TH_KF_LAUNCH(0); break;
      case 111: TH_KF_LAUNCH(111); break;    // bits 0-3, 5, 6
      case 3439: TH_KF_LAUNCH(3439); break;  // 111 + bits 8, 10, 11
#endif
      case 7535: TH_KF_LAUNCH(7535); break;  // 3439 + -lse2 from the dQ kernel (bit12; the default, attention.py)
#ifdef TH_KF_DIAG
      case 3567: TH_KF_LAUNCH(3567); break;  // 3439 + s_memtime stamps (th_kf_stamps)
      case 7663: TH_KF_LAUNCH(7663); break;  // 7535 + stamps
#endif
      default: return -3;                    // unreachable: kf_variant_known
    }
#undef TH_KF_LAUNCH
    TH_CHECK_LAUNCH();
  }
  if (!(flags & 8) && dq_dma) {
    const long nkh = (long)((S + KH_BK - 1) / KH_BK) * Hkv * B;
    fa_bwd_kh_kernel<<<(unsigned)nkh, 256, 0, s>>>((const ushort*)q, (const ushort*)k, (const ushort*)v,
                                                   (const ushort*)dout, lse, delta, (ushort*)dk, (ushort*)dv,
                                                   B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale * LOG2E, causal,
                                                   rcos, rsin);
    TH_CHECK_LAUNCH();
  }
  const long nk = (long)((S + B_BK - 1) / B_BK) * Hkv * B;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkv_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, B_LDS);
#ifdef TH_FA_DIAG
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkv_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, B_LDS);
#endif
    attr_set = true;
  }
#ifdef TH_FA_DIAG
  // flags bit1: the old (kv-block-major) order for dK/dV (default: KV-head-major)
  if (flags & 2)
    fa_bwd_dkv_kernel<false><<<(unsigned)nk, B_THREADS, B_LDS, s>>>(
        (const ushort*)q, (const ushort*)k, (const ushort*)v, (const ushort*)dout, lse, delta, (ushort*)dk,
        (ushort*)dv, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale * LOG2E, causal, !(flags & 4));
  else
#endif
    fa_bwd_dkv_kernel<true><<<(unsigned)nk, B_THREADS, B_LDS, s>>>(
        (const ushort*)q, (const ushort*)k, (const ushort*)v, (const ushort*)dout, lse, delta, (ushort*)dk,
        (ushort*)dv, B, S, Hq, Hkv, ld, bs, ldo, bso, scale, scale * LOG2E, causal, !(flags & 4));
  TH_CHECK_LAUNCH();
}

#ifdef TH_KF_DIAG
// kf stamp accumulators (VAR bit7 builds): reset = 1 zeroes them, else copies the 8 sums to out
extern "C" int th_kf_stamps(unsigned long long* out, int reset) {
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_kf_stamp), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kf_stamp), 8 * sizeof(unsigned long long));
}
#endif

extern "C" int th_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                 const void* dout, const float* lse, float* delta, float* dq_acc,
                                 void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv, int D,
                                 int causal, long ld, long bs, long ldo, long bso, float scale,
                                 int flags, hipStream_t s) {
  (void)dq_acc;
  return flash_bwd_impl(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, D, causal, ld, bs, ldo, bso,
                        scale, nullptr, nullptr, flags, s);
}

// The same backward with the rotary backward of dQ / dK folded into the kernels (ops/attention.py)
extern "C" int th_flash_attn_bwd_rope(const void* q, const void* k, const void* v, const void* o,
                                      const void* dout, const float* lse, float* delta, void* dq, void* dk,
                                      void* dv, int B, int S, int Hq, int Hkv, int D, int causal, long ld,
                                      long bs, long ldo, long bso, float scale, const float* rcos,
                                      const float* rsin, int flags, hipStream_t s) {
  return flash_bwd_impl(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, D, causal, ld, bs, ldo, bso,
                        scale, rcos, rsin, flags, s);
}
