// Microbenchmark: what one MFMA gap costs at one wave per SIMD (the kf / NT-GEMM regime).
//
// Every variant runs the same 64-MFMA step loop as kf's tile body (v_mfma_f32_32x32x16_bf16 through
// inline asm, the operand of MFMA i+3 read from LDS in the gap of MFMA i) with more of kf's gap
// content switched on per variant, and reports shader cycles per MFMA (s_memtime around the loop,
// median wave).  Build and run:
//   hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize scripts/mfma_gap_bench.hip -o scripts/mfma_gap_bench
//   ./scripts/mfma_gap_bench            # one JSON line per variant
//
// Variants (bits): 1 = ds_read_b128 operand per MFMA, 2 = two ds_read_b64_tr_b16 instead, 4 = the
// accumulators in VGPRs ("+v", kf's S|dP chains) instead of AGPRs, 8 = one softmax element per gap
// (v_exp + v_mul + packing), 16 = `s_nop 1` in front of every MFMA, 32 = two independent
// accumulators alternating (kf's S|dP pattern) instead of the kf phase-2 pattern (4 accumulators,
// pairs of dependent MFMAs), 64 = kf's softmax element per gap (independent exp2 / mul / bf16
// conversions into operands the MFMAs of this phase do not read; bit 8 instead chains each element's
// result into the next MFMA's B operand and into the next element), 128 = 9 LDS-DMA pieces
// (global_load_lds_dwordx4, 1 KB each, L2-resident source) in gaps 0-8, 256 = a vmcnt(0) + s_barrier
// at MFMA 0 of every 64 (kf's per-tile synchronisation).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
#define LDS_AS __attribute__((address_space(3)))

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <bool V, bool PAD>
__device__ __forceinline__ void mfma(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (V) {
    if constexpr (PAD)
      asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    else
      asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  } else {
    if constexpr (PAD)
      asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
    else
      asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  }
}

__device__ __forceinline__ void glds16(const void* sbase, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(lds), "v"(voff), "s"(sbase) : "memory", "m0");
}

template <int VAR>
__global__ __launch_bounds__(256, 1) void gap_kernel(const bf16x8* __restrict__ src, float* __restrict__ out,
                                                     unsigned long long* __restrict__ cyc, int iters,
                                                     const char* __restrict__ gsrc) {
  __shared__ __attribute__((aligned(1024))) char smem[65536];
  constexpr bool RD = VAR & 3, TR = VAR & 2, VACC = VAR & 4, SM = VAR & 8, PAD = VAR & 16, ALT = VAR & 32;
  constexpr bool BAR = VAR & 256, DMA = VAR & 128;  // per-tile barrier (kf: at MFMA 0); + 9 LDS-DMA pieces in gaps 0-8
  constexpr bool SMI = VAR & 64;  // kf-like softmax: independent elements, packed outputs not read by the MFMAs
  const int tid = threadIdx.x, lane = tid & 63;
  // fill LDS with finite bf16 data
  for (int i = tid; i < 65536 / 16; i += 256) reinterpret_cast<bf16x8*>(smem)[i] = src[i & 1023];
  __syncthreads();
  bf16x8 bop[4];
  for (int j = 0; j < 4; ++j) bop[j] = src[(lane + 64 * j) & 1023];
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = f32x16(0.f);
  if constexpr (!VACC) {
    for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[j]));
    asm volatile("s_nop 4" ::);
  }
  f32x16 sm = f32x16(0.1f);
  bf16x8 packed = bop[0];
  f32x16 xs[2], ys[2];  // kf's S' / dP' accumulators of the two query halves as the softmax inputs
  for (int k = 0; k < 2; ++k)
    for (int e = 0; e < 16; ++e) {
      xs[k][e] = -0.01f * (float)(e + (lane & 7) + k);
      ys[k][e] = 0.5f + 0.01f * (float)e;
    }
  bf16x8 po[2][2], dso[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) po[a][b] = dso[a][b] = bop[0];
  // kf-like addresses: 16-B row reads with an XOR swizzle; transposed reads 8 B
  const int wv = tid >> 6;
  const char* base = smem + wv * 16384;
  auto rd = [&](int i) -> bf16x8 {
    if constexpr (TR) {
      const char* p0 = base + ((i * 1024 + lane * 8) & 16383);
      const char* p1 = base + ((i * 1024 + 512 + lane * 8) & 16383);
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(p0));
      const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(p1));
      const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    } else {
      return *reinterpret_cast<const bf16x8*>(base + ((i * 1024 + ((lane ^ (i & 7)) * 16)) & 16383));
    }
  };
  bf16x8 opr[4];
  for (int i = 0; i < 3; ++i) opr[i] = RD ? rd(i) : bop[i];
  __syncthreads();
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
    if constexpr (SMI) {  // loop-carried (one op per element, as kf's -lse init), so nothing is hoisted
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) xs[k][e] = xs[k][e] * 0.999f;
    }
    static_for<0, 64>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (BAR && i == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (DMA && i < 9) {
        const unsigned lds0 = (unsigned)(uintptr_t)(char LDS_AS*)smem;
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + 32768 + wv * 8192 + (i & 7) * 1024);
        const unsigned chunk = (unsigned)(((it * 9 + i) * 4 + wv) & 4095);  // 4 MB of L2-resident source
        glds16(gsrc, chunk * 1024u + (unsigned)lane * 16u, dst);
      }
      bf16x8 nx = bop[(i + 3) & 3];
      if constexpr (RD) nx = rd((i + 3) & 63);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 a = opr[i & 3];
      if constexpr (ALT)
        mfma<VACC, PAD>(acc[i & 1], a, bop[(i >> 1) & 3]);
      else
        mfma<VACC, PAD>(acc[(i >> 1) & 3], a, packed);
      if constexpr (SMI && i >= 16 && i < 48) {  // kf: half 0's elements in gaps 16-31, half 1's in 32-47
        constexpr int r = (i - 16) & 15, h2 = (i - 16) >> 4;
        const float pv = __builtin_amdgcn_exp2f(xs[h2][r]);
        const float ds = pv * ys[h2][r];
        po[h2][r >> 3][r & 7] = (__bf16)pv;
        dso[h2][r >> 3][r & 7] = (__bf16)ds;
      }
      if constexpr (SM) {
        const int r = i & 15;
        const float pv = __builtin_amdgcn_exp2f(sm[r]);
        const float ds = pv * sm[(r + 1) & 15];
        packed[r & 7] = (__bf16)pv;
        packed[(r + 1) & 7] = (__bf16)ds;
        sm[r] = ds * 0.5f;
      }
      __builtin_amdgcn_sched_barrier(0);
      opr[(i + 3) & 3] = nx;
    });
  }
  unsigned long long t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  asm volatile("s_nop 15\n\ts_nop 15" ::);
  float s = 0.f;
  for (int j = 0; j < 4; ++j) {
    if constexpr (!VACC) asm volatile("" : "+a"(acc[j]));
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  }
  for (int e = 0; e < 16; ++e) s += sm[e];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 8; ++e) s += (float)po[a][b][e] + (float)dso[a][b][e];
  out[blockIdx.x * 256 + tid] = s;  // keep everything live
  if (lane == 0) cyc[blockIdx.x * 4 + wv] = t1 - t0;
}

template <int VAR>
static void run(const bf16x8* src, float* out, unsigned long long* cyc, int nblk, int iters, const char* g) {
  gap_kernel<VAR><<<nblk, 256>>>(src, out, cyc, 2, g);  // warm
  gap_kernel<VAR><<<nblk, 256>>>(src, out, cyc, iters, g);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("{\"variant\": %d, \"error\": \"launch\"}\n", VAR);
    return;
  }
  std::vector<unsigned long long> h(nblk * 4);
  (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double med = (double)h[h.size() / 2];
  std::printf("{\"variant\": %d, \"rd\": %d, \"tr\": %d, \"vacc\": %d, \"softmax\": %d, \"pad\": %d, \"alt\": %d, "
              "\"softmax_kf\": %d, \"dma\": %d, \"barrier\": %d, \"cycles_per_mfma\": %.2f}\n",
              VAR, (VAR & 3) ? 1 : 0, (VAR & 2) ? 1 : 0, (VAR & 4) ? 1 : 0, (VAR & 8) ? 1 : 0, (VAR & 16) ? 1 : 0,
              (VAR & 32) ? 1 : 0, (VAR & 64) ? 1 : 0, (VAR & 128) ? 1 : 0, (VAR & 256) ? 1 : 0,
              med / (64.0 * iters));
  std::fflush(stdout);
}

int main() {
  const int nblk = 256, iters = 2000;
  bf16x8* src;
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&src, 1024 * sizeof(bf16x8));
  (void)hipMalloc(&out, nblk * 256 * sizeof(float));
  (void)hipMalloc(&cyc, nblk * 4 * sizeof(unsigned long long));
  std::vector<unsigned short> hs(1024 * 8);
  for (size_t i = 0; i < hs.size(); ++i) hs[i] = 0x3c00 + (unsigned short)(i % 64);  // ~1.0 .. 1.5 in bf16
  (void)hipMemcpy(src, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
  char* g;
  (void)hipMalloc(&g, 4 << 20);
  (void)hipMemset(g, 0, 4 << 20);
  run<0>(src, out, cyc, nblk, iters, g);               // bare asm MFMAs, AGPR accumulators
  run<1>(src, out, cyc, nblk, iters, g);               // + ds_read_b128 operand per MFMA
  run<2>(src, out, cyc, nblk, iters, g);               // + 2 ds_read_b64_tr_b16 instead
  run<1 | 16>(src, out, cyc, nblk, iters, g);          // + s_nop 1 per MFMA
  run<1 | 4 | 32>(src, out, cyc, nblk, iters, g);      // VGPR accumulators, 2 alternating (kf S|dP)
  run<1 | 8>(src, out, cyc, nblk, iters, g);           // + softmax chained into the next MFMA
  run<1 | 64>(src, out, cyc, nblk, iters, g);          // kf-like softmax (independent elements)
  run<2 | 64>(src, out, cyc, nblk, iters, g);          // + tr reads
  run<1 | 64 | 256>(src, out, cyc, nblk, iters, g);    // + one barrier per 64 MFMAs
  run<1 | 64 | 256 | 128>(src, out, cyc, nblk, iters, g);  // + 9 LDS-DMA pieces per 64 MFMAs (kf)
  run<1 | 256 | 128>(src, out, cyc, nblk, iters, g);   // barrier + DMA without softmax
  (void)hipFree(g);
  (void)hipFree(src);
  (void)hipFree(out);
  (void)hipFree(cyc);
  return 0;
}
