// Microbenchmark: what a single-pass flash backward's dQ sum would cost on MI355X (verdict r04 item 2).
//
// A single-pass backward (S, dP, dV, dK and dQ in ONE kernel, one workgroup per key block) must sum each
// query row's dQ over every key block at or before it (causal).  This replays exactly those adds for the
// training shape -- B 8, S 4096, 32 query / 8 kv heads, d 128 -- without any of the MFMA work: workgroup =
// (batch, kv head, key block), 4 waves; for each of the G = 4 query heads of the kv head and each 64-row
// query tile at or after the key block, the workgroup adds a 64 x 128 f32 tile into dQ (wave w: rows
// 16w..16w+15, each row two 256-B wave instructions).  Modes:
//   0  global_atomic_add_f32 (no return) -- the atomic form
//   1  plain 16-B stores of the same bytes -- the floor of an ordered hand-off's writes (its reads not counted)
// for key blocks of 128 (kf's block) and 256 keys.  Prints one JSON line per (mode, block) with the bytes,
// the time and the rate; mode 0 checks every 4096th element against its contribution count.
//   hipcc -O3 --offload-arch=gfx950 scripts/dq_atomic_bench.hip -o scripts/dq_atomic_bench && ./scripts/dq_atomic_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int B = 8, S = 4096, HQ = 32, HKV = 8, G = HQ / HKV, D = 128, BQ = 64;

template <int MODE, int BK>
__global__ __launch_bounds__(256) void dq_sum(float* __restrict__ dq) {
  const int nkb = S / BK;
  const int wg = blockIdx.x;
  const int kb = wg % nkb, hk = (wg / nkb) % HKV, b = wg / (nkb * HKV);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t0 = kb * BK / BQ;
  for (int g = 0; g < G; ++g) {
    const int hq = hk * G + g;
    for (int t = t0; t < S / BQ; ++t) {
#pragma unroll 4
      for (int r = 0; r < 16; ++r) {
        const long row = (long)b * S + t * BQ + 16 * w + r;
        float* p = dq + row * (HQ * D) + hq * D;
        if constexpr (MODE == 0) {
          __builtin_amdgcn_global_atomic_fadd_f32(p + lane, 1.0f);
          __builtin_amdgcn_global_atomic_fadd_f32(p + 64 + lane, 1.0f);
        } else {
          if (lane < 32) reinterpret_cast<float4*>(p)[lane] = make_float4(1.f, 1.f, 1.f, 1.f);
        }
      }
    }
  }
}

template <int MODE, int BK>
void run(float* dq, size_t n) {
  const int grid = B * HKV * (S / BK);
  double adds = 0;  // f32 elements added
  for (int kb = 0; kb < S / BK; ++kb) adds += (double)B * HKV * G * (S / BQ - kb * BK / BQ) * BQ * D;
  hipMemset(dq, 0, n * 4);
  dq_sum<MODE, BK><<<grid, 256>>>(dq);  // warm
  hipDeviceSynchronize();
  hipMemset(dq, 0, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 3;
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) dq_sum<MODE, BK><<<grid, 256>>>(dq);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  long bad = -1;
  if (MODE == 0) {
    std::vector<float> h(n);
    hipMemcpy(h.data(), dq, n * 4, hipMemcpyDeviceToHost);
    bad = 0;
    for (size_t i = 0; i < n; i += 4096) {
      const long row = (long)(i / (HQ * D)) % S;
      const float want = (float)reps * (float)(row / BK + 1);  // key blocks at or before this query
      if (h[i] != want) ++bad;
    }
  }
  printf("{\"mode\": \"%s\", \"key_block\": %d, \"workgroups\": %d, \"bytes_GB\": %.3f, \"ms\": %.3f, "
         "\"TB_per_s\": %.3f, \"check_mismatches\": %ld}\n",
         MODE == 0 ? "atomic_add_f32" : "plain_store", BK, grid, adds * 4 / 1e9, ms, adds * 4 / (ms * 1e-3) / 1e12, bad);
}

int main() {
  const size_t n = (size_t)B * S * HQ * D;
  float* dq = nullptr;
  if (hipMalloc(&dq, n * 4) != hipSuccess) return 1;
  run<0, 128>(dq, n);
  run<0, 256>(dq, n);
  run<1, 128>(dq, n);
  run<1, 256>(dq, n);
  hipFree(dq);
  return 0;
}
