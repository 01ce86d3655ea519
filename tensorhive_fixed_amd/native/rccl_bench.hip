// rccl-bench: RCCL-over-xGMI collective microbenchmark for MI355X nodes.
//
// One process drives every visible GPU (ncclCommInitAll) so it runs without a launcher:
//   rccl-bench [--gpus N] [--min BYTES] [--max BYTES] [--iters K] [--op allreduce|reducescatter|allgather|all]
//              [--direct] | --check-virtual-peers P [--min BYTES]
// For each bf16 message size it reports algorithm bandwidth (bytes/time) and bus bandwidth
// (allreduce: 2(n-1)/n x algbw; reduce-scatter / all-gather: (n-1)/n x algbw) as JSON lines.
// `--direct` adds a one-shot peer-to-peer all-reduce HIP kernel for comparison: every GPU reads
// its slice from all peers over its 7 xGMI links at once (hipDeviceEnablePeerAccess), sums in
// f32 and writes the slice back to every peer -- the shape a ring cannot use, since a ring is
// bound to one link per hop.  These numbers pick the DDP gradient bucket size of the payload.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)
#define NK(x)                                                                               \
  do {                                                                                      \
    ncclResult_t r_ = (x);                                                                  \
    if (r_ != ncclSuccess) {                                                                \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

typedef unsigned short u16;

__device__ __forceinline__ float b2f(u16 u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ u16 f2b(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

// one-shot all-reduce of slice [lo, hi) of n elements: sum over all peers' buffers, write to all
__global__ void direct_allreduce(u16** bufs, int npeers, long lo, long hi) {
  for (long i = lo + blockIdx.x * (long)blockDim.x + threadIdx.x; i < hi; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < npeers; ++p) s += b2f(bufs[p][i]);
    const u16 v = f2b(s);
    for (int p = 0; p < npeers; ++p) bufs[p][i] = v;
  }
}

// Correctness check of direct_allreduce without N GPUs: `vpeers` buffers on ONE device stand in
// for the peers (the kernel only sees an array of peer pointers, so the indexing, slicing and
// f32 accumulation are exactly what runs across xGMI).  Every slice is reduced by its own launch,
// as each GPU would; the result must equal the host's f32 sum rounded to bf16, bit for bit, in
// every peer buffer.  Prints one JSON line; exit code 0 iff it matches.
static u16 h_f2b(float f) {  // round-to-nearest-even, as (__bf16)f
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (u16)(u >> 16);
}
static float h_b2f(u16 b) {
  unsigned u = (unsigned)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static int check_direct(int vpeers, long count) {
  CK(hipSetDevice(0));
  std::vector<u16*> bufs(vpeers);
  std::vector<std::vector<u16>> host(vpeers, std::vector<u16>(count));
  for (int p = 0; p < vpeers; ++p) {
    for (long i = 0; i < count; ++i)  // distinct, exactly representable-ish values per peer and index
      host[p][i] = h_f2b(0.001f * (float)((i * 7 + p * 13) % 1024) - 0.37f * (float)(p + 1));
    CK(hipMalloc((void**)&bufs[p], count * sizeof(u16)));
    CK(hipMemcpy(bufs[p], host[p].data(), count * sizeof(u16), hipMemcpyHostToDevice));
  }
  u16** dptrs = nullptr;
  CK(hipMalloc((void**)&dptrs, sizeof(u16*) * vpeers));
  CK(hipMemcpy(dptrs, bufs.data(), sizeof(u16*) * vpeers, hipMemcpyHostToDevice));
  const long slice = (count + vpeers - 1) / vpeers;
  for (int r = 0; r < vpeers; ++r) {
    const long lo = r * slice, hi = lo + slice < count ? lo + slice : count;
    if (lo < hi) direct_allreduce<<<256, 256>>>(dptrs, vpeers, lo, hi);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  long bad = 0;
  double max_err = 0.0;
  std::vector<u16> got(count);
  for (int p = 0; p < vpeers; ++p) {
    CK(hipMemcpy(got.data(), bufs[p], count * sizeof(u16), hipMemcpyDeviceToHost));
    for (long i = 0; i < count; ++i) {
      float s = 0.f;
      for (int q = 0; q < vpeers; ++q) s += h_b2f(host[q][i]);
      const u16 want = h_f2b(s);
      if (got[i] != want) {
        ++bad;
        const double e = fabs((double)h_b2f(got[i]) - (double)h_b2f(want));
        max_err = e > max_err ? e : max_err;
      }
    }
  }
  printf("{\"check\":\"direct_allreduce\",\"virtual_peers\":%d,\"elements\":%ld,\"mismatches\":%ld,"
         "\"max_abs_err\":%g,\"ok\":%s}\n", vpeers, count, bad, max_err, bad == 0 ? "true" : "false");
  fflush(stdout);
  for (int p = 0; p < vpeers; ++p) CK(hipFree(bufs[p]));
  CK(hipFree(dptrs));
  return bad == 0 ? 0 : 3;
}

int main(int argc, char** argv) {
  int ngpu = 0, iters = 20;
  int vpeers = 0;
  long mn = 8l << 20, mx = 1l << 30;
  std::string op = "all";
  bool direct = false;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--gpus") && i + 1 < argc) ngpu = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--min") && i + 1 < argc) mn = atol(argv[++i]);
    else if (!strcmp(argv[i], "--max") && i + 1 < argc) mx = atol(argv[++i]);
    else if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--op") && i + 1 < argc) op = argv[++i];
    else if (!strcmp(argv[i], "--direct")) direct = true;
    else if (!strcmp(argv[i], "--check-virtual-peers") && i + 1 < argc) vpeers = atoi(argv[++i]);
  }
  if (vpeers > 0) return check_direct(vpeers, (mn / 2) + 37);  // odd length: ragged last slice
  int avail = 0;
  CK(hipGetDeviceCount(&avail));
  if (ngpu <= 0 || ngpu > avail) ngpu = avail;
  if (ngpu < 1) {
    fprintf(stderr, "no GPUs\n");
    return 1;
  }
  std::vector<int> devs(ngpu);
  for (int i = 0; i < ngpu; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(ngpu);
  NK(ncclCommInitAll(comms.data(), ngpu, devs.data()));
  std::vector<hipStream_t> st(ngpu);
  std::vector<u16*> sbuf(ngpu), rbuf(ngpu);
  for (int i = 0; i < ngpu; ++i) {
    CK(hipSetDevice(i));
    CK(hipStreamCreate(&st[i]));
    CK(hipMalloc((void**)&sbuf[i], mx));
    CK(hipMalloc((void**)&rbuf[i], mx));
    CK(hipMemset(sbuf[i], 0, mx));
  }
  const char* ops[] = {"allreduce", "reducescatter", "allgather"};
  for (long bytes = mn; bytes <= mx; bytes *= 2) {
    const size_t count = bytes / 2;
    for (const char* o : ops) {
      if (op != "all" && op != o) continue;
      auto run = [&]() {
        NK(ncclGroupStart());
        for (int i = 0; i < ngpu; ++i) {
          if (!strcmp(o, "allreduce"))
            NK(ncclAllReduce(sbuf[i], rbuf[i], count, ncclBfloat16, ncclSum, comms[i], st[i]));
          else if (!strcmp(o, "reducescatter"))
            NK(ncclReduceScatter(sbuf[i], rbuf[i], count / ngpu, ncclBfloat16, ncclSum, comms[i], st[i]));
          else
            NK(ncclAllGather(sbuf[i], rbuf[i], count / ngpu, ncclBfloat16, comms[i], st[i]));
        }
        NK(ncclGroupEnd());
      };
      run();
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        CK(hipStreamSynchronize(st[i]));
      }
      auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < iters; ++k) run();
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        CK(hipStreamSynchronize(st[i]));
      }
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
      const double alg = bytes / sec / 1e9;
      const double factor = !strcmp(o, "allreduce") ? 2.0 * (ngpu - 1) / ngpu : (double)(ngpu - 1) / ngpu;
      printf("{\"op\":\"%s\",\"gpus\":%d,\"bytes\":%ld,\"time_us\":%.1f,\"algbw_GBps\":%.2f,\"busbw_GBps\":%.2f}\n",
             o, ngpu, bytes, sec * 1e6, alg, alg * factor);
      fflush(stdout);
    }
    if (direct && ngpu > 1) {
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        for (int j = 0; j < ngpu; ++j)
          if (i != j) {
            hipError_t e = hipDeviceEnablePeerAccess(j, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) CK(e);
          }
      }
      std::vector<u16**> dptrs(ngpu);
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        CK(hipMalloc((void**)&dptrs[i], sizeof(u16*) * ngpu));
        CK(hipMemcpy(dptrs[i], sbuf.data(), sizeof(u16*) * ngpu, hipMemcpyHostToDevice));
      }
      const long slice = (long)count / ngpu;
      auto run = [&]() {
        for (int i = 0; i < ngpu; ++i) {
          CK(hipSetDevice(i));
          direct_allreduce<<<1024, 256, 0, st[i]>>>(dptrs[i], ngpu, i * slice, (i + 1) * slice);
        }
        for (int i = 0; i < ngpu; ++i) {
          CK(hipSetDevice(i));
          CK(hipStreamSynchronize(st[i]));
        }
      };
      run();
      auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < iters; ++k) run();
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
      const double alg = bytes / sec / 1e9;
      printf("{\"op\":\"direct_allreduce\",\"gpus\":%d,\"bytes\":%ld,\"time_us\":%.1f,\"algbw_GBps\":%.2f,"
             "\"busbw_GBps\":%.2f}\n", ngpu, bytes, sec * 1e6, alg, alg * 2.0 * (ngpu - 1) / ngpu);
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        CK(hipFree(dptrs[i]));
      }
    }
  }
  for (int i = 0; i < ngpu; ++i) ncclCommDestroy(comms[i]);
  return 0;
}
