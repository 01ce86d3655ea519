// rccl-bench: RCCL-over-xGMI collective microbenchmark for MI355X nodes.
//
// Two modes:
//   * single process (default): one process drives every visible GPU (ncclCommInitAll), runs
//     without a launcher;
//   * --per-rank: one process per GPU, as the training job runs -- started by torchrun
//     (`TH_RCCL_PER_RANK=1 torchrun --no-python --nproc-per-node N rccl-bench`), RANK / WORLD_SIZE
//     / LOCAL_RANK from the environment, ncclCommInitRank with a unique id that rank 0 publishes
//     in a file (no MPI); every rank times its own loop and the MAX over ranks is reported.  Under
//     torchrun the options travel as TH_RCCL_MIN / _MAX / _ITERS / _OP (torchrun's own parser
//     would take --min / --max for abbreviations of its options).
//   rccl-bench [--per-rank] [--gpus N] [--min BYTES] [--max BYTES] [--iters K]
//              [--op allreduce|reducescatter|allgather|all] [--direct] | --check-virtual-peers P [--min BYTES]
// Output (JSON lines; schema pinned by core/rccl_bench.py and tests/test_rccl_bench.py): one
// header {"rccl_bench":1,"mode","world","rccl_version","env":{NCCL_*..}} then, per bf16 message size
// and op, {"op","mode","gpus","bytes","time_us","algbw_GBps","busbw_GBps"} with bus bandwidth
// = 2(n-1)/n x algbw (all-reduce) or (n-1)/n x algbw (reduce-scatter / all-gather).
// `--direct` (single-process mode) adds a one-shot peer-to-peer all-reduce HIP kernel for
// comparison: every GPU reads its slice from all peers over its 7 xGMI links at once
// (hipDeviceEnablePeerAccess) with 16-byte loads, sums in f32 and writes the slice back to every
// peer with 16-byte stores -- the shape a ring cannot use, since a ring is bound to one link per
// hop.  These numbers pick the DDP gradient bucket size of the payload.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include <unistd.h>

#include <chrono>
#include <string>
#include <vector>

extern char** environ;

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

// One-shot all-reduce of slice [lo, hi) of n elements: sum over all peers' buffers, write to all.
// 16-byte path: each thread owns 8 consecutive bf16 (one uint4 per peer), loads the uint4 of
// EVERY peer first (up to 8 independent 16-B xGMI reads in flight per thread), sums in f32 in
// peer order, rounds once to bf16 and stores one uint4 to every peer.  `lo` must be a multiple of
// 8 elements for the vector part (slices are cut that way); a ragged tail of < 8 elements at the
// end of the slice takes the scalar path.  Peer count <= 8 (the node's GPUs).
constexpr int kMaxPeers = 8;

__device__ __forceinline__ void add8(float (&acc)[8], const uint4 v) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc[2 * j] += __uint_as_float(w[j] << 16);
    acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
  }
}

__global__ __launch_bounds__(256) void direct_allreduce(u16** bufs, int npeers, long lo, long hi) {
  const long nvec = (hi - lo) / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const long e = lo + 8 * v;
    uint4 in[kMaxPeers];
#pragma unroll
    for (int p = 0; p < kMaxPeers; ++p)
      if (p < npeers) in[p] = *reinterpret_cast<const uint4*>(bufs[p] + e);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < kMaxPeers; ++p)
      if (p < npeers) add8(acc, in[p]);
    uint4 out;
    out.x = (unsigned)f2b(acc[0]) | ((unsigned)f2b(acc[1]) << 16);
    out.y = (unsigned)f2b(acc[2]) | ((unsigned)f2b(acc[3]) << 16);
    out.z = (unsigned)f2b(acc[4]) | ((unsigned)f2b(acc[5]) << 16);
    out.w = (unsigned)f2b(acc[6]) | ((unsigned)f2b(acc[7]) << 16);
#pragma unroll
    for (int p = 0; p < kMaxPeers; ++p)
      if (p < npeers) *reinterpret_cast<uint4*>(bufs[p] + e) = out;
  }
  for (long i = lo + 8 * nvec + blockIdx.x * (long)blockDim.x + threadIdx.x; i < hi; i += stride) {  // tail
    float s = 0.f;
    for (int p = 0; p < npeers; ++p) s += b2f(bufs[p][i]);
    const u16 v = f2b(s);
    for (int p = 0; p < npeers; ++p) bufs[p][i] = v;
  }
}

// slice [lo, hi) of rank r: 8-element aligned cuts, the last slice takes the remainder
static void slice_of(long count, int n, int r, long* lo, long* hi) {
  long per = (count + n - 1) / n;
  per = (per + 7) / 8 * 8;
  *lo = (long)r * per < count ? (long)r * per : count;
  *hi = *lo + per < count ? *lo + per : count;
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
  for (int r = 0; r < vpeers; ++r) {
    long lo, hi;
    slice_of(count, vpeers, r, &lo, &hi);
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

static std::string env_json() {
  std::string o = "{";
  bool first = true;
  for (char** e = environ; *e; ++e) {
    const std::string kv(*e);
    if (kv.rfind("NCCL_", 0) != 0 && kv.rfind("RCCL_", 0) != 0 && kv.rfind("HSA_ENABLE_IPC", 0) != 0) continue;
    const size_t eq = kv.find('=');
    std::string k = kv.substr(0, eq), v = eq == std::string::npos ? "" : kv.substr(eq + 1), vv;
    for (char c : v) {
      if (c == '"' || c == '\\') vv += '\\';
      if ((unsigned char)c >= 0x20) vv += c;
    }
    o += std::string(first ? "" : ",") + "\"" + k + "\":\"" + vv + "\"";
    first = false;
  }
  return o + "}";
}

static void header(const char* mode, int world) {
  int ver = 0;
  ncclGetVersion(&ver);
  printf("{\"rccl_bench\":1,\"mode\":\"%s\",\"world\":%d,\"rccl_version\":%d,\"env\":%s}\n", mode, world, ver,
         env_json().c_str());
  fflush(stdout);
}

static void emit(const char* op, const char* mode, int n, long bytes, double sec) {
  const double alg = bytes / sec / 1e9;
  const double factor = strstr(op, "allreduce") ? 2.0 * (n - 1) / n : (double)(n - 1) / n;
  printf("{\"op\":\"%s\",\"mode\":\"%s\",\"gpus\":%d,\"bytes\":%ld,\"time_us\":%.1f,\"algbw_GBps\":%.2f,"
         "\"busbw_GBps\":%.2f}\n", op, mode, n, bytes, sec * 1e6, alg, alg * factor);
  fflush(stdout);
}

static ncclResult_t launch(const char* o, u16* sb, u16* rb, size_t count, int n, ncclComm_t c, hipStream_t s) {
  if (!strcmp(o, "allreduce")) return ncclAllReduce(sb, rb, count, ncclBfloat16, ncclSum, c, s);
  if (!strcmp(o, "reducescatter")) return ncclReduceScatter(sb, rb, count / n, ncclBfloat16, ncclSum, c, s);
  return ncclAllGather(sb, rb, count / n, ncclBfloat16, c, s);
}

// One process per GPU under torchrun: ncclCommInitRank with a file-published unique id.
static int per_rank(long mn, long mx, int iters, const std::string& op) {
  const char* er = getenv("RANK");
  const char* ew = getenv("WORLD_SIZE");
  const char* el = getenv("LOCAL_RANK");
  if (!er || !ew) {
    fprintf(stderr, "rccl-bench --per-rank: RANK / WORLD_SIZE not set (start it with torchrun --no-python)\n");
    return 2;
  }
  const int rank = atoi(er), world = atoi(ew), local = el ? atoi(el) : rank;
  int avail = 0;
  CK(hipGetDeviceCount(&avail));
  if (avail < 1) return 1;
  CK(hipSetDevice(local % avail));
  const char* dir = getenv("TH_NCCL_ID_DIR");
  const char* run = getenv("TORCHELASTIC_RUN_ID");
  const char* port = getenv("MASTER_PORT");
  const std::string path = std::string(dir ? dir : "/tmp") + "/rccl-bench-" + (run ? run : "run") + "-" +
                           (port ? port : "0") + ".id";
  ncclUniqueId id;
  if (rank == 0) {
    NK(ncclGetUniqueId(&id));
    const std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(&id, sizeof id, 1, f) != 1) return 1;
    fclose(f);
    if (rename(tmp.c_str(), path.c_str()) != 0) return 1;
  } else {
    bool got = false;
    for (int t = 0; t < 1200 && !got; ++t) {  // up to 60 s
      FILE* f = fopen(path.c_str(), "rb");
      if (f) {
        got = fread(&id, sizeof id, 1, f) == 1;
        fclose(f);
      }
      if (!got) usleep(50000);
    }
    if (!got) {
      fprintf(stderr, "rank %d: no unique id at %s\n", rank, path.c_str());
      return 1;
    }
  }
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, world, id, rank));
  if (rank == 0) unlink(path.c_str());
  hipStream_t st;
  CK(hipStreamCreate(&st));
  u16 *sb, *rb;
  double* tbuf;
  CK(hipMalloc((void**)&sb, mx));
  CK(hipMalloc((void**)&rb, mx));
  CK(hipMalloc((void**)&tbuf, sizeof(double)));
  CK(hipMemset(sb, 0, mx));
  if (rank == 0) header("per_rank", world);
  const char* ops[] = {"allreduce", "reducescatter", "allgather"};
  for (long bytes = mn; bytes <= mx; bytes *= 2) {
    const size_t count = bytes / 2;
    for (const char* o : ops) {
      if (op != "all" && op != o) continue;
      NK(launch(o, sb, rb, count, world, comm, st));  // warm-up, also lines the ranks up
      CK(hipStreamSynchronize(st));
      NK(ncclAllReduce(tbuf, tbuf, 1, ncclFloat64, ncclSum, comm, st));  // every rank starts together
      CK(hipStreamSynchronize(st));
      auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < iters; ++k) NK(launch(o, sb, rb, count, world, comm, st));
      CK(hipStreamSynchronize(st));
      double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
      CK(hipMemcpy(tbuf, &sec, sizeof sec, hipMemcpyHostToDevice));
      NK(ncclAllReduce(tbuf, tbuf, 1, ncclFloat64, ncclMax, comm, st));
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(&sec, tbuf, sizeof sec, hipMemcpyDeviceToHost));
      if (rank == 0) emit(o, "per_rank", world, bytes, sec);
    }
  }
  CK(hipFree(sb));
  CK(hipFree(rb));
  CK(hipFree(tbuf));
  ncclCommDestroy(comm);
  return 0;
}

int main(int argc, char** argv) {
  int ngpu = 0, iters = 20;
  int vpeers = 0;
  long mn = 8l << 20, mx = 1l << 30;
  std::string op = "all";
  bool direct = false, rank_mode = false;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--gpus") && i + 1 < argc) ngpu = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--min") && i + 1 < argc) mn = atol(argv[++i]);
    else if (!strcmp(argv[i], "--max") && i + 1 < argc) mx = atol(argv[++i]);
    else if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--op") && i + 1 < argc) op = argv[++i];
    else if (!strcmp(argv[i], "--direct")) direct = true;
    else if (!strcmp(argv[i], "--per-rank")) rank_mode = true;
    else if (!strcmp(argv[i], "--check-virtual-peers") && i + 1 < argc) vpeers = atoi(argv[++i]);
    else {
      fprintf(stderr, "usage: rccl-bench [--per-rank] [--gpus N] [--min B] [--max B] [--iters K] [--op OP] [--direct]\n"
                      "       rccl-bench --check-virtual-peers P [--min B]\n");
      return 2;
    }
  }
  if (getenv("TH_RCCL_PER_RANK") && !strcmp(getenv("TH_RCCL_PER_RANK"), "1")) {
    rank_mode = true;
    if (getenv("TH_RCCL_MIN")) mn = atol(getenv("TH_RCCL_MIN"));
    if (getenv("TH_RCCL_MAX")) mx = atol(getenv("TH_RCCL_MAX"));
    if (getenv("TH_RCCL_ITERS")) iters = atoi(getenv("TH_RCCL_ITERS"));
    if (getenv("TH_RCCL_OP")) op = getenv("TH_RCCL_OP");
  }
  if (mn < 16 || mx < mn || iters < 1) return 2;
  if (vpeers > 0) {
    if (vpeers > kMaxPeers) return 2;
    return check_direct(vpeers, (mn / 2) + 37);  // odd length: ragged last slice
  }
  if (rank_mode) return per_rank(mn, mx, iters, op);
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
  header("single_process", ngpu);
  const char* ops[] = {"allreduce", "reducescatter", "allgather"};
  for (long bytes = mn; bytes <= mx; bytes *= 2) {
    const size_t count = bytes / 2;
    for (const char* o : ops) {
      if (op != "all" && op != o) continue;
      auto run = [&]() {
        NK(ncclGroupStart());
        for (int i = 0; i < ngpu; ++i) NK(launch(o, sbuf[i], rbuf[i], count, ngpu, comms[i], st[i]));
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
      emit(o, "single_process", ngpu, bytes,
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters);
    }
    if (direct && ngpu > 1 && ngpu <= kMaxPeers) {
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
      auto run = [&]() {
        for (int i = 0; i < ngpu; ++i) {
          long lo, hi;
          slice_of((long)count, ngpu, i, &lo, &hi);
          CK(hipSetDevice(i));
          direct_allreduce<<<1024, 256, 0, st[i]>>>(dptrs[i], ngpu, lo, hi);
        }
        for (int i = 0; i < ngpu; ++i) {
          CK(hipSetDevice(i));
          CK(hipStreamSynchronize(st[i]));
        }
      };
      run();
      auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < iters; ++k) run();
      emit("direct_allreduce", "single_process", ngpu, bytes,
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters);
      for (int i = 0; i < ngpu; ++i) {
        CK(hipSetDevice(i));
        CK(hipFree(dptrs[i]));
      }
    }
  }
  for (int i = 0; i < ngpu; ++i) ncclCommDestroy(comms[i]);
  return 0;
}
