// scanbench.hip — microbenchmark of k_scan variants and pure-read ceilings.
// Not part of the product; build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   -I include tools/scanbench.hip -o tools/scanbench
#include "../mapache_amd/csrc/mcdc_kernels.hip"
#include "../mapache_amd/csrc/gear_table.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <string>

using namespace mcdc;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ __launch_bounds__(512) void k_read_coalesced(const uint4 *p, uint64_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int RUN>
__global__ __launch_bounds__(512) void k_read_strided(const uint8_t *base, uint64_t nruns, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t ntiles = nruns / 64;
  uint32_t acc = 0;
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const uint4 *p = reinterpret_cast<const uint4 *>(base + (t * 64 + lane) * (uint64_t)RUN);
#pragma unroll 4
    for (int i = 0; i < RUN / 16; ++i) {
      const uint4 v = p[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// compute ceiling: same work, but every run reads one of 1024 L2-resident runs
template <int RUN, int PF, int CH>
__global__ __launch_bounds__(512, 2) void k_scan_l2(Work W, DevParams P) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = W.gear16[i >> 5];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nfull = W.n_al / RUN;
  const uint64_t ntiles = nfull / 64;
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    scan_run_full<RUN, PF>(tab, lo, W, P, run, 1 + (run & 1023));
  }
}

static float time_it(hipStream_t st, int iters, const std::function<void()> &f, float *best) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  f();  // warm
  CK(hipStreamSynchronize(st));
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(a, st));
    f();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  *best = ts[0];
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  const uint64_t n = (argc > 1 ? strtoull(argv[1], 0, 10) : 16ull) << 30;
  const std::string mode = argc > 2 ? argv[2] : "all";
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint8_t *d;
  CK(hipMalloc(&d, n));
  launch_fill_random(d, 0, n, 0x6d61706163686521ull, st);
  uint64_t g16[256];
  for (int i = 0; i < 256; ++i) g16[i] = kGear[i] << 16;
  uint64_t *dg16;
  CK(hipMalloc(&dg16, 2048));
  CK(hipMemcpy(dg16, g16, 2048, hipMemcpyHostToDevice));
  const uint64_t nruns_max = n / 2048 + 1;
  uint8_t *cnt;
  uint32_t *ent, *sink;
  CK(hipMalloc(&cnt, nruns_max));
  CK(hipMalloc(&ent, nruns_max * 8 * 4));
  uint32_t *sum;
  CK(hipMalloc(&sum, nruns_max * 4));
  CK(hipMalloc(&sink, 64));
  DevParams P{};
  P.min = 16384; P.avg = 65536; P.max = 262144; P.cap = 8;
  P.ms = 0x0000d90703537000ull; P.ml = 0x0000d90f03530000ull;
  P.ms16 = P.ms << 16; P.ml16 = P.ml << 16;
  P.pf_hi = (uint32_t)((P.ms & P.ml) >> 16);
  Work W{};
  W.base = d; W.n_al = n; W.gear16 = dg16; W.run_cnt = cnt; W.run_ent = ent; W.run_sum = sum;
  W.nruns = (n + kRun - 1) / kRun;
  CK(hipStreamSynchronize(st));
  auto report = [&](const char *name, float med, float best) {
    printf("%-44s median %8.3f ms  %7.3f TB/s   best %7.3f TB/s\n", name, med, n / (med * 1e9), n / (best * 1e9));
    fflush(stdout);
  };
  auto cands = [&](uint64_t nr) {
    std::vector<uint8_t> c(nr);
    CK(hipMemcpy(c.data(), cnt, nr, hipMemcpyDeviceToHost));
    uint64_t tot = 0;
    for (auto x : c) tot += x;
    return tot;
  };
  float best, med;
  const int it = 7;
  auto prod = [&] { launch_scan(W, P, cus, st); };
  if (mode == "prod") {
    med = time_it(st, 3, prod, &best);
    report("scan product (quad-coalesced)", med, best);
    return 0;
  }
  if (mode == "var") {
    const uint64_t nr = W.nruns;
    std::vector<uint32_t> sv0, sv1;
    auto snap = [&](std::vector<uint8_t> &cv, std::vector<uint32_t> &ev) {
      cv.resize(nr); ev.resize(nr * 8);
      CK(hipMemcpy(cv.data(), cnt, nr, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ev.data(), ent, nr * 8 * 4, hipMemcpyDeviceToHost));
      sv1.resize(nr);
      CK(hipMemcpy(sv1.data(), sum, nr * 4, hipMemcpyDeviceToHost));
    };
    std::vector<uint8_t> c0, c1; std::vector<uint32_t> e0, e1;
    CK(hipMemset(ent, 0, nr * 8 * 4));
    {
      const uint64_t blocks = std::min<uint64_t>((W.nruns / 64 + 7) / 8, (uint64_t)cus * 2);
      hipLaunchKernelGGL((k_scan_t<kRun, 2, 1, 1, 512>), dim3(blocks), dim3(512), 0, st, W, P);
    }
    CK(hipStreamSynchronize(st)); snap(c0, e0); sv0 = sv1;
    auto check = [&](const char *name, const std::function<void()> &f) {
      CK(hipMemset(ent, 0, nr * 8 * 4)); CK(hipMemset(cnt, 0, nr));
      f(); CK(hipStreamSynchronize(st)); snap(c1, e1);
      bool ok = c0 == c1 && sv0 == sv1;
      for (uint64_t r = 0; ok && r < nr; ++r) {
        if (c0[r] > 8) continue;
        std::vector<uint32_t> x(e0.begin() + 8 * r, e0.begin() + 8 * r + c0[r]), y(e1.begin() + 8 * r, e1.begin() + 8 * r + c0[r]);
        std::sort(x.begin(), x.end()); std::sort(y.begin(), y.end());
        ok = x == y;
      }
      med = time_it(st, 5, f, &best);
      char nm[96]; snprintf(nm, sizeof nm, "%s %s", name, ok ? "[ok]" : "[MISMATCH]");
      report(nm, med, best);
    };
    check("product k_scan_q", prod);
    check("lane-strided k_scan_t (reference)", [&] {
      const uint64_t blocks = std::min<uint64_t>((W.nruns / 64 + 7) / 8, (uint64_t)cus * 2);
      hipLaunchKernelGGL((k_scan_t<kRun, 2, 1, 1, 512>), dim3(blocks), dim3(512), 0, st, W, P);
    });
    return 0;
  }
  if (mode == "sweep") {
    for (uint64_t sz = 32ull << 20; sz <= n; sz *= 2) {
      Work Ws = W; Ws.n_al = sz; Ws.nruns = (sz + kRun - 1) / kRun;
      const int reps = (int)std::max<uint64_t>(1, (4ull << 30) / sz);
      med = time_it(st, 5, [&] { for (int r = 0; r < reps; ++r) launch_scan(Ws, P, cus, st); }, &best);
      printf("sweep %8.1f MiB x%3d: %7.3f TB/s (best %7.3f)\n", sz / 1048576.0, reps,
             sz * (double)reps / (med * 1e9), sz * (double)reps / (best * 1e9));
      fflush(stdout);
    }
    return 0;
  }
  for (int bpc : {2, 4}) {
    med = time_it(st, it, [&] {
      hipLaunchKernelGGL(k_read_coalesced, dim3(cus * bpc), dim3(512), 0, st, (const uint4 *)d, n / 16, sink);
    }, &best);
    char nm[64];
    snprintf(nm, sizeof nm, "read coalesced %d blk/CU", bpc);
    report(nm, med, best);
  }
  med = time_it(st, it, [&] {
    hipLaunchKernelGGL(k_read_strided<4096>, dim3(cus * 2), dim3(512), 0, st, (const uint8_t *)d, n / 4096, sink);
  }, &best);
  report("read lane-strided RUN=4096", med, best);
  {
    const uint64_t nr = n / 2048;
    const uint64_t blocks = std::min<uint64_t>((nr / 64 + 7) / 8, (uint64_t)cus * 2);
    med = time_it(st, it, [&] {
      hipLaunchKernelGGL((k_scan_l2<2048, 1, 1>), dim3(blocks), dim3(512), 0, st, W, P);
    }, &best);
    report("lane-strided scan, L2-resident (compute)", med, best);
    CK(hipMemsetAsync(cnt, 0, nruns_max, st));
    med = time_it(st, it, [&] {
      hipLaunchKernelGGL((k_scan_t<2048, 2, 1, 1, 512>), dim3(blocks), dim3(512), 0, st, W, P);
    }, &best);
    printf("lane-strided cands %llu\n", (unsigned long long)cands(nr));
    report("lane-strided scan RUN=2048 (previous)", med, best);
  }
  CK(hipMemsetAsync(cnt, 0, nruns_max, st));
  med = time_it(st, it, prod, &best);
  printf("product cands %llu\n", (unsigned long long)cands(W.nruns));
  report("product scan (quad-coalesced, RUN=kRun)", med, best);
  return 0;
}
