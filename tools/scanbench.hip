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

// Diagnostic: s_memtime stamps split each group into load-wait and compute.
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
template <int RUN, int L2>
__global__ __launch_bounds__(512, 2) void k_scan_diag(Work W, DevParams P, uint64_t *dbg) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = W.gear16[i >> 5];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t ntiles = W.n_al / RUN / 64;
  uint64_t twait = 0, tcomp = 0, tall0 = stamp();
  const uint32_t pf = P.pf_hi, cap = P.cap;
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    const uint64_t ar = L2 ? 1 + (run & 1023) : run;
    const uint4 *p = reinterpret_cast<const uint4 *>(W.base + ar * (uint64_t)RUN);
    uint64_t h = 0;
    uint32_t *ent = W.run_ent + run * (uint64_t)cap;
    uint32_t cnt = 0;
    constexpr int G = RUN / 64;
    uint4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], b0, b1, b2, b3;
    for (int g = 0; g < G; g += 2) {
      const uint4 *qb = p + 4 * (g + 1);
      const uint4 *qa = p + 4 * (g + 2 < G ? g + 2 : g + 1);
      b0 = qb[0]; b1 = qb[1]; b2 = qb[2]; b3 = qb[3];
      uint64_t t0 = stamp();
      __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): group g landed
      asm volatile("" ::: "memory");
      uint64_t t1 = stamp();
      scan16(tab, lo, a0, h, pf, P.ms16, P.ml16, 64 * g, cnt, ent, cap);
      scan16(tab, lo, a1, h, pf, P.ms16, P.ml16, 64 * g + 16, cnt, ent, cap);
      scan16(tab, lo, a2, h, pf, P.ms16, P.ml16, 64 * g + 32, cnt, ent, cap);
      scan16(tab, lo, a3, h, pf, P.ms16, P.ml16, 64 * g + 48, cnt, ent, cap);
      a0 = qa[0]; a1 = qa[1]; a2 = qa[2]; a3 = qa[3];
      uint64_t t2 = stamp();
      __builtin_amdgcn_s_waitcnt(0x0F74);
      asm volatile("" ::: "memory");
      uint64_t t3 = stamp();
      scan16(tab, lo, b0, h, pf, P.ms16, P.ml16, 64 * g + 64, cnt, ent, cap);
      scan16(tab, lo, b1, h, pf, P.ms16, P.ml16, 64 * g + 80, cnt, ent, cap);
      scan16(tab, lo, b2, h, pf, P.ms16, P.ml16, 64 * g + 96, cnt, ent, cap);
      scan16(tab, lo, b3, h, pf, P.ms16, P.ml16, 64 * g + 112, cnt, ent, cap);
      uint64_t t4 = stamp();
      twait += (t1 - t0) + (t3 - t2);
      tcomp += (t2 - t1) + (t4 - t3);
    }
    W.run_cnt[run] = cnt > cap ? kRunOverflow : (uint8_t)cnt;
  }
  uint64_t tall = stamp() - tall0;
  if (lane == 0) { dbg[wid * 4 + 0] = twait; dbg[wid * 4 + 1] = tcomp; dbg[wid * 4 + 2] = tall; }
}

// Calibration: the product's quad-coalesced ping-pong load pattern with no
// hashing (known byte count for FETCH_SIZE calibration).
template <int RUN>
__global__ __launch_bounds__(1024) void k_read_quad(const uint8_t *base, uint64_t n, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63, qi = lane >> 2, qj = lane & 3;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t ntiles = n / RUN / 64;
  constexpr int G = RUN / 64;
  uint32_t acc = 0;
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const uint8_t *tb = base + t * 64 * (uint64_t)RUN;
    const uint32_t o0 = 4 * qi * RUN + 16 * qj;
#define LQ(k, gg) (*reinterpret_cast<const uint4 *>(tb + (uint64_t)(uint32_t)(o0 + (k) * RUN + 64 * (gg))))
    uint4 a0 = LQ(0, 0), a1 = LQ(1, 0), a2 = LQ(2, 0), a3 = LQ(3, 0);
    uint4 b0 = LQ(0, 1), b1 = LQ(1, 1), b2 = LQ(2, 1), b3 = LQ(3, 1);
#pragma unroll 1
    for (int g = 0; g < G; g += 2) {
      acc ^= (a0.x ^ a0.y ^ a0.z ^ a0.w) + (a1.x ^ a1.y ^ a1.z ^ a1.w) + (a2.x ^ a2.y ^ a2.z ^ a2.w) + (a3.x ^ a3.y ^ a3.z ^ a3.w);
      const int gn = g + 2 < G ? g + 2 : G - 1;
      a0 = LQ(0, gn); a1 = LQ(1, gn); a2 = LQ(2, gn); a3 = LQ(3, gn);
      acc ^= (b0.x ^ b0.y ^ b0.z ^ b0.w) + (b1.x ^ b1.y ^ b1.z ^ b1.w) + (b2.x ^ b2.y ^ b2.z ^ b2.w) + (b3.x ^ b3.y ^ b3.z ^ b3.w);
      const int gm = g + 3 < G ? g + 3 : G - 1;
      b0 = LQ(0, gm); b1 = LQ(1, gm); b2 = LQ(2, gm); b3 = LQ(3, gm);
    }
#undef LQ
  }
  if (acc == 0x12345678u) sink[0] = acc;
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
  // everything the product scan writes besides the run data (round 3: the
  // candidate bitmaps, the call's error words; the dynamic tile counter)
  const size_t bits_bytes = 16 * (W.nruns / 64 + 2);
  CK(hipMalloc(&W.run_bits, bits_bytes));
  CK(hipMalloc(&W.err, 64));
  CK(hipMalloc(&W.tile_ctr, 64));
  CK(hipMemset(W.run_bits, 0, bits_bytes));
  CK(hipMemset(W.err, 0, 64));
  W.long_n = W.err + 3;
  W.first_static = 1;
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
  auto prod = [&] {  // (as run_pipeline: bitmaps and the tile counter cleared before the launch)
    (void)hipMemsetAsync(W.run_bits, 0, bits_bytes, st);
    (void)hipMemsetAsync(W.tile_ctr, 0, 8, st);
    launch_scan(W, P, cus, st, 0, ~0ull, true, scan_pieces(W.n_al / kRun, cus), true);
  };
  if (mode == "quadread") {
    med = time_it(st, 3, [&] {
      hipLaunchKernelGGL(k_read_quad<kRun>, dim3(cus), dim3(1024), 0, st, (const uint8_t *)d, n, sink);
    }, &best);
    report("quad-coalesced reads only (calibration)", med, best);
    return 0;
  }
  if (mode == "prod") {
    med = time_it(st, 3, prod, &best);
    report("scan product (quad-coalesced)", med, best);
    return 0;
  }
  if (mode == "var") {
    const uint64_t nr = W.nruns;
    auto snap = [&](std::vector<uint8_t> &cv, std::vector<uint32_t> &ev) {
      cv.resize(nr); ev.resize(nr * 8);
      CK(hipMemcpy(cv.data(), cnt, nr, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ev.data(), ent, nr * 8 * 4, hipMemcpyDeviceToHost));
    };
    std::vector<uint8_t> c0, c1; std::vector<uint32_t> e0, e1;
    CK(hipMemset(ent, 0, nr * 8 * 4));
    {
      const uint64_t blocks = std::min<uint64_t>((W.nruns / 64 + 7) / 8, (uint64_t)cus * 2);
      hipLaunchKernelGGL((k_scan_t<kRun, 2, 1, 1, 512>), dim3(blocks), dim3(512), 0, st, W, P);
    }
    CK(hipStreamSynchronize(st)); snap(c0, e0);
    auto check = [&](const char *name, const std::function<void()> &f) {
      CK(hipMemset(ent, 0, nr * 8 * 4)); CK(hipMemset(cnt, 0, nr));
      f(); CK(hipStreamSynchronize(st)); snap(c1, e1);
      bool ok = c0 == c1;
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
      med = time_it(st, 5, [&] {
        for (int r = 0; r < reps; ++r) {
          (void)hipMemsetAsync(Ws.tile_ctr, 0, 8, st);
          launch_scan(Ws, P, cus, st, 0, ~0ull, true, scan_pieces(Ws.n_al / kRun, cus), true);
        }
      }, &best);
      printf("sweep %8.1f MiB x%3d: %7.3f TB/s (best %7.3f)\n", sz / 1048576.0, reps,
             sz * (double)reps / (med * 1e9), sz * (double)reps / (best * 1e9));
      fflush(stdout);
    }
    return 0;
  }
  if (mode == "diag") {
    uint64_t *dbg; CK(hipMalloc(&dbg, 8 * 4 * 8192)); CK(hipMemset(dbg, 0, 8 * 4 * 8192));
    const uint64_t nr = n / 2048;
    const uint64_t blocks = std::min<uint64_t>((nr / 64 + 7) / 8, (uint64_t)cus * 2);
    for (int l2 = 0; l2 < 2; ++l2) {
      med = time_it(st, 3, [&] {
        if (l2) hipLaunchKernelGGL((k_scan_diag<2048, 1>), dim3(blocks), dim3(512), 0, st, W, P, dbg);
        else hipLaunchKernelGGL((k_scan_diag<2048, 0>), dim3(blocks), dim3(512), 0, st, W, P, dbg);
      }, &best);
      std::vector<uint64_t> h(4 * blocks * 8);
      CK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
      double w = 0, c = 0, a = 0;
      for (uint64_t i = 0; i < blocks * 8; ++i) { w += h[4 * i]; c += h[4 * i + 1]; a += h[4 * i + 2]; }
      printf("diag %s: %.3f TB/s  per-wave cycles: wait %.3g compute %.3g all %.3g  (wait %.1f%%)  clk %.2f GHz\n",
             l2 ? "L2 " : "HBM", n / (med * 1e9), w / (blocks * 8), c / (blocks * 8), a / (blocks * 8),
             100.0 * w / (w + c), a / (blocks * 8) / (med * 1e-3) / 1e9);
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
