// ubench.hip — instruction-level microbenchmarks for the scan kernel design
// (not part of the product).  Reports lane-steps per second for:
//   chain1/2/4 : dependent v_lshl_add_u64 chains (1, 2, 4 independent per lane)
//   lds        : v_perm + ds_read_b64 lookups (independent, xor-accumulated)
//   lds+chain  : perm + lookup + 1 chain (no test)
//   full       : perm + lookup + chain + and/min test (the scan inner loop)
//   full32     : same, hash kept as two 32-bit halves with explicit carry
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int ITERS = 4096;

template <int MODE>
__global__ __launch_bounds__(1024) void kb(const uint64_t *g16, uint64_t *out, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = g16[i >> 5];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  uint32_t w = seed * 2654435761u + threadIdx.x * 40503u + blockIdx.x;
  uint64_t h0 = w, h1 = w * 3, h2 = w * 5, h3 = w * 7;
  uint32_t acc = 0xffffffff;
  uint64_t x = 0;
  const uint32_t pf = 0xd9070353u;
  for (int it = 0; it < ITERS; ++it) {
    w = w * 1664525u + 1013904223u;  // new data word each 4 steps (1 VALU)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = __builtin_amdgcn_perm(w, lo, 0x0c0c0000u | ((4u + k) << 8));
      if constexpr (MODE == 0) {  // chain1
        h0 = (h0 << 1) + (uint64_t)a;
      } else if constexpr (MODE == 1) {  // chain2
        h0 = (h0 << 1) + (uint64_t)a;
        h1 = (h1 << 1) + (uint64_t)a;
      } else if constexpr (MODE == 2) {  // chain4
        h0 = (h0 << 1) + (uint64_t)a;
        h1 = (h1 << 1) + (uint64_t)a;
        h2 = (h2 << 1) + (uint64_t)a;
        h3 = (h3 << 1) + (uint64_t)a;
      } else if constexpr (MODE == 3) {  // lds
        x ^= *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + a);
      } else if constexpr (MODE == 4) {  // lds + chain
        h0 = (h0 << 1) + *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + a);
      } else if constexpr (MODE == 5) {  // full
        h0 = (h0 << 1) + *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + a);
        acc = min(acc, (uint32_t)(h0 >> 32) & pf);
      } else if constexpr (MODE == 6) {  // full, 32-bit halves
        const uint64_t g = *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + a);
        uint32_t lo32 = (uint32_t)h0, hi32 = (uint32_t)(h0 >> 32);
        uint32_t nlo = (lo32 << 1) + (uint32_t)g;
        uint32_t carry = nlo < (lo32 << 1);
        hi32 = __builtin_amdgcn_alignbit(hi32, lo32, 31) + (uint32_t)(g >> 32) + carry;
        h0 = ((uint64_t)hi32 << 32) | nlo;
        acc = min(acc, hi32 & pf);
      } else if constexpr (MODE == 7) {  // perm only
        x += a;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3 ^ x ^ acc;
}

template <int MODE>
void run(const char *name, const uint64_t *g16, uint64_t *out, int blocks, int threads, int cus) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL(kb<MODE>, dim3(blocks), dim3(threads), 0, 0, g16, out, 1u);
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(kb<MODE>, dim3(blocks), dim3(threads), 0, 0, g16, out, (uint32_t)r);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double steps = (double)blocks * threads * ITERS * 4;
  const double per_s = steps / (t[2] * 1e-3);
  printf("%-12s blocks=%5d thr=%4d  %8.3f ms  %8.2f G lane-steps/s  (= %.2f TB/s if 1 step/byte)  per-CU-clk@2.4G %.2f\n",
         name, blocks, threads, t[2], per_s / 1e9, per_s / 1e12, per_s / cus / 2.4e9);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t *g16, *out;
  CK(hipMalloc(&g16, 2048)); CK(hipMalloc(&out, 64ull << 20));
  std::vector<uint64_t> h(256); for (int i = 0; i < 256; ++i) h[i] = (0x9e3779b97f4a7c15ull * (i + 1)) << 16;
  CK(hipMemcpy(g16, h.data(), 2048, hipMemcpyHostToDevice));
  for (int cfg = 0; cfg < 3; ++cfg) {   // 4, 16, 32 waves per CU (64 KiB LDS per block: <= 2 blocks/CU)
    const int thr = cfg == 0 ? 256 : 1024, bpc = cfg == 2 ? 2 : 1;
    printf("--- %d waves/CU\n", bpc * thr / 64);
    run<7>("perm", g16, out, cus * bpc, thr, cus);
    run<0>("chain1", g16, out, cus * bpc, thr, cus);
    run<1>("chain2", g16, out, cus * bpc, thr, cus);
    run<2>("chain4", g16, out, cus * bpc, thr, cus);
    run<3>("lds", g16, out, cus * bpc, thr, cus);
    run<4>("lds+chain", g16, out, cus * bpc, thr, cus);
    run<5>("full", g16, out, cus * bpc, thr, cus);
    run<6>("full32", g16, out, cus * bpc, thr, cus);
  }
  return 0;
}
