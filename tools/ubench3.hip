// ubench3.hip — issue rate of the BLAKE3 G-function mix on gfx950 (cycles per
// wave-instruction per SIMD, in-kernel s_memtime), to check the VALU model the
// chunk-ID kernel is priced against.  Not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench3.hip -o tools/ubench3
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);   \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr int ITERS = 1024;

__device__ __forceinline__ uint64_t memtime() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// one G (12 VALU) on (a, b, c, d) with message words x, y, as the compiler emits it
#define G(a, b, c, d, x, y)                                                                   \
  asm volatile(                                                                              \
      "v_add3_u32 %0, %0, %1, %4\n\t"                                                        \
      "v_xor_b32 %3, %3, %0\n\t"                                                             \
      "v_alignbit_b32 %3, %3, %3, 16\n\t"                                                    \
      "v_add_u32 %2, %2, %3\n\t"                                                             \
      "v_xor_b32 %1, %1, %2\n\t"                                                             \
      "v_alignbit_b32 %1, %1, %1, 12\n\t"                                                    \
      "v_add3_u32 %0, %0, %1, %5\n\t"                                                        \
      "v_xor_b32 %3, %3, %0\n\t"                                                             \
      "v_alignbit_b32 %3, %3, %3, 8\n\t"                                                     \
      "v_add_u32 %2, %2, %3\n\t"                                                             \
      "v_xor_b32 %1, %1, %2\n\t"                                                             \
      "v_alignbit_b32 %1, %1, %1, 7"                                                         \
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)                                                   \
      : "v"(x), "v"(y));

// the product's compression (mcdc_blake3.hip) restated: 7 rounds of 8 G
struct Sched { uint8_t v[7][16]; };
constexpr Sched kS = {{{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                       {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                       {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                       {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                       {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                       {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                       {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}}};
__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
#define B3_G(a, b, c, d, mx, my) \
  a = a + b + (mx); d = rotr(d ^ a, 16); c = c + d; b = rotr(b ^ c, 12); \
  a = a + b + (my); d = rotr(d ^ a, 8); c = c + d; b = rotr(b ^ c, 7);
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint32_t ctr) {
  uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  uint32_t s8 = 0x6A09E667u, s9 = 0xBB67AE85u, s10 = 0x3C6EF372u, s11 = 0xA54FF53Au;
  uint32_t s12 = ctr, s13 = 0, s14 = 64, s15 = 3;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    B3_G(s0, s4, s8, s12, m[kS.v[r][0]], m[kS.v[r][1]])
    B3_G(s1, s5, s9, s13, m[kS.v[r][2]], m[kS.v[r][3]])
    B3_G(s2, s6, s10, s14, m[kS.v[r][4]], m[kS.v[r][5]])
    B3_G(s3, s7, s11, s15, m[kS.v[r][6]], m[kS.v[r][7]])
    B3_G(s0, s5, s10, s15, m[kS.v[r][8]], m[kS.v[r][9]])
    B3_G(s1, s6, s11, s12, m[kS.v[r][10]], m[kS.v[r][11]])
    B3_G(s2, s7, s8, s13, m[kS.v[r][12]], m[kS.v[r][13]])
    B3_G(s3, s4, s9, s14, m[kS.v[r][14]], m[kS.v[r][15]])
  }
  cv[0] = s0 ^ s8; cv[1] = s1 ^ s9; cv[2] = s2 ^ s10; cv[3] = s3 ^ s11;
  cv[4] = s4 ^ s12; cv[5] = s5 ^ s13; cv[6] = s6 ^ s14; cv[7] = s7 ^ s15;
}

template <int MODE>
__global__ __launch_bounds__(1024) void kb(uint64_t *out, uint32_t seed, const uint4 *src = nullptr) {
  uint32_t s[16], m0 = seed * 7 + threadIdx.x, m1 = m0 ^ 0x55;
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = seed * (i + 3) + threadIdx.x * (i + 1);
  uint4 nq[4] = {};
  if constexpr (MODE == 11) {  // de-phase the waves: wave w sleeps ~w * 420 cycles first
    for (uint32_t k = 0; k < (threadIdx.x >> 6); ++k) __builtin_amdgcn_s_sleep(7);
  }
  const uint64_t c0 = memtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (MODE == 0) {  // xor x16 independent
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(s[i]) : "v"(m0));
    } else if constexpr (MODE == 1) {  // alignbit x16
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(s[i]));
    } else if constexpr (MODE == 2) {  // add3 x16
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(s[i]) : "v"(m0), "v"(m1));
    } else if constexpr (MODE == 3) {  // 4 independent G (a round's column step): 48 VALU
      G(s[0], s[4], s[8], s[12], m0, m1) G(s[1], s[5], s[9], s[13], m1, m0)
      G(s[2], s[6], s[10], s[14], m0, m1) G(s[3], s[7], s[11], s[15], m1, m0)
    } else if constexpr (MODE == 4) {  // interleaved: xor/alignbit pairs x8 (rotate of a xor)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        asm volatile("v_xor_b32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 12" : "+v"(s[i]) : "v"(s[i + 8]));
    } else if constexpr (MODE == 5) {  // rotate as perm (16, 8) instead of alignbit
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(s[i]) : "v"(0x01000302u));
    } else if constexpr (MODE == 7 || MODE == 11) {  // the real compression, message words in registers
      uint32_t cv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) cv[i] = s[i];
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = s[i] ^ (uint32_t)it;
      compress(cv, m, (uint32_t)it);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = cv[i];
    } else if constexpr (MODE == 10) {  // as MODE 8, lanes 16 KiB apart (k_b3_leaves' pattern)
      uint32_t cv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) cv[i] = s[i];
      const uint4 *q = src + ((((threadIdx.x & 63) * 1024 + (blockIdx.x * 16 + (threadIdx.x >> 6)) * 4 + it * 4) & 0x7ffff) & ~3);
      const uint4 a0 = nq[0], a1 = nq[1], a2 = nq[2], a3 = nq[3];
      nq[0] = q[0]; nq[1] = q[1]; nq[2] = q[2]; nq[3] = q[3];
      const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                              a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
      compress(cv, m, (uint32_t)it);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = cv[i];
    } else if constexpr (MODE == 8 || MODE == 9) {  // compression fed by global loads (L2-resident source),
      // MODE 8: the next block requested before compressing (as k_b3_leaves), MODE 9: loaded and waited first
      static_assert(true, "");
      uint32_t cv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) cv[i] = s[i];
      const uint4 *q = src + ((threadIdx.x + blockIdx.x * 64 + it * 4096) & 0x1ffff) * 4;  // 8 MiB window
      uint4 a0, a1, a2, a3;
      if constexpr (MODE == 9) {
        a0 = q[0]; a1 = q[1]; a2 = q[2]; a3 = q[3];
      } else {
        a0 = nq[0]; a1 = nq[1]; a2 = nq[2]; a3 = nq[3];
        nq[0] = q[0]; nq[1] = q[1]; nq[2] = q[2]; nq[3] = q[3];
      }
      const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                              a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
      compress(cv, m, (uint32_t)it);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = cv[i];
    } else if constexpr (MODE == 6) {  // xor then 16-bit rotate via v_pk_... : v_xor + v_alignbyte
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(s[i]));
    }
  }
  const uint64_t c1 = memtime();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= s[i];
  if ((threadIdx.x & 63) == 0) {
    out[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2 + 0] = c1 - c0;
    out[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2 + 1] = x;
  }
}

// waves/CU as `waves` waves per workgroup, one workgroup per CU; or (split > 1)
// as `split` workgroups of waves/split waves each per CU
template <int MODE>
int run(const char *name, int ops, uint64_t *out, int cus, int waves, int split = 1, const uint4 *src = nullptr) {
  const int wpg = waves / split;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<MODE>, dim3(cus * split), dim3(64 * wpg), 0, 0, out, 1u + rep, src);
    CK(hipDeviceSynchronize());
  }
  std::vector<uint64_t> h((size_t)cus * split * 16 * 2);
  CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> cyc;
  for (int b = 0; b < cus * split; ++b)
    for (int w = 0; w < wpg; ++w) cyc.push_back((double)h[(b * 16 + w) * 2]);
  std::sort(cyc.begin(), cyc.end());
  const double c = cyc[cyc.size() / 2];
  const double wi = (double)ITERS * ops * waves;  // wave-instructions per CU
  printf("%-18s waves/CU=%2d in %d WG  %.2f clk per wave-instr per SIMD\n", name, waves, split, c / (wi / 4));
  fflush(stdout);
  return 0;
}

template <int MODE>
int run_wall(const char *name, int ops, uint64_t *out, int cus, int waves) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kb<MODE>, dim3(cus), dim3(64 * waves), 0, 0, out, 1u + rep, nullptr);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double wi = (double)ITERS * ops * waves;  // wave-instructions per CU
  printf("%-18s waves/CU=%2d  wall %.3f ms  %.3f ns per wave-instr per SIMD\n", name, waves, best,
         best * 1e6 / (wi / 4));
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t *out;
  CK(hipMalloc(&out, (size_t)cus * 16 * 16 * 2 * 8));  // room for 16 workgroups per CU
  uint4 *src;
  CK(hipMalloc(&src, (size_t)8 << 20));
  CK(hipMemset(src, 0x5a, (size_t)8 << 20));
  run_wall<11>("compress dephased", 696, out, cus, 16);
  run_wall<7>("compress in phase", 696, out, cus, 16);
  run<10>("compress+strided", 696, out, cus, 16, 1, src);
  run<8>("compress+prefetch", 696, out, cus, 16, 1, src);
  run<9>("compress+load", 696, out, cus, 16, 1, src);
  run<8>("compress+prefetch", 696, out, cus, 8, 1, src);
  run<7>("compress (real)", 696, out, cus, 16, 4);
  run<7>("compress (real)", 696, out, cus, 16, 2);
  run<3>("4 x G", 48, out, cus, 16, 4);
  run<3>("4 x G", 48, out, cus, 16, 16);
  run<7>("compress (real)", 696, out, cus, 16, 16);
  for (int waves : {16, 12, 8, 4}) {
    run<0>("v_xor_b32", 16, out, cus, waves);
    run<1>("v_alignbit_b32", 16, out, cus, waves);
    run<2>("v_add3_u32", 16, out, cus, waves);
    run<5>("v_perm rot16", 16, out, cus, waves);
    run<6>("v_alignbyte rot16", 16, out, cus, waves);
    run<4>("xor+alignbit", 16, out, cus, waves);
    run<3>("4 x G", 48, out, cus, waves);
    run<7>("compress (real)", 696, out, cus, waves);
  }
  return 0;
}
