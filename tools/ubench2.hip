// ubench2.hip — per-instruction issue rates on one CU-full of waves, timed
// in-kernel with s_memtime (core clock) and s_memrealtime (100 MHz), so the
// result is in cycles per wave-instruction independent of DVFS.
// Not part of the product.  build: hipcc --offload-arch=gfx950 -O3 tools/ubench2.hip -o tools/ubench2
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

constexpr int ITERS = 2048;

__device__ __forceinline__ uint64_t memtime() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ uint64_t realtime() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int MODE>
__global__ __launch_bounds__(1024) void kb(uint64_t *out, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = 0x9e3779b97f4a7c15ull * (i + seed);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19;
  uint32_t b0 = a0 ^ 1, b1 = a1 ^ 1, b2 = a2 ^ 1, b3 = a3 ^ 1, b4 = a4 ^ 1, b5 = a5 ^ 1, b6 = a6 ^ 1, b7 = a7 ^ 1;
  uint64_t h0 = a0, h1 = a1, h2 = a2, h3 = a3, h4 = a4, h5 = a5, h6 = a6, h7 = a7;
  const uint32_t k = seed | 1, sel = 0x0c0c0400u + seed - 1;
  const uint64_t g = 0x1234567ull * seed;
  const uint64_t c0 = memtime(), r0 = realtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (MODE == 0) {  // v_add_u32 x8
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 1) {  // v_perm_b32 x8
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(lo), "s"(sel));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 2) {  // v_lshl_add_u64 x8
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(h##i) : "v"(g));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 3) {  // v_min3_u32 x8
#define X(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 4) {  // v_and_b32 with SGPR x8
#define X(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a##i) : "s"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 5) {  // ds_read_b64 x8 (independent, conflict-free)
#define X(i) asm volatile("ds_read_b64 %0, %1" : "=v"(h##i) : "v"(((a##i & 0xff) << 8) | lo));
      R8(X) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      R8(X) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#undef X
    } else if constexpr (MODE == 6) {  // v_add_co + v_addc (64-bit add as 2 x 32)
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(a##i), "+v"(b##i) : "v"(k) : "vcc");
      R8(X)
#undef X
    } else if constexpr (MODE == 7) {  // v_bitop3_b32 x8
#define X(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 8) {  // v_pk_min_u16 x8
#define X(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 9) {  // v_lshlrev_b64 x8
#define X(i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(h##i));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 10) {  // v_alignbit_b32 x8
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 11) {  // v_mad_u64_u32 x8
#define X(i) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(h##i) : "v"(k), "v"(lo) : "s0", "s1");
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 12) {  // v_pk_add_u16 x8
#define X(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 13) {  // v_cndmask + v_cmp (per lane select)
#define X(i) asm volatile("v_cmp_eq_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(k) : "vcc");
      R8(X)
#undef X
    } else if constexpr (MODE == 14) {  // v_mov_b32_sdwa byte->byte1 (address build)
#define X(i) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 15) {  // v_and_b32 VGPR,VGPR
#define X(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 16) {  // v_min_u32 VOP2
#define X(i) asm volatile("v_min_u32 %0, %1, %0" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 17) {  // v_lshl_or_b32
#define X(i) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 18) {  // v_and_or_b32
#define X(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 19) {  // v_perm_b32 with VGPR selector
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(lo), "v"(sel));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 20) {  // v_add_u32 with SGPR
#define X(i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a##i) : "s"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 21) {  // v_xor_b32
#define X(i) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 22) {  // v_add3_u32
#define X(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 23) {  // v_and_b32_sdwa (byte select of src0) -> dst byte1 preserve
#define X(i) asm volatile("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3 src1_sel:DWORD" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 24) {  // v_mov_b32
#define X(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a##i) : "v"(b##i));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 25) {  // v_max3_u32
#define X(i) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(k), "v"(lo));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 26) {  // v_min_u32_sdwa (word select)
#define X(i) asm volatile("v_min_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(a##i) : "v"(k));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 27) {  // v_lshl_add_u64 with SGPR addend
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(h##i) : "s"(g));
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 28) {  // v_cmp_eq_u32 into SGPR pair (s_or accumulation left out)
#define X(i) asm volatile("v_cmp_eq_u32 s[2:3], %0, %1" :: "v"(a##i), "v"(k) : "s2", "s3");
      R8(X) R8(X)
#undef X
    } else if constexpr (MODE == 29) {  // real step mix: perm, lshl_add, and, 0.5 min3 (8 chains)
#define X(i) asm volatile("v_perm_b32 %0, %0, %2, %3\n\tv_lshl_add_u64 %1, %1, 1, %4\n\tv_and_b32 %0, %5, %0" : "+v"(a##i), "+v"(h##i) : "v"(lo), "s"(sel), "v"(g), "s"(k));
      R8(X)
#undef X
    } else if constexpr (MODE == 30) {  // alt mix: sdwa mov, lshl_add, bitop3-and
#define X(i) asm volatile("v_mov_b32_sdwa %0, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\tv_lshl_add_u64 %1, %1, 1, %4\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0xc0" : "+v"(a##i), "+v"(h##i) : "v"(k), "v"(lo), "v"(g));
      R8(X)
#undef X
    }
  }
  const uint64_t c1 = memtime(), r1 = realtime();
  const uint64_t x = h0 ^ h1 ^ h2 ^ h3 ^ h4 ^ h5 ^ h6 ^ h7 ^ a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
  if (lane == 0) {
    out[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 3 + 0] = c1 - c0;
    out[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 3 + 1] = r1 - r0;
    out[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 3 + 2] = x;
  }
}

template <int MODE>
int run(const char *name, int ops, uint64_t *out, int cus, int waves) {
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<MODE>, dim3(cus), dim3(64 * waves), 0, 0, out, 1u + rep);
    CK(hipDeviceSynchronize());
  }
  std::vector<uint64_t> h((size_t)cus * 16 * 3);
  CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> cyc, clk;
  for (int b = 0; b < cus; ++b)
    for (int w = 0; w < waves; ++w) {
      cyc.push_back((double)h[(b * 16 + w) * 3]);
      clk.push_back((double)h[(b * 16 + w) * 3] / (double)h[(b * 16 + w) * 3 + 1] * 0.1);
    }
  std::sort(cyc.begin(), cyc.end());
  std::sort(clk.begin(), clk.end());
  const double c = cyc[cyc.size() / 2];
  const double wi = (double)ITERS * ops * waves;  // wave-instructions per CU
  printf("%-16s waves/CU=%2d  %.3f wave-instr/clk/CU  (%.2f clk per wave-instr per SIMD)  clk %.2f GHz\n", name, waves,
         wi / c, c / (wi / 4), clk[clk.size() / 2]);
  fflush(stdout);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t *out;
  CK(hipMalloc(&out, (size_t)cus * 16 * 3 * 8));
  for (int waves : {16, 8}) {
    run<0>("v_add_u32", 16, out, cus, waves);
    run<20>("v_add_u32 sgpr", 16, out, cus, waves);
    run<1>("v_perm_b32 s", 16, out, cus, waves);
    run<19>("v_perm_b32 v", 16, out, cus, waves);
    run<14>("v_mov_b32_sdwa", 16, out, cus, waves);
    run<23>("v_and_b32_sdwa", 16, out, cus, waves);
    run<2>("v_lshl_add_u64", 16, out, cus, waves);
    run<27>("lshl_add_u64 s", 16, out, cus, waves);
    run<3>("v_min3_u32", 16, out, cus, waves);
    run<25>("v_max3_u32", 16, out, cus, waves);
    run<16>("v_min_u32", 16, out, cus, waves);
    run<26>("v_min_u32_sdwa", 16, out, cus, waves);
    run<4>("v_and_b32 s", 16, out, cus, waves);
    run<15>("v_and_b32 v", 16, out, cus, waves);
    run<21>("v_xor_b32", 16, out, cus, waves);
    run<7>("v_bitop3_b32", 16, out, cus, waves);
    run<17>("v_lshl_or_b32", 16, out, cus, waves);
    run<18>("v_and_or_b32", 16, out, cus, waves);
    run<22>("v_add3_u32", 16, out, cus, waves);
    run<24>("v_mov_b32", 16, out, cus, waves);
    run<28>("v_cmp_eq_u32 s", 16, out, cus, waves);
    run<13>("cmp+cndmask", 16, out, cus, waves);
    run<5>("ds_read_b64", 16, out, cus, waves);
    run<29>("mix perm/lsh/and", 24, out, cus, waves);
    run<30>("mix sdwa/lsh/bop3", 24, out, cus, waves);
  }
  return 0;
}
