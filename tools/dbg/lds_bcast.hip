// Microbenchmark for the k_emit_long LDS item: the product's
// chunk_hash over all-zero chunks with the GEAR table in LDS, many launches,
// every result checked against the known value.  Variants isolate the shape
// that lost LDS results in the probe (tools/dbg/lds_probe.py):
//   mode 0  chunk_hash from the LDS table (as k_emit_long with an LDS copy)
//   mode 1  chunk_hash from the global table (the product's k_emit_long)
//   mode 2  mode 0 with an s_nop-free wave (no other change) on random bytes
//           checked against the global-table hash computed in the same lane
// Usage: lds_bcast <mode> <launches> <chunks per launch>
#include "../../mapache_amd/csrc/mcdc_kernels.hip"
#include "../../mapache_amd/csrc/gear_table.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace mcdc;

__device__ unsigned long long g_bad[1 + 64 * 8];

__global__ __launch_bounds__(256) void k_test(Work W, DevParams P, uint64_t nchunks, uint64_t fend, uint64_t expect,
                                              int mode) {
  __shared__ uint64_t gtl[256];
  load_gear_lds(gtl, W);
#ifdef TOP_VGPR  // touch one register so that the kernel's VGPR count is TOP_VGPR + 1
#define STR2(x) #x
#define STR(x) STR2(x)
  asm volatile("v_mov_b32 v" STR(TOP_VGPR) ", 0" ::: "v" STR(TOP_VGPR));
#endif
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nchunks; i += stride) {
    if (mode >= 3) {  // delay like k_emit_long's cont_node walk: dependent global loads
      uint64_t x = i & 7;
      for (int k = 0; k < mode * 4; ++k) x = reinterpret_cast<const uint64_t *>(W.base)[x & 7] + ((x + 1) & 7);
      if (x == 12345678) g_bad[0] += 1;  // never: keeps the walk
    }
    const uint64_t pos = 1 + i * P.max;
    const ChunkQ cq = chunk_q(P, pos, P.max, fend);
    uint64_t h, want = expect;
    if (mode == 1) h = chunk_hash(W, W.gear, cq);
    else if (mode >= 3) h = chunk_hash(W, gtl, cq);
    else h = chunk_hash(W, gtl, cq);
    if (mode == 2) want = chunk_hash(W, W.gear, cq);
    if (h != want) {
      const unsigned long long k = atomicAdd(&g_bad[0], 1ull);
      if (k < 64) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_bad[1 + 8 * k] = blockIdx.x;
        g_bad[2 + 8 * k] = threadIdx.x;
        g_bad[3 + 8 * k] = i;
        g_bad[4 + 8 * k] = h;
        g_bad[5 + 8 * k] = want;
        g_bad[6 + 8 * k] = hw;
        g_bad[7 + 8 * k] = xcc;
        g_bad[8 + 8 * k] = __builtin_amdgcn_read_exec();
      }
    }
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char **argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int launches = argc > 2 ? atoi(argv[2]) : 1000;
  const uint64_t nchunks = argc > 3 ? strtoull(argv[3], nullptr, 10) : 80000;
  DevParams P{};
  P.min = 64; P.avg = 256; P.max = 1024;
  P.ms = 0x0000d90003530000ull; P.ml = 0x0000000018035100ull;  // unused by chunk_hash
  const uint64_t n = 16 + nchunks * P.max + 4096;
  uint8_t *d = nullptr;
  uint64_t *gear = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipMalloc(&gear, 2048));
  CK(hipMemcpy(gear, kGear, 2048, hipMemcpyHostToDevice));
  if (mode == 2) launch_fill_random(d, 0, n, 12345, 0);
  else CK(hipMemset(d, 0, n));
  Work W{};
  W.base = d;
  W.n_al = n;
  W.gear = gear;
  // expected hash of a forced 1024-byte chunk of zeros: sum_{s<64} GEAR[0] << s
  uint64_t expect = 0;
  for (int s = 0; s < 64; ++s) expect += kGear[0] << s;
  unsigned long long z = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_bad), &z, 8));
  const uint64_t fend = 1 + nchunks * P.max + 2048;  // every chunk has a successor: forced cuts
  for (int l = 0; l < launches; ++l) {
    hipLaunchKernelGGL(k_test, dim3(1024), dim3(256), 0, 0, W, P, nchunks, fend, expect, mode);
    if ((l & 63) == 63) CK(hipDeviceSynchronize());
  }
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> b(1 + 64 * 8);
  CK(hipMemcpyFromSymbol(b.data(), HIP_SYMBOL(g_bad), b.size() * 8));
  printf("mode %d launches %d chunks/launch %llu waves/launch %llu expect 0x%llx bad %llu\n", mode, launches,
         (unsigned long long)nchunks, (unsigned long long)((nchunks + 63) / 64), (unsigned long long)expect, b[0]);
  for (unsigned long long k = 0; k < b[0] && k < 16; ++k)
    printf("  blk %llu tid %llu i %llu h 0x%llx want 0x%llx hwid 0x%llx xcc %llu exec 0x%llx\n", b[1 + 8 * k],
           b[2 + 8 * k], b[3 + 8 * k], b[4 + 8 * k], b[5 + 8 * k], b[6 + 8 * k], b[7 + 8 * k], b[8 + 8 * k]);
  return 0;
}
