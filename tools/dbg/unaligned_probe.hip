// Does a global_load_dwordx4 from a byte-misaligned address return the 16
// bytes at that address on this box (SH_MEM_CONFIG unaligned mode), or the
// aligned line?  Decides whether k_b3_leaves can drop its v_alignbyte merge.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void k_probe(const uint8_t *src, uint4 *dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // lane i reads 16 bytes at src + 16 * (i / 16) + i % 16 (every misalignment)
  const uint8_t *p = src + 16 * (i / 16) + (i % 16);
  uint4 v;
  asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  dst[i] = v;
}

int main() {
  const int n = 4096;
  std::vector<uint8_t> h(16 * n + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t *d; uint4 *o;
  if (hipMalloc(&d, h.size()) || hipMalloc(&o, n * 16)) { printf("alloc failed\n"); return 2; }
  hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(n / 256), dim3(256), 0, 0, d, o, n);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
  std::vector<uint8_t> r(n * 16);
  hipMemcpy(r.data(), o, n * 16, hipMemcpyDeviceToHost);
  int bad = 0, bad_aligned = 0;
  for (int i = 0; i < n; ++i) {
    const size_t a = 16 * (i / 16) + (i % 16);
    if (memcmp(&r[16 * i], &h[a], 16) != 0) ++bad;
    if (memcmp(&r[16 * i], &h[a & ~(size_t)3], 16) != 0) ++bad_aligned;
  }
  printf("unaligned_probe: %d of %d loads differ from the bytes at the address; %d differ from the dword-aligned bytes\n",
         bad, n, bad_aligned);
  return 0;
}
