// mcdc_zframe.hip — CDNA4 (gfx950) zstd frames in raw-block ("store") mode
// for every chunk of a boundary list, in HBM: the format half of
// SecureStorage::compress (/root/reference/src/repository/storage.rs:74-84)
// without the entropy coding, so chunk -> frame -> seal stays on the GPU and
// the stored blobs remain readable by mapache's decoder (storage.rs:87-94:
// zstd Decoder, window_log_max 20).
//
// Frame (RFC 8878): magic 28 B5 2F FD; Frame_Header_Descriptor 0x00 (no
// content size, multi-segment, no checksum, no dictionary); Window_Descriptor
// 0x50 (2^20 bytes: storage.rs:31 WindowLog(log2 AVG_CHUNK_SIZE)); then raw
// blocks of at most 128 KiB, each a 3-byte little-endian header
// (Last_Block | Block_Type 0 << 1 | Block_Size << 3) and the bytes; an empty
// chunk is one empty last block.  Raw blocks are what zstd itself emits for
// data it cannot compress; for compressible data the host stage
// (host/zstd_stage.hpp) gives the reference's compression.
//
// Layout: frame i starts at a 16-byte aligned output offset (aligned stores;
// the sealing entry points take the frames as (offset, length) extents, so
// the gaps are never read).  One workgroup per chunk; each thread writes
// whole 16-byte output quads: inside a block's data a quad is one misaligned
// 16-byte load (gfx950 reads it as the bytes at that address,
// tools/dbg/unaligned_probe.hip), quads touching a header are assembled byte
// by byte.  HBM-bound: each input byte read once, written once.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "mcdc_zframe.h"

namespace mcdc {

namespace {

constexpr uint64_t kZBlock = 131072, kZHdr = 6, kZBlkHdr = 3;

__device__ __host__ __forceinline__ uint64_t zblocks(uint64_t len) { return len ? (len + kZBlock - 1) / kZBlock : 1; }
__device__ __host__ __forceinline__ uint64_t zframe_len(uint64_t len) { return kZHdr + kZBlkHdr * zblocks(len) + len; }

// byte p of the frame of a len-byte chunk at src
__device__ __forceinline__ uint8_t zbyte(const uint8_t *src, uint64_t len, uint64_t p) {
  if (p < kZHdr) {
    const uint8_t h[6] = {0x28, 0xB5, 0x2F, 0xFD, 0x00, 0x50};
    return h[p];
  }
  const uint64_t q = p - kZHdr, k = q / (kZBlock + kZBlkHdr), r = q % (kZBlock + kZBlkHdr);
  const uint64_t nb = zblocks(len);
  if (r < kZBlkHdr) {
    const uint64_t bsz = k + 1 < nb ? kZBlock : len - k * kZBlock;
    const uint32_t h = (uint32_t)(k + 1 == nb) | (uint32_t)(bsz << 3);
    return (uint8_t)(h >> (8 * r));
  }
  return src[k * kZBlock + (r - kZBlkHdr)];
}

__global__ void k_zframe_sizes(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *sz, uint32_t *err) {
  MCDC_VGPR_PAD(8);  // 8 used: not an exact fill (MCDC_VGPR_PAD)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const DevChunk c = chunks[i];
    const bool ok = c.offset <= nbytes && c.length <= nbytes - c.offset && c.length < (1ull << 31);
    if (!ok) atomicOr(err, 1u);
    sz[i] = ok ? (zframe_len(c.length) + 15) / 16 * 16 : 0;  // (16-byte aligned starts)
  } else if (i == n) {
    sz[i] = 0;
  }
}

typedef uint32_t zf_u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) zf_u32x4 *zf_gq;

// Same-box A/B (tools/zf_ab.sh, 16 GiB, 215 074 chunks): non-temporal frame
// stores 7.07 ms vs 7.40-7.56 ms plain; non-temporal loads, 2-4 quads per
// thread per step and 512/1024-thread workgroups gave nothing repeatable.
#ifndef MCDC_ZF_NT  // non-temporal stores of the frames (bit 0), loads of the chunk bytes (bit 1)
#define MCDC_ZF_NT 1
#endif
#ifndef MCDC_ZF_THREADS  // threads per chunk's workgroup
#define MCDC_ZF_THREADS 256
#endif

// the 16 bytes of output quad p of the frame of a len-byte chunk at src
__device__ __forceinline__ uint4 zquad(const uint8_t *__restrict__ src, uint64_t len, uint32_t fl32, uint32_t p) {
  // a quad wholly inside one block's data: one misaligned 16-byte load
  if (p >= kZHdr && p + 16 <= fl32) {
    const uint32_t a = p - (uint32_t)kZHdr, k = a / (uint32_t)(kZBlock + kZBlkHdr),
                   r = a - k * (uint32_t)(kZBlock + kZBlkHdr);
    if (r >= kZBlkHdr && r + 16 <= kZBlock + kZBlkHdr) {
      const uint32_t s = k * (uint32_t)kZBlock + (r - (uint32_t)kZBlkHdr);
#if MCDC_ZF_NT & 2
      const zf_u32x4 x = __builtin_nontemporal_load(reinterpret_cast<zf_gq>(reinterpret_cast<uintptr_t>(src + s)));
#else
      const zf_u32x4 x = *reinterpret_cast<zf_gq>(reinterpret_cast<uintptr_t>(src + s));
#endif
      return make_uint4(x.x, x.y, x.z, x.w);
    }
  }
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t b = 0; b < 16 && p + b < fl32; ++b) w[b >> 2] |= (uint32_t)zbyte(src, len, p + b) << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void zstore(uint8_t *__restrict__ dst, uint32_t fl32, uint32_t p, uint4 v) {
  if (p + 16 <= fl32) {
#if MCDC_ZF_NT & 1
    zf_u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<zf_u32x4 *>(dst + p));
#else
    *reinterpret_cast<uint4 *>(dst + p) = v;
#endif
  } else {  // the frame's last, partial quad: its own bytes only (the rest is the alignment gap)
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t b = 0; p + b < fl32; ++b) dst[p + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
  }
}

__global__ __launch_bounds__(MCDC_ZF_THREADS) void k_zframe_write(const uint8_t *__restrict__ base,
                                                                  const DevChunk *chunks, uint64_t n,
                                                                  const uint64_t *off, uint8_t *__restrict__ out,
                                                                  uint64_t *ext) {
  const uint64_t i = blockIdx.x;
  if (i >= n) return;
  const DevChunk c = chunks[i];
  const uint64_t fl = zframe_len(c.length), o = off[i];
  if (threadIdx.x == 0) {
    ext[2 * i] = o;
    ext[2 * i + 1] = fl;
  }
  const uint8_t *src = base + c.offset;
  uint8_t *dst = out + o;
  // (32-bit positions: chunks of 2 GiB and more are rejected by k_zframe_sizes)
  const uint32_t fl32 = (uint32_t)fl, step = 16 * blockDim.x;
  for (uint32_t p = 16 * threadIdx.x; p < fl32; p += step) zstore(dst, fl32, p, zquad(src, c.length, fl32, p));
}

}  // namespace

size_t zframe_tmp_bytes(uint64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n + 1);
  return b;
}

void launch_zframe_sizes(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *sz, uint64_t *off,
                         uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(k_zframe_sizes, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, chunks, n, nbytes, sz,
                     err);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, sz, off, (int)n + 1, st);
}

void launch_zframe_write(const uint8_t *base, const DevChunk *chunks, uint64_t n, const uint64_t *off, uint8_t *out,
                         uint64_t *ext, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_zframe_write, dim3((unsigned)n), dim3(MCDC_ZF_THREADS), 0, st, base, chunks, n, off, out,
                       ext);
}

// One workgroup per segment (grid-stride over segments): the bytes before the
// first 16-byte boundary of the source and after the last one byte by byte,
// the middle in aligned 16-byte loads and stores (the destination offset is
// congruent to the source's modulo 16, launch_gather's contract).
__global__ __launch_bounds__(256) void k_gather(const uint8_t *__restrict__ src, const uint64_t *__restrict__ ext,
                                                uint64_t n, uint8_t *__restrict__ dst) {
  MCDC_VGPR_PAD(16);  // (not an exact fill)
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t so = ext[3 * i], dof = ext[3 * i + 1], len = ext[3 * i + 2];
    const uint64_t head = min<uint64_t>(len, (16 - ((uintptr_t)(src + so) & 15)) & 15), nq = (len - head) / 16,
                   body = 16 * nq;
    for (uint64_t k = threadIdx.x; k < head; k += blockDim.x) dst[dof + k] = src[so + k];
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src + so + head);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst + dof + head);
    for (uint64_t k = threadIdx.x; k < nq; k += blockDim.x) d4[k] = s4[k];
    for (uint64_t k = head + body + threadIdx.x; k < len; k += blockDim.x) dst[dof + k] = src[so + k];
  }
}

void launch_gather(const uint8_t *src, const uint64_t *ext, uint64_t n, uint8_t *dst, hipStream_t st) {
  if (n == 0) return;
  const unsigned g = (unsigned)(n < 65536 ? n : 65536);
  hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, st, src, ext, n, dst);
}

}  // namespace mcdc
