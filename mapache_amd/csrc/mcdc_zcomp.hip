// mcdc_zcomp.hip — CDNA4 (gfx950) zstd compression of every chunk of a
// boundary list, in HBM: SecureStorage::compress
// (/root/reference/src/repository/storage.rs:74-84) on the GPU, so the save
// path chunk -> IDs -> compress -> seal never leaves HBM.  One zstd frame per
// chunk (the blob mapache stores), in the crate's frame layout (magic, no
// content size, window 2^20, no checksum); blocks of 16 KiB, each either
// compressed (raw literals + predefined-FSE sequences, mcdc_zstd.h) or raw when
// that is not smaller.  Decodes with mapache's decoder (storage.rs:87-94).
//
// Per batch of blocks (a block = 16 KiB of one chunk; batches bound the
// scratch):
//   k_zc_blocks  block records of the batch's chunks (chunk, index, source)
//   k_zc_match   ONE WAVE PER BLOCK: greedy LZ parse.  A 2048-entry hash
//                table in LDS (positions, ds_max_u32 so the result does not
//                depend on lane timing) is primed with the previous 16 KiB of
//                the same chunk (matches reach back up to 32 KiB); the wave
//                hashes 64 positions at once (every step-th position after
//                match-free strides), verifies and extends each lane's
//                candidate, then walks the lanes' matches greedily (ballot +
//                readlane, wave-uniform); long matches are extended 64 bytes
//                per step.  Literals go to the block's staging slot, sequences
//                (<= kZcSeqCap = 4096 per block, then the rest are literals) straight to
//                scratch (8 KiB of LDS per wave: 20 waves per CU).
//   k_zc_encode  ONE LANE PER BLOCK: the serial FSE bitstream of the block's
//                sequences (three interleaved state machines, tables in LDS);
//                block kept compressed only if smaller than raw
//   scan         piece sizes (frame header on a chunk's first block, block
//                header, content) -> output offsets, frames back to back
//   k_zc_final   ONE WAVE PER BLOCK: headers + content (staging or input)
//                into the output, 16-byte loads/stores; frame extents.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "mcdc_zcomp.h"
#include "mcdc_zstd.h"

namespace mcdc {

namespace {

using namespace zs;

// 2048 positions (8 KiB of LDS per wave: 20 waves per CU; the compiler then
// allocates 88 VGPRs instead of the 136 it gives a 16 KiB table's 10 waves)
constexpr uint32_t kHtLog = 11, kHt = 1u << kHtLog;

__device__ __forceinline__ uint32_t ld4(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ uint32_t zhash(uint32_t v) { return (v * 2654435761u) >> (32 - kHtLog); }
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__global__ void k_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint32_t *err,
                             uint64_t *bound) {
  MCDC_VGPR_PAD(12);  // (not an exact fill)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t raw = 0;
  if (i < n) {
    const DevChunk c = chunks[i];
    const bool ok = c.offset <= nbytes && c.length <= nbytes - c.offset && c.length < (1ull << 31);
    if (!ok) atomicOr(err, 1u);
    const uint64_t nb = c.length ? (c.length + kZcBlock - 1) / kZcBlock : 1;
    cnt[i] = nb;
    raw = kFrameHdr + kBlockHdr * nb + c.length;
  } else if (i == n) {
    cnt[i] = 0;
  }
  for (int o = 32; o > 0; o >>= 1) raw += __shfl_down(raw, o);
  if (lane_id() == 0 && raw) atomicAdd(reinterpret_cast<unsigned long long *>(bound), (unsigned long long)raw);
}

__global__ void k_zc_blocks(const DevChunk *chunks, const uint64_t *first, uint64_t c0, uint64_t c1, uint64_t b0,
                            ZcBlock *blocks) {
  MCDC_VGPR_PAD(16);  // (not an exact fill)
  const uint64_t c = c0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= c1) return;
  const DevChunk ch = chunks[c];
  const uint64_t f = first[c], nb = first[c + 1] - f;
  for (uint64_t b = 0; b < nb; ++b) {
    ZcBlock z;
    z.src = ch.offset + b * kZcBlock;
    z.len = (uint32_t)(ch.length - b * kZcBlock < kZcBlock ? ch.length - b * kZcBlock : kZcBlock);
    z.chunk = (uint32_t)c;
    z.b = (uint32_t)b;
    z.nb = (uint32_t)nb;
    z.nlit = z.nseq = z.csize = 0;
    blocks[f + b - b0] = z;
  }
}

// Copy bytes [a, a + n) of src to dst, the whole wave (64 lanes) together.
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t lane) {
  for (uint32_t k = lane; k < n; k += 64) dst[k] = src[k];
}

// Match length at p against c, up to 32 bytes, from one 32-byte load on
// each side (two misaligned 16-byte loads each; no dependent loop).
__device__ __forceinline__ uint32_t match32(const uint8_t *p0, uint32_t p, uint32_t c, uint32_t end) {
  if (p + 32 <= end) {
    const uint4 x0 = *reinterpret_cast<const uint4 *>(p0 + p), x1 = *reinterpret_cast<const uint4 *>(p0 + p + 16);
    const uint4 y0 = *reinterpret_cast<const uint4 *>(p0 + c), y1 = *reinterpret_cast<const uint4 *>(p0 + c + 16);
    const uint32_t d[8] = {x0.x ^ y0.x, x0.y ^ y0.y, x0.z ^ y0.z, x0.w ^ y0.w,
                           x1.x ^ y1.x, x1.y ^ y1.y, x1.z ^ y1.z, x1.w ^ y1.w};
    uint32_t m = 32;
#pragma unroll
    for (int k = 7; k >= 0; --k)
      if (d[k]) m = 4 * k + ((uint32_t)__builtin_ctz(d[k]) >> 3);
    return m;
  }
  uint32_t m = 0;  // the block's last 31 bytes
  while (p + m < end && m < 32 && p0[c + m] == p0[p + m]) ++m;
  return m;
}

// Lane i of a stride looks at position s0 + i * step.  step grows after
// match-free strides (1, 2, 4, 8: zstd's fast strategies skip ahead the same
// way on data that does not compress) and drops back to 1 at a match.
// Literal runs are copied 64 at a time: lane (k mod 64) keeps run k's source,
// length and destination, and the wave copies the 64 runs together.
__global__ __launch_bounds__(64) void k_zc_match(const uint8_t *base, ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                 uint64_t *seqs) {
  __shared__ uint32_t ht[kHt];
  const uint64_t bi = blockIdx.x;
  if (bi >= nblk) return;
  const uint32_t lane = lane_id();
  ZcBlock B = blocks[bi];
  const uint32_t prime = B.b ? kZcBlock : 0;  // the previous 16 KiB of the chunk
  const uint8_t *p0 = base + B.src - prime;   // positions are relative to p0
  const uint32_t end = prime + B.len;
  for (uint32_t k = lane; k < kHt; k += 64) ht[k] = 0;
  __syncthreads();
  for (uint32_t q = lane; q + 4 <= prime; q += 64) atomicMax(&ht[zhash(ld4(p0 + q))], q + 1);
  __syncthreads();
  uint8_t *lit = stage + bi * kZcSlot + kLitHdr;
  uint64_t *sq = seqs + bi * kZcSeqCap;
  uint32_t nlit = 0, nseq = 0, cursor = prime, lit0 = prime, step = 1, miss = 0;
  uint32_t run_src = 0, run_len = 0, run_dst = 0;  // this lane's pending literal run
  auto flush_runs = [&]() {
    uint32_t mx = run_len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
    for (uint32_t k = 0; k < mx; ++k)
      if (k < run_len) lit[run_dst + k] = p0[run_src + k];
    run_len = 0;
  };
  for (uint32_t s0 = prime; s0 + 4 <= end;) {
    const uint32_t p = s0 + lane * step;
    const bool ok = p + 4 <= end;
    const uint32_t v = ok ? ld4(p0 + p) : 0u;
    const uint32_t h = zhash(v);
    const uint32_t cand = ok ? ht[h] : 0u;
    if (ok) atomicMax(&ht[h], p + 1);  // (issued after every lane's read: one wave, in order)
    uint32_t mlen = 0, c = 0;
    if (cand) {
      c = cand - 1;
      if (c < p && p - c < kWindow && ld4(p0 + c) == v) mlen = match32(p0, p, c, end);
    }
    const uint64_t m = __ballot(mlen >= kMinMatch);
    if (cursor < s0) cursor = s0;  // positions before s0 that no match covered are literals
    const uint32_t span = 64 * step;
    bool stop = false;
    while (true) {
      if (cursor >= s0 + span) break;
      const uint32_t first_lane = (cursor - s0 + step - 1) / step;  // lanes at or after the cursor
      if (first_lane >= 64) break;
      const uint64_t mm = m & (~0ull << first_lane);
      if (!mm) break;
      const uint32_t i = (uint32_t)__builtin_ctzll(mm);
      const uint32_t pos = s0 + i * step;
      uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)mlen, (int)i);
      const uint32_t off = pos - (uint32_t)__builtin_amdgcn_readlane((int)c, (int)i);
      if (ml == 32) {  // extend 64 bytes per step: lane k compares byte pos + ml + k
        for (;;) {
          const uint32_t q = pos + ml + lane;
          const bool same = q < end && p0[q] == p0[q - off];
          const uint64_t diff = __ballot(!same);
          ml += diff ? (uint32_t)__builtin_ctzll(diff) : 64u;
          if (diff) break;
        }
      }
      if (lane == (nseq & 63)) {
        run_src = lit0;
        run_len = pos - lit0;
        run_dst = nlit;
        sq[nseq] = seq_pack(pos - lit0, ml, off);
      }
      nlit += pos - lit0;
      ++nseq;
      if ((nseq & 63) == 0) flush_runs();
      cursor = pos + ml;
      lit0 = cursor;
      if (nseq == kZcSeqCap) {  // the rest of the block: literals
        stop = true;
        break;
      }
    }
    if (stop) break;
    if (m) {
      miss = 0;
      step = 1;
    } else if (++miss >= 4 && step < 8) {
      step *= 2;
      miss = 0;
    }
    s0 = cursor > s0 + span ? cursor : s0 + span;
  }
  if (nseq) {  // (no sequence: the block is stored raw from the input, nothing to stage)
    flush_runs();
    wave_copy(lit + nlit, p0 + lit0, end - lit0, lane);
    nlit += end - lit0;
  }
  if (lane == 0) {
    blocks[bi].nlit = nlit;
    blocks[bi].nseq = nseq;
  }
}

__global__ __launch_bounds__(256) void k_zc_encode(ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                   const uint64_t *seqs, ZTables T, uint64_t *piece) {
  MCDC_VGPR_PAD(64);  // (not an exact fill)
  __shared__ ZTables t;
  for (uint32_t k = threadIdx.x; k < sizeof(ZTables) / 4; k += blockDim.x)
    reinterpret_cast<uint32_t *>(&t)[k] = reinterpret_cast<const uint32_t *>(&T)[k];
  __syncthreads();
  const uint64_t bi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= nblk) {
    if (bi == nblk) piece[bi] = 0;
    return;
  }
  ZcBlock B = blocks[bi];
  uint32_t csize = 0;
  if (B.nseq) {
    uint8_t *st = stage + bi * kZcSlot;
    put_raw_lit_header(st, B.nlit);
    const uint32_t at = kLitHdr + B.nlit;
    // kept only if smaller than the raw block
    const uint32_t cap = B.len > at + 1 ? B.len - at - 1 : 0;
    const uint64_t *sq = seqs + bi * kZcSeqCap;
    const uint32_t ss = cap ? encode_sequences(t, [&](uint32_t i) { return sq[i]; }, B.nseq, st + at, cap) : 0;
    if (ss) csize = at + ss;
  }
  blocks[bi].csize = csize;
  piece[bi] = (B.b == 0 ? kFrameHdr : 0) + kBlockHdr + (csize ? csize : B.len);
}

__global__ __launch_bounds__(64) void k_zc_final(const uint8_t *base, const ZcBlock *blocks, uint64_t nblk,
                                                 const uint8_t *stage, const uint64_t *poff, const uint64_t *obase,
                                                 uint8_t *out, uint64_t *ext) {
  MCDC_VGPR_PAD(24);  // (not an exact fill)
  const uint64_t bi = blockIdx.x;
  if (bi >= nblk) return;
  const uint32_t lane = lane_id();
  const ZcBlock B = blocks[bi];
  const uint64_t o = *obase + poff[bi];
  uint8_t *d = out + o;
  if (B.b == 0) {
    if (lane < kFrameHdr) d[lane] = lane < 4 ? (uint8_t)(kMagic >> (8 * lane)) : lane == 4 ? kFhd : kWd;
    if (lane == 0) ext[2 * (uint64_t)B.chunk] = o;
    d += kFrameHdr;
  }
  const bool comp = B.csize != 0;
  const uint32_t size = comp ? B.csize : B.len;
  if (lane < kBlockHdr) {
    const uint32_t h = (B.b + 1 == B.nb ? 1u : 0u) | (comp ? 2u : 0u) << 1 | size << 3;
    d[lane] = (uint8_t)(h >> (8 * lane));
  }
  d += kBlockHdr;
  const uint8_t *s = comp ? stage + bi * kZcSlot : base + B.src;
  // bytes up to the output's 16-byte grid, then aligned 16-byte stores fed by
  // misaligned 16-byte loads (gfx950 reads them as the bytes at the address,
  // tools/dbg/unaligned_probe.hip), the tail byte by byte
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)d & 15)) & 15) < size ? (uint32_t)((16 - ((uintptr_t)d & 15)) & 15)
                                                                         : size;
  if (lane < head) d[lane] = s[lane];
  const uint32_t nq = (size - head) / 16;
  for (uint32_t k = lane; k < nq; k += 64)
    *reinterpret_cast<uint4 *>(d + head + 16 * k) = *reinterpret_cast<const uint4 *>(s + head + 16 * k);
  for (uint32_t k = head + 16 * nq + lane; k < size; k += 64) d[k] = s[k];
  if (B.b + 1 == B.nb && lane == 0) {
    const uint64_t first = bi - B.b;  // the chunk's first block is in the same batch
    const uint64_t fo = *obase + poff[first];
    ext[2 * (uint64_t)B.chunk + 1] = o + (B.b == 0 ? kFrameHdr : 0) + kBlockHdr + size - fo;
  }
}

__global__ void k_zc_advance(uint64_t *obase, const uint64_t *poff, uint64_t nblk) {
  MCDC_VGPR_PAD(8);  // (not an exact fill)
  if (threadIdx.x == 0 && blockIdx.x == 0) *obase += poff[nblk];
}

}  // namespace

size_t zc_tmp_bytes(uint64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n + 1);
  return b;
}

void launch_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint64_t *first,
                       uint32_t *err, uint64_t *bound, void *tmp, size_t tmp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(k_zc_nblocks, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, chunks, n, nbytes, cnt,
                     err, bound);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, cnt, first, (int)n + 1, st);
}

void launch_zc_batch(const uint8_t *base, const DevChunk *chunks, const uint64_t *first, uint64_t c0, uint64_t c1,
                     uint64_t b0, uint64_t nblk, ZcBlock *blocks, uint8_t *stage, uint64_t *seqs,
                     const zs::ZTables &T, uint64_t *piece, uint64_t *poff, uint64_t *obase, uint8_t *out,
                     uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st) {
  if (nblk == 0) return;
  hipLaunchKernelGGL(k_zc_blocks, dim3((unsigned)((c1 - c0 + 255) / 256)), dim3(256), 0, st, chunks, first, c0, c1,
                     b0, blocks);
  hipLaunchKernelGGL(k_zc_match, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, seqs);
  hipLaunchKernelGGL(k_zc_encode, dim3((unsigned)((nblk + 1 + 255) / 256)), dim3(256), 0, st, blocks, nblk, stage,
                     seqs, T, piece);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, piece, poff, (int)nblk + 1, st);
  hipLaunchKernelGGL(k_zc_final, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, poff, obase, out,
                     ext);
  hipLaunchKernelGGL(k_zc_advance, dim3(1), dim3(64), 0, st, obase, poff, nblk);
}

}  // namespace mcdc
