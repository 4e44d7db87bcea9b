// mcdc_zcomp.hip — CDNA4 (gfx950) zstd compression of every chunk of a
// boundary list, in HBM: SecureStorage::compress
// (/root/reference/src/repository/storage.rs:74-84) on the GPU, so the save
// path chunk -> IDs -> compress -> seal never leaves HBM.  One zstd frame per
// chunk (the blob mapache stores), in the crate's frame layout (magic, no
// content size, window 2^20, no checksum); blocks of 16 KiB, each either
// compressed (Huffman / RLE / raw literals + FSE sequences, predefined or per-block tables,
// mcdc_zstd.h) or raw when that is not smaller.  Decodes with mapache's decoder (storage.rs:87-94).
//
// Per batch of blocks (a block = 16 KiB of one chunk; batches bound the
// scratch):
//   k_zc_blocks  block records of the batch's chunks (chunk, index, source)
//   k_zc_match   ONE WAVE PER BLOCK: greedy LZ parse.  An 8192-entry hash
//                table in LDS (16-bit positions, colliding lanes resolved to
//                the largest, ht_put) is primed with the previous 16 KiB of
//                the same chunk (matches reach back up to 32 KiB); the wave
//                hashes 64 positions at once (every step-th position after
//                match-free strides), verifies and extends each lane's
//                candidate, then walks the lanes' matches greedily (ballot +
//                readlane, wave-uniform); long matches are extended 64 bytes
//                per step.  Literals go to the block's staging slot, sequences
//                (<= kZcSeqCap = 4096 per block, then the rest are literals) straight to
//                scratch (16 KiB of LDS per wave: 10 waves per CU).
//   k_zc_huff    ONE WAVE PER BLOCK: the block's literals (all of a block
//                without matches) as a Huffman-coded (or RLE) literals
//                section when smaller than raw: histogram in LDS, symbols
//                ranked by the wave, the length-limited canonical code by one
//                lane, then the streams (four above 1023 literals) by the
//                whole wave, bit positions from wave scans, assembled in LDS
//   k_zc_encode  ONE LANE PER BLOCK, 64 blocks per wave sharing one table
//                set: code histograms of the wave's blocks, per symbol type a
//                shared table or the predefined one (seq_plan), the shared
//                tables built by the wave in LDS; each block takes the shared
//                table of a type only when its own sequences cost less with
//                it (description included); then each lane writes its block's
//                serial FSE bitstream (three interleaved state machines);
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

// 8192 positions of 16 bits (16 KiB of LDS per wave: 10 waves per CU).
// Positions are relative to the block's priming window (< 32 KiB, + 1 so 0
// means empty), so 16 bits hold them; 4x the slots of the 32-bit 2048-entry
// table in the same LDS per CU keeps ~30 % more of the text's matches
// (tools/zc_model.cpp: literals 68 -> 35 % of the input).
#ifndef MCDC_ZC_HLOG
#define MCDC_ZC_HLOG 13  // (compile-time A/B knob)
#endif
constexpr uint32_t kHtLog = MCDC_ZC_HLOG, kHt = 1u << kHtLog;
static_assert(2 * kZcBlock <= 0xFFFF + 1, "16-bit positions");

__device__ __forceinline__ uint32_t ld4(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
// Hash of the 5 bytes at a position (4 in v, the fifth in b4): a 5-byte key
// keeps 4-byte coincidences out of the table (tools/zc_model.cpp: text
// 2.21 -> 2.25, CSV-like records 2.92 -> 3.05).
__device__ __forceinline__ uint32_t zhash(uint32_t v, uint32_t b4) {
  return (v * 2654435761u + (b4 & 0xFFu) * 0x85EBCA77u) >> (32 - kHtLog);
}
// Positions go into the table with plain 16-bit LDS stores (there is no
// 16-bit max atomic), so when lanes of one store collide on a slot the
// hardware keeps one of them; the slot must end at the largest (the latest
// position, as a max would keep it) so the parse does not depend on which.
// A store is read back after it has landed; lanes that see a smaller value
// store again (ht_fix), until none does.  The read-back is issued with the
// store and consumed later (priming: 8 strides at a time; the parse: at the
// top of the next stride), so its latency is off the critical path.  Later
// stores of larger positions only raise a slot, so a lane seeing a value >= its
// own is done.  Called by the whole wave (ballot).
// (relaxed workgroup-scope atomics: LDS loads and stores the compiler may not
// merge or forward -- a volatile generic pointer compiled to flat accesses)
__device__ __forceinline__ void ht_st(uint16_t *ht, uint32_t h, uint32_t v) {
  __hip_atomic_store(ht + h, (uint16_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t ht_ld(uint16_t *ht, uint32_t h) {
  return __hip_atomic_load(ht + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ht_fix(uint16_t *ht, uint32_t h, uint32_t v, bool ok, uint32_t rb) {
  bool again = ok && rb < v;
  while (__ballot(again)) {
    if (again) ht_st(ht, h, v);
    again = again && ht_ld(ht, h) < v;
  }
}
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
    z.nlit = z.nseq = z.csize = z.lsize = 0;
    blocks[f + b - b0] = z;
  }
}

// Copy bytes [a, a + n) of src to dst, the whole wave (64 lanes) together,
// four bytes per lane per round loaded before any is stored.
__device__ __forceinline__ void wave_copy(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint32_t n,
                                          uint32_t lane) {
  for (uint32_t k0 = 0; k0 < n; k0 += 256) {
    uint8_t b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = k0 + 64 * j + lane;
      b[j] = k < n ? src[k] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = k0 + 64 * j + lane;
      if (k < n) dst[k] = b[j];
    }
  }
}

// Length of the common prefix of two 32-byte strings (x at p, y at c).
__device__ __forceinline__ uint32_t match32_xor(uint4 x0, uint4 x1, uint4 y0, uint4 y1) {
  const uint32_t d[8] = {x0.x ^ y0.x, x0.y ^ y0.y, x0.z ^ y0.z, x0.w ^ y0.w,
                         x1.x ^ y1.x, x1.y ^ y1.y, x1.z ^ y1.z, x1.w ^ y1.w};
  uint32_t m = 32;
#pragma unroll
  for (int k = 7; k >= 0; --k)
    if (d[k]) m = 4 * k + ((uint32_t)__builtin_ctz(d[k]) >> 3);
  return m;
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

// One wave parses a run of up to kZcRun consecutive blocks of a chunk,
// keeping the table from block to block (the run's first block primes it
// with the previous 16 KiB, as every block did before runs: that re-hash was
// a large share of the parse).
// Lane i of a stride looks at position s0 + i * step.  step grows after
// match-free strides (1, 2, 4, 8: zstd's fast strategies skip ahead the same
// way on data that does not compress) and drops back to 1 at a match.
// Literal runs are copied 64 at a time: lane (k mod 64) keeps run k's source,
// length and destination, and the wave copies the 64 runs together.
__global__ __launch_bounds__(64) void k_zc_match(const uint8_t *base, ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                 uint64_t *seqs) {
  __shared__ __attribute__((aligned(16))) uint16_t ht[kHt];
  const uint64_t bi0 = blockIdx.x;
  if (bi0 >= nblk) return;
  const uint32_t lane = lane_id();
  ZcBlock B = blocks[bi0];
  if (B.b % kZcRun) return;  // (parsed by its run's first wave)
  // a run's blocks are consecutive records of the batch (a batch holds whole chunks)
  const uint32_t nrun = B.nb - B.b < kZcRun ? B.nb - B.b : kZcRun;
  for (uint32_t k = lane; k < kHt / 8; k += 64) reinterpret_cast<uint4 *>(ht)[k] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (uint32_t r = 0; r < nrun; ++r) {
  const uint64_t bi = bi0 + r;
  if (r) {
    // the table as the previous block's parse left it, its positions moved to
    // this block's frame (p0 advances by the previous block's prime: 0 after
    // a chunk's first block, else 16 KiB; positions before the new p0 drop)
    const uint32_t shift = B.b ? (uint32_t)kZcBlock : 0u;
    B = blocks[bi];
    if (shift) {
      for (uint32_t k = lane; k < kHt / 2; k += 64) {
        const uint32_t w = reinterpret_cast<uint32_t *>(ht)[k];
        const uint32_t lo = w & 0xFFFFu, hi = w >> 16;
        reinterpret_cast<uint32_t *>(ht)[k] = (lo > shift ? lo - shift : 0u) | (hi > shift ? hi - shift : 0u) << 16;
      }
    }
    __syncthreads();
  }
  const uint32_t prime = B.b ? kZcBlock : 0;  // the previous 16 KiB of the chunk
  const uint8_t *p0 = base + B.src - prime;   // positions are relative to p0
  const uint32_t end = prime + B.len;
  if (r == 0) {  // a run's first block: the table primed with the previous 16 KiB
    for (uint32_t q0 = 0; q0 < prime; q0 += 8 * 64) {  // (prime: 0 or 16 KiB, a multiple of 512)
      uint32_t h[8], rb[8];
      bool ok[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t q = q0 + 64 * j + lane;
        ok[j] = q + 4 <= prime;  // (the block's own bytes are not read here)
        h[j] = ok[j] ? zhash(ld4(p0 + q), p0[q + 4]) : 0u;  // (q + 4 <= prime: byte q + 4 is the block's own at worst)
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (ok[j]) ht_st(ht, h[j], q0 + 64 * j + lane + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) rb[j] = ht_ld(ht, h[j]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ht_fix(ht, h[j], q0 + 64 * j + lane + 1, ok[j], rb[j]);
    }
  }
  __syncthreads();
  uint8_t *lit = stage + bi * kZcSlot + kLitHdr;
  uint64_t *sq = seqs + bi * kZcSeqCap;
  uint32_t nlit = 0, nseq = 0, cursor = prime, lit0 = prime, step = 1, miss = 0;
  uint32_t run_src = 0, run_len = 0, run_dst = 0;  // this lane's pending literal run
  // 64 bytes of each lane's run per step: four 16-byte loads in flight, then
  // byte stores (a byte-at-a-time copy paid one memory round trip per byte:
  // the loads could not pass the stores to the possibly aliasing staging slot)
  auto flush_runs = [&]() {
    uint32_t mx = run_len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
    for (uint32_t k0 = 0; k0 < mx; k0 += 64) {
      uint4 w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t k = k0 + 16 * j;
        w[j] = make_uint4(0, 0, 0, 0);
        if (k < run_len) {
          if (run_src + k + 16 <= end) {
            w[j] = *reinterpret_cast<const uint4 *>(p0 + run_src + k);
          } else {  // (the block's last bytes: no read past them)
            uint32_t b[4] = {0, 0, 0, 0};
            for (uint32_t i = 0; i < 16 && run_src + k + i < end; ++i) b[i >> 2] |= (uint32_t)p0[run_src + k + i] << (8 * (i & 3));
            w[j] = make_uint4(b[0], b[1], b[2], b[3]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t k = k0 + 16 * j;
        if (k < run_len) {
          const uint32_t n = run_len - k < 16 ? run_len - k : 16;
          const uint32_t b[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
          uint8_t *d = lit + run_dst + k;
#pragma unroll
          for (uint32_t i = 0; i < 16; ++i)
            if (i < n) d[i] = (uint8_t)(b[i >> 2] >> (8 * (i & 3)));
        }
      }
    }
    run_len = 0;
  };
  uint32_t fh = 0, fv = 0, frb = 0;  // the previous stride's store, checked at the top of this one
  bool fok = false;
  for (uint32_t s0 = prime; s0 + 4 <= end;) {
    ht_fix(ht, fh, fv, fok, frb);
    const uint32_t p = s0 + lane * step;
    const bool ok = p + 4 <= end, full = p + 32 <= end;
    // this position's 32 bytes up front (they hold v), so a candidate costs one
    // more round trip (its 32 bytes), not two (4 bytes to verify, then 32)
    uint4 x0 = make_uint4(0, 0, 0, 0), x1 = x0;
    if (full) {
      x0 = *reinterpret_cast<const uint4 *>(p0 + p);
      x1 = *reinterpret_cast<const uint4 *>(p0 + p + 16);
    }
    const uint32_t v = full ? x0.x : ok ? ld4(p0 + p) : 0u;
    const uint32_t h = zhash(v, full ? x0.y : p + 5 <= end ? p0[p + 4] : 0u);
    const uint32_t cand = ok ? ht[h] : 0u;
    {  // (issued after every lane's read: one wave, in order)
      if (ok) ht_st(ht, h, p + 1);
      frb = ok ? ht_ld(ht, h) : 0u;
      fh = h;
      fv = p + 1;
      fok = ok;
    }
    uint32_t mlen = 0, c = 0;
    if (cand) {
      c = cand - 1;
      if (c < p && p - c < kWindow) {
        if (full) {
          const uint4 y0 = *reinterpret_cast<const uint4 *>(p0 + c), y1 = *reinterpret_cast<const uint4 *>(p0 + c + 16);
          mlen = match32_xor(x0, x1, y0, y1);
        } else if (ld4(p0 + c) == v) {
          mlen = match32(p0, p, c, end);
        }
      }
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
  ht_fix(ht, fh, fv, fok, frb);  // (the last stride's store: the next block reads the table)
  if (nseq) {  // (no sequence: the block is stored raw from the input, nothing to stage)
    flush_runs();
    wave_copy(lit + nlit, p0 + lit0, end - lit0, lane);
    nlit += end - lit0;
  }
  if (lane == 0) {
    blocks[bi].nlit = nlit;
    blocks[bi].nseq = nseq;
  }
  __syncthreads();
  }
}

// Inclusive sum over the wave's 64 lanes.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, d);
    if (lane >= d) v += t;
  }
  return v;
}

// The literals section of a compressed block: Huffman-coded or RLE when that
// is smaller than the raw section (3-byte header + the literals), written
// over the staging slot's raw literals; B.lsize its size, 0 = raw.  Literals
// >= 128 keep the raw section (the direct weight representation covers
// symbols 0..128; 128 itself is not worth the check).  The whole wave works
// on every step but the tree (one lane, ~2n dependent steps on LDS):
//   count    16 bytes per lane per step into 8 LDS histogram copies, leaving
//            at the first KiB that holds a byte >= 128 (random data: 1 KiB)
//   rank     symbols by count (ties by symbol), one rank per lane
//   tree     huf_build on the ranked symbols (lane 0)
//   sizes    bits per stream (wave sums); give up unless smaller than raw
//   streams  64 literals per round, last first: code lengths -> wave scan ->
//            bit positions -> codes OR-ed into the section assembled in LDS
//            (literal loads 8 rounds ahead)
//   store    header, tree, jump table; the section to the slot, 16-byte stores
__global__ __launch_bounds__(64) void k_zc_huff(const uint8_t *base, ZcBlock *blocks, uint64_t nblk, uint8_t *stage) {
  // the section under assembly; its first 8 KiB hold the histogram copies and
  // then the tree's scratch before it is cleared
  __shared__ __attribute__((aligned(16))) uint32_t out[kZcSlot / 4];
  __shared__ HufCT ct;
  uint32_t(*hist)[256] = reinterpret_cast<uint32_t(*)[256]>(out);
  HufWork &hw = *reinterpret_cast<HufWork *>(out + 8 * 256);
  static_assert(8 * 256 * 4 + sizeof(HufWork) <= sizeof(out), "LDS");
  const uint64_t bi = blockIdx.x;
  if (bi >= nblk) return;
  const uint32_t lane = lane_id();
  const ZcBlock B = blocks[bi];
  // a block without sequences: all of it literals, read from the input (k_zc_match staged nothing)
  const uint32_t n = B.nseq ? B.nlit : B.len;
  if (n < 32) return;  // (lsize stays 0: raw literals)
  uint8_t *st = stage + bi * kZcSlot;
  const uint8_t *src = B.nseq ? st + kLitHdr : base + B.src;
  for (uint32_t k = lane; k < 8 * 256; k += 64) out[k] = 0;
  __syncthreads();
  // count (misaligned 16-byte loads: gfx950 reads the bytes at the address)
  for (uint32_t k0 = 0; k0 < n; k0 += 1024) {
    const uint32_t k = k0 + 16 * lane;
    uint32_t w[4] = {0, 0, 0, 0}, m = 0;
    if (k + 16 <= n) {
      const uint4 v = *reinterpret_cast<const uint4 *>(src + k);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
      m = 16;
    } else if (k < n) {
      m = n - k;
#pragma unroll
      for (uint32_t j = 0; j < 16; ++j)
        if (j < m) w[j >> 2] |= (uint32_t)src[k + j] << (8 * (j & 3));
    }
    if (__ballot(((w[0] | w[1] | w[2] | w[3]) & 0x80808080u) != 0)) return;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
      if (j < m) atomicAdd(&hist[lane & 7][(w[j >> 2] >> (8 * (j & 3))) & 0x7F], 1u);
  }
  __syncthreads();
  uint32_t c[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t k = lane + 64 * h;
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) v += hist[j][k];
    c[h] = v;
  }
  __syncthreads();
  hist[0][lane] = c[0];
  hist[0][lane + 64] = c[1];
  if (lane == 0) hist[0][128] = 0;  // (huf_build reads 129 counts)
  // rank: symbols by count ascending, ties by symbol (huf_build's stable order)
  const uint64_t p0 = __ballot(c[0] != 0), p1 = __ballot(c[1] != 0);
  const uint32_t distinct = (uint32_t)(__builtin_popcountll(p0) + __builtin_popcountll(p1));
  if (distinct == 1) {  // RLE literals: 3-byte header + the byte
    if (lane == 0) {
      put_rle_lit_header(st, n);
      st[3] = (uint8_t)(p0 ? __builtin_ctzll(p0) : 64 + __builtin_ctzll(p1));
      blocks[bi].lsize = 4;
    }
    return;
  }
  __syncthreads();
  uint32_t r[2] = {0, 0};
  for (uint32_t t = 0; t < 128; t += 4) {
    const uint4 q = *reinterpret_cast<const uint4 *>(&hist[0][t]);  // (broadcast)
    const uint32_t qs[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        r[h] += (qs[j] && (qs[j] < c[h] || (qs[j] == c[h] && t + j < lane + 64 * h))) ? 1u : 0u;
  }
  if (c[0]) hw.sym[r[0]] = (uint16_t)lane;
  if (c[1]) hw.sym[r[1]] = (uint16_t)(lane + 64);
  __syncthreads();
  if (lane == 0) huf_build(hist[0], ct, hw, true);
  __syncthreads();
  // bits per stream (stream k: literals [k seg, min((k + 1) seg, n)))
  const bool one = n < 1024;
  const uint32_t seg = one ? n : (n + 3) / 4, ns = one ? 1 : 4;
  uint32_t sb[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < ns; ++k) {
    const uint32_t a = k * seg, e = min(a + seg, n);
    uint32_t b = 0;
#pragma unroll 8
    for (uint32_t i = a + lane; i < e; i += 64) b += ct.nb[src[i]];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += (uint32_t)__shfl_xor((int)b, d);
    sb[k] = b;
  }
  uint32_t ssz[4];
  const uint32_t total = huf_section_size(ct, n, sb, one, ssz);
  if (total >= kLitHdr + n) return;  // not smaller than raw
  const uint32_t tree = 1 + (ct.last + 1) / 2;
  const uint32_t csize = tree + (one ? 0 : 6) + ssz[0] + (one ? 0 : ssz[1] + ssz[2] + ssz[3]);
  if (one && csize >= 1024) return;  // (one stream: 10-bit sizes)
  const uint32_t hdr = lit_hdr_size(n, csize, one);
  const uint32_t nq = (total + 15) / 16;  // 16-byte units of the section
  for (uint32_t k = lane; k < nq; k += 64) reinterpret_cast<uint4 *>(out)[k] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  // the streams
  uint32_t o = hdr + tree + (one ? 0 : 6);  // byte offset of stream k in the section
  for (uint32_t k = 0; k < ns; ++k) {
    const uint32_t a = k * seg, e = min(a + seg, n), len = e - a;
    uint32_t carry = 8 * o;  // bit position of the next round's first literal
    for (uint32_t r0 = 0; r0 < len; r0 += 8 * 64) {
      uint32_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t q = r0 + 64 * j + lane;
        x[j] = q < len ? (uint32_t)src[e - 1 - q] : 0x100u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (r0 + 64 * j >= len) break;
        const uint32_t nb = x[j] < 0x100u ? ct.nb[x[j]] : 0u;
        const uint32_t incl = wave_incl_sum(nb, lane);
        const uint32_t pos = carry + incl - nb;
        if (nb) {
          const uint32_t code = ct.code[x[j]], sft = pos & 31;
          atomicOr(&out[pos >> 5], code << sft);
          if (sft + nb > 32) atomicOr(&out[(pos >> 5) + 1], code >> (32 - sft));
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
    }
    if (lane == 0) atomicOr(&out[carry >> 5], 1u << (carry & 31));  // the end mark
    o += ssz[k];
  }
  __syncthreads();
  if (lane == 0) {
    uint8_t *sec = reinterpret_cast<uint8_t *>(out);
    put_huf_lit_header(sec, n, csize, one);
    huf_tree_desc(ct, sec + hdr);
    if (!one)
      for (int k = 0; k < 3; ++k) {
        sec[hdr + tree + 2 * k] = (uint8_t)ssz[k];
        sec[hdr + tree + 2 * k + 1] = (uint8_t)(ssz[k] >> 8);
      }
    blocks[bi].lsize = total;
  }
  __syncthreads();
  // (every read of the staged literals is done: the section replaces them)
  for (uint32_t k = lane; k < nq; k += 64) reinterpret_cast<uint4 *>(st)[k] = reinterpret_cast<const uint4 *>(out)[k];
}

// Modular inverse of an odd a modulo 2^32 (Newton: each step doubles the bits).
__device__ __forceinline__ uint32_t inv_odd(uint32_t a) {
  uint32_t x = a;  // correct to 3 bits
#pragma unroll
  for (int k = 0; k < 4; ++k) x *= 2u - a * x;
  return x;
}

// fse_build (mcdc_zstd.h) of a distribution without "less than 1" entries,
// by the whole wave: the spread puts the j-th symbol occurrence (symbols in
// order, norm[s] each) at position j * step mod size, so position u holds the
// symbol whose cumulative range holds j = u * step^-1; a symbol's states are
// its positions in ascending order, ranked 64 positions per round with a
// same-symbol ballot mask.  cum / seen: LDS scratch of 54 entries.
__device__ void fse_build_wave(const int16_t *norm, uint32_t tl, FseCTL &ct, uint32_t *cum, uint32_t *seen,
                               uint32_t lane) {
  const uint32_t size = 1u << tl, mask = size - 1;
  const int32_t n = lane < 53 ? norm[lane] : 0;
  const uint32_t incl = wave_incl_sum((uint32_t)n, lane), ex = incl - (uint32_t)n;
  if (lane < 53) {
    cum[lane] = ex;
    seen[lane] = 0;
    if (n == 0) {
      ct.dnb[lane] = ((tl + 1) << 16) - size;
      ct.dfs[lane] = 0;
    } else if (n == 1) {
      ct.dnb[lane] = (tl << 16) - size;
      ct.dfs[lane] = (int32_t)ex - 1;
    } else {
      const uint32_t mb = tl - highbit((uint32_t)n - 1);
      ct.dnb[lane] = (mb << 16) - ((uint32_t)n << mb);
      ct.dfs[lane] = (int32_t)ex - n;
    }
  }
  if (lane == 53) cum[53] = size;
  if (lane == 0) ct.log = tl;
  __syncthreads();
  const uint32_t inv = inv_odd((size >> 1) + (size >> 3) + 3) & mask;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t u0 = 0; u0 < size; u0 += 64) {
    const uint32_t u = u0 + lane;
    const bool act = u < size;  // (size 32: half the wave)
    const uint32_t j = (u * inv) & mask;
    uint32_t lo = 0, hi = 53;  // cum[lo] <= j < cum[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cum[mid] <= j) lo = mid;
      else hi = mid;
    }
    uint64_t m = __ballot(act);
#pragma unroll
    for (int bt = 0; bt < 6; ++bt) {
      const uint64_t v = __ballot((lo >> bt) & 1);
      m &= ((lo >> bt) & 1) ? v : ~v;
    }
    const uint32_t base = seen[lo];
    __syncthreads();
    if (act) {
      ct.state[cum[lo] + base + (uint32_t)__builtin_popcountll(m & lt)] = (uint16_t)(size + u);
      if ((m >> lane) == 1ull) seen[lo] = base + (uint32_t)__builtin_popcountll(m);  // the group's last lane
    }
    __syncthreads();
  }
}

// One lane per block, 64 blocks per wave sharing one set of tables (a
// block's own tables would not fit 64 times in LDS, and one wave per block
// leaves the serial bitstream 64x less parallel):
//   plan     code histograms over the wave's blocks with 64 or more
//            sequences; seq_plan (lane 0) picks per symbol type the shared
//            table or the predefined one, pricing the descriptions once per
//            block; the shared tables built by the wave, the predefined
//            ones copied beside them, bits per code of both in LDS
//   choose   each block prices its own sequences under both and takes the
//            shared table for a type only if that is smaller with its
//            description
//   encode   each lane writes its block's serial FSE bitstream (three
//            interleaved state machines); block kept compressed only if
//            smaller than raw
constexpr uint32_t kEncOwnMin = 64;  // sequences for a block to consider the shared tables

__global__ __launch_bounds__(64) void k_zc_encode(ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                  const uint64_t *seqs, ZTables T, uint64_t *piece) {
  MCDC_VGPR_PAD(40);  // (not an exact fill)
  __shared__ FseCTL t[3], pt[3];  // shared (own) and predefined tables
  __shared__ SeqPlan P;
  __shared__ float bits[2][3][53];  // bits per code: [shared / predefined][LL, OF, ML][code]
  __shared__ uint32_t hist[3][53], cum[54], seen[54];
  const uint32_t lane = lane_id();
  const uint64_t bi = (uint64_t)blockIdx.x * 64 + lane;
  const bool valid = bi < nblk;
  if (bi == nblk) piece[nblk] = 0;
  ZcBlock B{};
  if (valid) B = blocks[bi];
  const uint32_t ns = B.nseq;
  const uint64_t *sq = seqs + bi * kZcSeqCap;
  const FseCT *pre[3] = {&T.ll, &T.of, &T.ml};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pt[k].state[lane] = pre[k]->state[lane];
    if (lane < 53) {
      pt[k].dfs[lane] = pre[k]->dfs[lane];
      pt[k].dnb[lane] = pre[k]->dnb[lane];
      hist[k][lane] = 0;
    }
    if (lane == 0) pt[k].log = pre[k]->log;
  }
  __syncthreads();
  const bool cand = ns >= kEncOwnMin;
  if (cand)
    for (uint32_t i = 0; i < ns; ++i) {
      const uint64_t q = sq[i];
      atomicAdd(&hist[0][ll_code(seq_ll(q))], 1u);
      atomicAdd(&hist[1][highbit(seq_off(q) + 3)], 1u);
      atomicAdd(&hist[2][ml_code(seq_ml(q) - 3)], 1u);
    }
  const uint32_t ncand = (uint32_t)__builtin_popcountll(__ballot(cand));
  uint32_t total = cand ? ns : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) total += (uint32_t)__shfl_xor((int)total, d);
  __syncthreads();
  if (lane == 0) seq_plan(hist[0], hist[1], hist[2], total, P, ncand ? ncand : 1);
  __syncthreads();
  const int16_t *pnorm[3] = {kLLNorm, kOFNorm, kMLNorm};
  const uint32_t npre[3] = {36, 29, 53};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (P.own[k]) fse_build_wave(P.norm[k], P.tl[k], t[k], cum, seen, lane);
    if (lane < 53) {
      const int32_t n = P.own[k] ? P.norm[k][lane] : 0;
      bits[0][k][lane] = n > 0 ? (float)P.tl[k] - log2f((float)n) : 1e9f;
      const int32_t m = lane < npre[k] ? (pnorm[k][lane] == -1 ? 1 : pnorm[k][lane]) : 0;
      bits[1][k][lane] = m > 0 ? (float)pt[k].log - log2f((float)m) : 1e9f;
    }
  }
  __syncthreads();
  uint32_t modes = 0;
  if (cand && (P.own[0] | P.own[1] | P.own[2])) {
    float c0[3] = {0, 0, 0}, c1[3] = {0, 0, 0};
    for (uint32_t i = 0; i < ns; ++i) {
      const uint64_t q = sq[i];
      const uint32_t code[3] = {ll_code(seq_ll(q)), highbit(seq_off(q) + 3), ml_code(seq_ml(q) - 3)};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        c0[k] += bits[0][k][code[k]];
        c1[k] += bits[1][k][code[k]];
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (P.own[k] && c0[k] + 8.0f * (float)P.dlen[k] < c1[k]) modes |= 2u << (6 - 2 * k);
  }
  uint32_t csize = 0;
  if (valid && (ns || B.lsize)) {  // (no sequences but a Huffman / RLE section: a literals-only block)
    uint8_t *st = stage + bi * kZcSlot;
    if (!B.lsize) put_raw_lit_header(st, B.nlit);
    const uint32_t at = B.lsize ? B.lsize : kLitHdr + B.nlit;  // (Huffman / RLE section written by k_zc_huff)
    const uint32_t cap = B.len > at + 1 ? B.len - at - 1 : 0;
    const FseCTL &tll = (modes >> 6) & 3 ? t[0] : pt[0];
    const FseCTL &tof = (modes >> 4) & 3 ? t[1] : pt[1];
    const FseCTL &tml = (modes >> 2) & 3 ? t[2] : pt[2];
    const uint32_t ss = cap ? encode_sequences_with(tll, tof, tml, modes, P.desc, P.doff, P.dlen,
                                                    [&](uint32_t i) { return sq[i]; }, ns, st + at, cap)
                            : 0;
    if (ss) csize = at + ss;
  }
  if (valid) {
    blocks[bi].csize = csize;
    piece[bi] = (B.b == 0 ? kFrameHdr : 0) + kBlockHdr + (csize ? csize : B.len);
  }
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
                     uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st, bool huf) {
  if (nblk == 0) return;
  hipLaunchKernelGGL(k_zc_blocks, dim3((unsigned)((c1 - c0 + 255) / 256)), dim3(256), 0, st, chunks, first, c0, c1,
                     b0, blocks);
  hipLaunchKernelGGL(k_zc_match, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, seqs);
  if (huf) hipLaunchKernelGGL(k_zc_huff, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage);
  hipLaunchKernelGGL(k_zc_encode, dim3((unsigned)((nblk + 1 + 63) / 64)), dim3(64), 0, st, blocks, nblk, stage, seqs,
                     T, piece);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, piece, poff, (int)nblk + 1, st);
  hipLaunchKernelGGL(k_zc_final, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, poff, obase, out,
                     ext);
  hipLaunchKernelGGL(k_zc_advance, dim3(1), dim3(64), 0, st, obase, poff, nblk);
}

}  // namespace mcdc
