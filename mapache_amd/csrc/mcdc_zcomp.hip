// mcdc_zcomp.hip — CDNA4 (gfx950) zstd compression of every chunk of a
// boundary list, in HBM: SecureStorage::compress
// (/root/reference/src/repository/storage.rs:74-84) on the GPU, so the save
// path chunk -> IDs -> compress -> seal never leaves HBM.  One zstd frame per
// chunk (the blob mapache stores), in the crate's frame layout (magic, no
// content size, window 2^20, no checksum); blocks of 16 KiB, each either
// compressed (Huffman / RLE / raw literals + predefined-FSE sequences,
// mcdc_zstd.h) or raw when that is not smaller.  Decodes with mapache's decoder (storage.rs:87-94).
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
//   k_zc_huff    ONE WAVE PER BLOCK: the block's literals (all of a block
//                without matches) as a Huffman-coded (or RLE) literals
//                section when smaller than raw: histogram in LDS, symbols
//                ranked by the wave, the length-limited canonical code by one
//                lane, then the streams (four above 1023 literals) by the
//                whole wave, bit positions from wave scans, assembled in LDS
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
    z.nlit = z.nseq = z.csize = z.lsize = 0;
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
  if (B.nseq || B.lsize) {  // (no sequences but a Huffman / RLE section: a literals-only block)
    uint8_t *st = stage + bi * kZcSlot;
    if (!B.lsize) put_raw_lit_header(st, B.nlit);
    const uint32_t at = B.lsize ? B.lsize : kLitHdr + B.nlit;  // (Huffman / RLE section written by k_zc_huff)
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
                     uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st, bool huf) {
  if (nblk == 0) return;
  hipLaunchKernelGGL(k_zc_blocks, dim3((unsigned)((c1 - c0 + 255) / 256)), dim3(256), 0, st, chunks, first, c0, c1,
                     b0, blocks);
  hipLaunchKernelGGL(k_zc_match, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, seqs);
  if (huf) hipLaunchKernelGGL(k_zc_huff, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage);
  hipLaunchKernelGGL(k_zc_encode, dim3((unsigned)((nblk + 1 + 255) / 256)), dim3(256), 0, st, blocks, nblk, stage,
                     seqs, T, piece);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, piece, poff, (int)nblk + 1, st);
  hipLaunchKernelGGL(k_zc_final, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, poff, obase, out,
                     ext);
  hipLaunchKernelGGL(k_zc_advance, dim3(1), dim3(64), 0, st, obase, poff, nblk);
}

}  // namespace mcdc
