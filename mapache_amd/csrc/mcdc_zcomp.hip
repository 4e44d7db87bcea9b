// mcdc_zcomp.hip — CDNA4 (gfx950) zstd compression of every chunk of a
// boundary list, in HBM: SecureStorage::compress
// (/root/reference/src/repository/storage.rs:74-84) on the GPU, so the save
// path chunk -> IDs -> compress -> seal never leaves HBM.  One zstd frame per
// chunk (the blob mapache stores), in the crate's frame layout (magic, no
// content size, window 2^20, no checksum); blocks of 32 KiB, each either
// compressed (Huffman / RLE / raw literals + FSE sequences, predefined or per-block tables,
// mcdc_zstd.h) or raw when that is not smaller.  Decodes with mapache's decoder (storage.rs:87-94).
//
// Per batch of blocks (a block = 32 KiB of one chunk; batches of whole chunks
// bound the scratch, mcdc_zcomp.h):
//   k_zc_blocks  block records of the batch's chunks (chunk, index, source)
//   k_zc_segorder the finder segments and the parse blocks, longest first
//   k_zc_probe   ONE WORKGROUP (16 waves) PER SEGMENT: order-0 entropy of each
//                block (a sample) and, for high-entropy blocks, a repeat test
//                over content-defined anchors: hopeless blocks (random,
//                compressed, encrypted data) are stored raw, every later
//                kernel skips them; the segment's far anchors into its far
//                table (chunks longer than a segment)
//   k_zc_far     (rescue) a hopeless block with a far match is not hopeless
//   k_zc_find    ONE WORKGROUP (16 waves, 1024 threads) PER SEGMENT of up to
//                8 blocks of a chunk: candidate matches for every position.
//                Two LDS tables (160 KiB: 2^15 slots for a 5-byte key and
//                2^13 for an 8-byte key, as zstd's double-fast pair) of
//                32-bit entries: a segment-relative position and a 13-bit tag
//                of the key.  Filled 1024 positions at a time: a tile reads
//                the tables as the earlier tiles left them, then inserts its
//                own positions with LDS max atomics (the latest position per
//                slot, deterministically).  One candidate per position, the
//                long key's when its tag matches, else the short key's,
//                verified on 16 bytes two tiles later (its loads in flight
//                meanwhile); per position one word (match length <= 16 << 24
//                | offset, 0 = none) to scratch.  A segment after a chunk's
//                first re-inserts the 64 KiB before it.
//   k_zc_far     far matches: anchors of a chunk's later segments look up the
//                latest anchors of the 5 segments before (the 2^20 window),
//                verified, extended backwards, written into the words
//   k_zc_parse   ONE WAVE PER BLOCK: the greedy parse over the words, 256
//                positions per window without a serial walk: capped matches
//                (16 verified bytes) get their true lengths per run of one
//                repeat (its last position extended, one per lane from a
//                ranked list, the end handed back by pointer jumping); the
//                chain from the cursor by pointer doubling (lane m composes
//                J over the bits of m); a match longer than 48 bytes on the
//                chain extended 2 KiB per wave step and the chain continued
//                from its end; match and literal indices by ballot ranks,
//                literal lengths and repeat code 1 from the match ranked
//                before; literals to the block's staging slot, sequences to
//                scratch
//   k_zc_huff    ONE WAVE PER BLOCK: the block's literals (all of a block
//                without matches) as a Huffman-coded (or RLE) literals
//                section when smaller than raw: histogram of the 256 byte
//                values in LDS, symbols ranked by the wave, the
//                length-limited canonical code and its description (direct
//                or FSE-compressed weights) by one lane, then the streams
//                (four above 1023 literals) by the whole wave in lane pieces
//   k_zc_plan    ONE WAVE PER BLOCK: per symbol type the block's own FSE
//   k_zc_chain   table or the predefined one (seq_plan); the three state
//   k_zc_encode  machines of 9 blocks per wave, two lanes each (their bits to
//                scratch); then every sequence's bits placed by the block's
//                wave; the block kept compressed only if smaller than raw
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

// Match finder tables in LDS: 2^15 slots for a 5-byte key and 2^13 for an
// 8-byte key (zstd's double-fast pair), 32-bit entries (position << 13 | tag,
// 0 = empty): 160 KiB, the whole of a CU's LDS.  Inserts are LDS max atomics,
// so a slot ends at the latest position whichever lane's atomic lands last.
// tools/zc_model2.cpp priced the choices on the bench's corpora (16/64/256
// KiB chunks; text / records / binary): one 2^14 table 2.44 / 3.20 / 1.74;
// 2^15 + 2^13 2.59 / 3.30 / 1.78; zstd level 3 2.68 / 3.23 / 1.78.  Tiles of
// 512 positions cost ~1 % on records and binary against exact most-recent
// insertion.
#ifndef MCDC_ZC_HS
#define MCDC_ZC_HS 15  // (compile-time A/B knobs)
#endif
#ifndef MCDC_ZC_HL
#define MCDC_ZC_HL 13
#endif
constexpr uint32_t kHsLog = MCDC_ZC_HS, kHlLog = MCDC_ZC_HL;
#ifndef MCDC_ZC_FT
#define MCDC_ZC_FT 1024  // (compile-time A/B knob)
#endif
#ifndef MCDC_ZC_DEPTH
#define MCDC_ZC_DEPTH 2  // (compile-time A/B knob: tiles of loads in flight in k_zc_find; 4 measured no faster)
#endif
constexpr uint32_t kFindThreads = MCDC_ZC_FT;  // threads per workgroup (16 waves)
constexpr uint32_t kMlCap = 16;               // match bytes verified per candidate (longer: k_zc_parse extends)
constexpr uint32_t kPrime = kZcPrime;         // bytes before a segment re-inserted (farther: k_zc_far)
// Match words: length (<= kMlCap) << 24 | offset; bit 31 marks a verified
// kMlCap match of the finder's own (readers take the length as (w >> 24) & 31)
constexpr uint32_t kZcLocalCap = 1u << 31;
// Per-block scratch, packed by the blocks' lengths (mcdc_zcomp.h): block bi
// of a batch owns words[B.w0, + zc_span(len)) -- a chunk's blocks are
// consecutive, so its words are contiguous, position p of the chunk at
// chunk base + p -- the staging slot stage[B.w0 + 64 bi, + span + 64) and
// kZcExtra bytes of extra[].  The words are the match words until
// k_zc_parse, which writes the block's sequences over them as it goes
// (sequence i, 8 bytes at 8 i, is written in the window of a position >= 4 i,
// after that window's words were read, and every word read later lies at 4 x
// a later position: never overtaken); the upper half then holds k_zc_huff's
// section under assembly, then k_zc_chain's state records (blocks of 512
// words or more; shorter ones keep them in extra[]).
__device__ __forceinline__ uint32_t blk_span(uint32_t len) { return (uint32_t)zc_span(len); }
__device__ __forceinline__ uint64_t *blk_seqs(uint32_t *words, const ZcBlock &B) {
  return reinterpret_cast<uint64_t *>(words + B.w0);
}
__device__ __forceinline__ uint32_t *blk_upper(uint32_t *words, const ZcBlock &B) {
  return words + B.w0 + blk_span(B.len) / 2;
}
__device__ __forceinline__ uint8_t *blk_slot(uint8_t *stage, const ZcBlock &B, uint64_t bi) {
  return stage + B.w0 + 64 * bi;
}
// (a chunk's position p: word chunk_words(...)[p]; B any of its blocks)
__device__ __forceinline__ uint32_t *chunk_words(uint32_t *words, const ZcBlock &B) {
  return words + (B.w0 - B.b * (uint32_t)kZcBlock);
}
static_assert(kZcBlock % 64 == 0, "a chunk's full blocks span whole 64-word steps: its words are contiguous");
// The parse's run ends (ends[]): kEndNext = take the next position's,
// kEndLong = still matching kRunExt bytes after kMlCap (the wave extends it)
constexpr uint32_t kRunExt = 32, kEndNext = 0xFFFFu, kEndLong = 0xFFFEu;

// Keys hashed with 24-bit multiplies (full rate; a 32-bit multiply issues at
// a quarter of it): the key cut into 24- and 16-bit pieces, each multiplied by
// an odd 24-bit constant, the low 32 bits of the products mixed; the index is
// the top bits, which every bit of a piece reaches.
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t k) { return (uint32_t)__umul24(a, k); }  // (HIP's returns int)
// The index is the top bits of the mixed value, the 13-bit tag the bits
// below them (kHsLog + 13 <= 32): one mix per key for both.
__device__ __forceinline__ uint32_t mix5(uint32_t lo, uint32_t hi) {
  const uint32_t a = lo & 0xFFFFFFu, b = lo >> 24 | (hi & 0xFFu) << 8;
  return mul24(a, 0x9E3779u) + mul24(b, 0xC2B2AFu);
}
__device__ __forceinline__ uint32_t mix8(uint32_t lo, uint32_t hi) {
  const uint32_t a = lo & 0xFFFFFFu, b = lo >> 24 | (hi & 0xFFFFu) << 8, c = hi >> 16;
  return mul24(a, 0x85EBCBu) ^ mul24(b, 0x27D4EBu) ^ mul24(c, 0x165667u);
}
static_assert(kHsLog + 13 <= 32 && kHlLog + 13 <= 32, "index and tag bits of one mixed value");
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// A workgroup barrier that orders LDS only: __syncthreads' workgroup fence
// waits for every outstanding global load too (vmcnt(0) on gfx9), which
// would drain the match finder's prefetches at each of its per-tile barriers.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Within one wave LDS operations complete in issue order: a wave-sized tile
// only has to keep the compiler from moving its table reads and inserts across
// each other.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
template <uint32_t NT>
__device__ __forceinline__ void tile_sync() {
  if constexpr (NT > 64) lds_sync();
  else wave_lds_order();
}

__global__ void k_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint64_t *wcnt,
                             uint32_t *err, uint64_t *bound, uint8_t *cls) {
  MCDC_VGPR_PAD(12);  // (not an exact fill)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t raw = 0;
  if (i < n) {
    const DevChunk c = chunks[i];
    const bool ok = c.offset <= nbytes && c.length <= nbytes - c.offset && c.length < (1ull << 31);
    if (!ok) atomicOr(err, 1u);
    const uint64_t nb = c.length ? (c.length + kZcBlock - 1) / kZcBlock : 1;
    cnt[i] = nb;
    wcnt[i] = zc_span(c.length);  // (= the sum of its blocks' spans: full blocks span kZcBlock)
    cls[i] = nb == 1 ? (uint8_t)zc_small_class(c.length) : (uint8_t)4;
    raw = kFrameHdr + kBlockHdr * nb + c.length;
  } else if (i == n) {
    cnt[i] = 0;
    wcnt[i] = 0;
  }
  for (int o = 32; o > 0; o >>= 1) raw += __shfl_down(raw, o);
  if (lane_id() == 0 && raw) atomicAdd(reinterpret_cast<unsigned long long *>(bound), (unsigned long long)raw);
}

__global__ void k_zc_blocks(const DevChunk *chunks, const uint64_t *first, const uint64_t *wfirst, uint64_t c0,
                            uint64_t c1, uint64_t b0, ZcBlock *blocks) {
  MCDC_VGPR_PAD(16);  // (not an exact fill)
  const uint64_t c = c0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= c1) return;
  const DevChunk ch = chunks[c];
  const uint64_t f = first[c], nb = first[c + 1] - f;
  const uint32_t w = (uint32_t)(wfirst[c] - wfirst[c0]);  // (the chunk's first word in the batch)
  for (uint64_t b = 0; b < nb; ++b) {
    ZcBlock z;
    z.src = ch.offset + b * kZcBlock;
    z.len = (uint32_t)(ch.length - b * kZcBlock < kZcBlock ? ch.length - b * kZcBlock : kZcBlock);
    z.chunk = (uint32_t)c;
    z.b = (uint32_t)b;
    z.nb = (uint32_t)nb;
    z.nlit = z.nseq = z.csize = z.lsize = z.flags = 0;
    z.w0 = w + (uint32_t)b * (uint32_t)kZcBlock;
    blocks[f + b - b0] = z;
  }
}

// A finder segment's cost in 4 KiB steps (its blocks plus the re-inserted
// bytes), with the chunks of one block (<= 32 KiB, no re-inserted bytes) at
// (len - 1) / 4096 = 0 .. 7 and every other segment at 8 or more, so that a
// descending sort puts the small chunks (k_zc_small) after the others, their
// size classes (kZcSmallClass) in contiguous ranges.
__device__ __forceinline__ uint32_t seg_cost(const ZcBlock *blocks, const ZcBlock &B, uint64_t r) {
  if (B.nb == 1) return B.len ? (B.len - 1) / 4096 : 0u;
  const uint32_t nsb = min<uint32_t>(kZcSegBlocks, B.nb - B.b);
  const uint32_t bytes = (nsb - 1) * kZcBlock + blocks[r + nsb - 1].len + (B.b ? kPrime : 0u);
  return max(bytes / 4096, 8u);
}

// The finder's segments by cost, longest first: a segment's blocks (<=
// kZcSegBlocks) plus, after a chunk's first segment, the kPrime bytes it
// re-inserts, by 4 KiB; order[i] = the record starting the i-th
// segment, then nblk (no segment).  And the blocks for k_zc_parse, longest
// first by 4 KiB steps: porder[i] = the i-th block.  One workgroup: counting
// sorts in LDS (the order within a bucket follows the atomics; it changes no
// output).
__global__ __launch_bounds__(1024) void k_zc_segorder(const ZcBlock *blocks, uint64_t nblk, uint32_t *order,
                                                      uint32_t *porder) {
  constexpr uint32_t kKeys = (kZcSegBlocks * kZcBlock + kPrime) / 4096 + 1;
  constexpr uint32_t kPKeys = kZcBlock / 4096 + 1;
  __shared__ uint32_t cnt[kKeys], at[kKeys], pcnt[kPKeys], pat[kPKeys];
  MCDC_VGPR_PAD(24);  // (not an exact fill)
  const uint32_t tid = threadIdx.x;
  if (tid < kKeys) cnt[tid] = 0;
  if (tid < kPKeys) pcnt[tid] = 0;
  __syncthreads();
  auto key = [&](const ZcBlock &B, uint64_t r) {  // (descending cost by 4 KiB: bucket 0 = the costliest)
    return kKeys - 1 - min(kKeys - 1, seg_cost(blocks, B, r));
  };
  auto pkey = [&](const ZcBlock &B) { return kPKeys - 1 - min<uint32_t>(kPKeys - 1, B.len / 4096); };
  for (uint64_t r = tid; r < nblk; r += 1024) {
    const ZcBlock B = blocks[r];
    if (B.b % kZcSegBlocks == 0) atomicAdd(&cnt[key(B, r)], 1u);
    atomicAdd(&pcnt[pkey(B)], 1u);
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t a = 0;
    for (uint32_t k = 0; k < kKeys; ++k) {
      at[k] = a;
      a += cnt[k];
    }
    cnt[0] = a;  // (the number of segments)
    a = 0;
    for (uint32_t k = 0; k < kPKeys; ++k) {
      pat[k] = a;
      a += pcnt[k];
    }
  }
  __syncthreads();
  const uint32_t nseg = cnt[0];
  for (uint64_t r = tid; r < nblk; r += 1024) {
    const ZcBlock B = blocks[r];
    if (B.b % kZcSegBlocks == 0) order[atomicAdd(&at[key(B, r)], 1u)] = (uint32_t)r;
    porder[atomicAdd(&pat[pkey(B)], 1u)] = (uint32_t)r;
  }
  for (uint64_t i = nseg + tid; i < nblk; i += 1024) order[i] = (uint32_t)nblk;
}

// Branch-free 16-byte load for prefetching (a branch around a load makes the
// compiler wait for it where the paths join): the 16 bytes at p, or, within
// 16 bytes of the end of the nbytes >= 16 readable, the last 16 bytes; fix16
// then realigns them (bytes past the end zero) where they are used.
__device__ __forceinline__ uint4 ld16c(const uint8_t *base, uint64_t p, uint64_t nbytes) {
  return *reinterpret_cast<const uint4 *>(base + (p + 16 <= nbytes ? p : nbytes - 16));
}
__device__ __forceinline__ uint4 fix16(uint4 x, uint64_t p, uint64_t nbytes) {
  // (selects only: a branch here would make the compiler wait for every load at its join)
  const uint32_t sh = p + 16 <= nbytes ? 0u : p >= nbytes ? 16u : (uint32_t)(p - (nbytes - 16));  // bytes to drop
  const uint64_t lo = (uint64_t)x.y << 32 | x.x, hi = (uint64_t)x.w << 32 | x.z;
  const uint32_t b = 8 * (sh & 7);
  const uint64_t lo1 = b ? (lo >> b | hi << (64 - b)) : lo, hi1 = hi >> b;  // shifted by sh % 8 bytes
  const uint64_t rlo = sh >= 16 ? 0 : sh >= 8 ? hi1 : lo1, rhi = sh >= 8 ? 0 : hi1;
  return make_uint4((uint32_t)rlo, (uint32_t)(rlo >> 32), (uint32_t)rhi, (uint32_t)(rhi >> 32));
}

// Loads the compiler's wait-count pass does not see (ald16s and the inline
// loads of the parse, Huffman and chain kernels).  On gfx9 one counter
// (vmcnt) covers loads and stores, and with a store pending the pass treats
// the counter as out of order and waits for zero before any use of a load:
// a loop that stores a result per step and prefetches two steps ahead gets
// every prefetch drained at the next step.  These kernels issue such loads
// themselves and wait with explicit s_waitcnt (counting only their own loads
// where the count is exact: loads return in order, a store may retire
// early), each wait taking the loaded registers as operands so that no use
// is scheduled before it; devaudit checks no such register is read early.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 to4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
// 16 bytes at sbase + off (a uniform base and a 32-bit offset: no 64-bit address math)
__device__ __forceinline__ u32x4 ald16s(const uint8_t *sbase, uint32_t off) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(v) : "v"(off), "s"(sbase) : "memory");
  return v;
}
__device__ __forceinline__ void ast32s(uint32_t *sbase, uint32_t off, uint32_t v) {
  asm volatile("global_store_dword %0, %1, %2" ::"v"(off), "v"(v), "s"(sbase) : "memory");
}

// Common prefix of two 16-byte strings, branch-free: the first differing bit
// of each dword (v_ffbl: ~0 for none), offset by the dword's position with
// clamping adds (~0 stays ~0), the minimum / 8 (the ctz-per-half form was
// compiled to divergent branches, both sides run in a mixed wave).
__device__ __forceinline__ uint32_t ffbl32(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t prefix16(uint4 x, uint4 y) {
  const uint32_t b0 = ffbl32(x.x ^ y.x);
  const uint32_t b1 = __builtin_elementwise_add_sat(ffbl32(x.y ^ y.y), 32u);
  const uint32_t b2 = __builtin_elementwise_add_sat(ffbl32(x.z ^ y.z), 64u);
  const uint32_t b3 = __builtin_elementwise_add_sat(ffbl32(x.w ^ y.w), 96u);
  return min(min(min(b0, b1), min(b2, b3)), 128u) >> 3;
}

// The match finder: one workgroup of NT threads per segment (up to
// kZcSegBlocks blocks of one chunk, the first record of the segment's blocks:
// other workgroups return).  Writes words[(block - batch start) * kZcBlock +
// position in block] for every position of the segment: match length (<=
// kMlCap) << 24 | offset, 0 = no match of 4 bytes or more.  Table entries
// are (position - prime0 + 1) << 13 | a 13-bit tag of the key (0 = empty),
// so a lookup knows whether the stored key is (almost surely) its own, and
// each position verifies ONE candidate: the long table's when its tag
// matches, else the short table's when that one does (tools/zc_model2.cpp:
// no ratio change against verifying both).  Per tile: the lookups (tables as
// the earlier tiles left them), the candidate's bytes requested, the tile
// two back verified (its bytes had two tiles' time to arrive), then the
// inserts; two LDS-only barriers per tile.
//
// Workgroups take the segments longest first (order[], k_zc_segorder): one
// workgroup fills a CU (its tables are the whole LDS), and a segment of 8
// blocks that started last would run on alone at the end of the launch.
template <uint32_t NT, uint32_t HS, uint32_t HL>
__global__ __launch_bounds__(NT) void k_zc_find_t(const uint8_t *base, uint64_t nbytes, const ZcBlock *blocks,
                                                  uint64_t nblk, uint32_t *words, const uint32_t *order) {
  static_assert(NT % 64 == 0 && HS + 13 <= 32 && HL + 13 <= 32, "tile and tables");
  constexpr uint32_t kFindTile = NT;  // positions per step
  constexpr uint32_t kDepth = MCDC_ZC_DEPTH;  // tiles of loads in flight (2 or 4)
  static_assert(kDepth == 2 || kDepth == 4, "finder pipeline depth");
  __shared__ __attribute__((aligned(16))) uint32_t hts[1u << HS], htl[1u << HL];
  const uint64_t bi0 = order[blockIdx.x];
  if (bi0 >= nblk) return;
  const ZcBlock B0 = blocks[bi0];
  if (B0.b % kZcSegBlocks) return;
  const uint32_t tid = threadIdx.x;
  // chunk geometry (a batch holds whole chunks: the chunk's last block is a record of this batch)
  const uint64_t csrc = B0.src - (uint64_t)B0.b * kZcBlock;
  const uint32_t clen = (B0.nb - 1) * (uint32_t)kZcBlock + blocks[bi0 + (B0.nb - 1 - B0.b)].len;
  const uint32_t seg0 = B0.b * (uint32_t)kZcBlock;
  const uint32_t seg1 = min(clen, seg0 + kZcSegBlocks * (uint32_t)kZcBlock);
  const uint32_t prime0 = seg0 > kPrime ? seg0 - kPrime : 0u;
  static_assert(kPrime + kZcSegBlocks * kZcBlock < (1u << 19), "entry positions take 19 bits");
  const uint8_t *cb = base + csrc;
  const uint64_t cbytes = nbytes - csrc;  // (bytes readable from the chunk start)
  // the segment's words: the chunk's blocks are consecutive records, so
  // position p's word is wseg[p]; positions outside the segment keep nothing
  uint32_t *wseg = chunk_words(words, B0);
  // (word stores: a 32-bit offset from the segment's first word; from the
  // chunk's, 4 p wraps for chunks of 1 GiB or more)
  uint32_t *const wseg0 = wseg + seg0;
  {  // a segment whose blocks k_zc_probe found hopeless: nothing to find
    bool all_raw = true;
    for (uint32_t k = 0; k * (uint32_t)kZcBlock < seg1 - seg0; ++k) all_raw &= (blocks[bi0 + k].flags & kZcRaw) != 0;
    if (all_raw) return;
  }
  if (clen < 16 || cbytes < 16) {  // (too short to match: every position a literal)
    for (uint32_t p = seg0 + tid; p < seg1; p += NT) wseg[p] = 0u;
    return;
  }
  for (uint32_t k = tid; k < (1u << HS) / 4; k += NT) reinterpret_cast<uint4 *>(hts)[k] = make_uint4(0, 0, 0, 0);
  for (uint32_t k = tid; k < (1u << HL) / 4; k += NT) reinterpret_cast<uint4 *>(htl)[k] = make_uint4(0, 0, 0, 0);
  // 16-byte loads at chunk offsets clamped to the last 16 readable bytes; a
  // tile within 16 bytes of the end realigns them (fix16), others use them as loaded
  const uint32_t last16 = (uint32_t)min<uint64_t>(cbytes - 16, 0xFFFFFFF0ull);
  // tiles from here: the tail (32-bit: a uniform compare stays on the scalar unit; positions are < 2^31)
  const uint32_t tail0 = (uint32_t)min<uint64_t>(cbytes >= kFindTile + 16 ? cbytes - (kFindTile + 16) : 0, 0xFFFFFFFFull);
  // Two tiles in flight: a tile's own bytes are requested two tiles ahead,
  // and its candidate's bytes are verified two tiles later (the counter
  // retires in order, so waiting for a tile's own bytes leaves the newer
  // requests in flight)
  struct Stage {
    bool v, k, tail;
    uint32_t p, q;
    uint4 x;
    u32x4 y;
  };
  // (kDepth tiles in flight: stage k holds tile t - kDepth + k; a tile's own
  // bytes are requested kDepth tiles ahead, its candidate's verified kDepth
  // tiles later)
  Stage s0{}, s1{}, s2{}, s3{};
  u32x4 n0 = ald16s(cb, min(prime0 + tid, last16)), n1 = ald16s(cb, min(prime0 + kFindTile + tid, last16));
  u32x4 n2 = {0, 0, 0, 0}, n3 = {0, 0, 0, 0};  // (unused at depth 2; never a copy of a pending load)
  if constexpr (kDepth == 4) {
    n2 = ald16s(cb, min(prime0 + 2 * kFindTile + tid, last16));
    n3 = ald16s(cb, min(prime0 + 3 * kFindTile + tid, last16));
  }
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)::"memory");
  auto verify = [&](const Stage &S) {
    const uint32_t bend = min(clen, (S.p / (uint32_t)kZcBlock + 1) * (uint32_t)kZcBlock);
    const uint32_t lim = S.p < bend ? min(kMlCap, bend - S.p) : 0u;
    uint4 y = to4(S.y);
    if (S.tail) y = fix16(y, S.q, cbytes);
    const uint32_t m = S.k ? min(prefix16(S.x, y), lim) : 0u;
    // (a full kMlCap match carries kZcLocalCap: k_zc_far's atomicMax keeps it)
    if (S.v)
      ast32s(wseg0, 4 * (S.p - seg0),
             m >= zs::kMinMatch ? (m << 24 | (S.p - S.q) | (m == kMlCap ? kZcLocalCap : 0u)) : 0u);
  };
#ifdef MCDC_ZC_TIMING  // (A/B: cycles per phase of wave 0 in some workgroups, printed)
  uint64_t tm[5] = {0, 0, 0, 0, 0}, tstart = __builtin_amdgcn_s_memtime(), tnow = 0;
  uint32_t nsteps = 0;
#define ZC_TICK(k) (tnow = __builtin_amdgcn_s_memtime(), tm[k] += tnow - tstart, tstart = tnow)
#else
#define ZC_TICK(k) ((void)0)
#endif
  // one tile; n: its own bytes on entry, the bytes of the tile kDepth ahead
  // on exit; S: the tile kDepth back on entry (verified here), this tile on
  // exit.  The loop below rotates kDepth (n, S) sets, so no register with a
  // pending load is ever copied.  Per step the memory operations are: the
  // verified word's store (or none), then the loads y (every lane: a lane
  // without a candidate reads its own position, so the count is fixed) and
  // n; a step's loads are used kDepth steps later, after the 2 (kDepth - 1)
  // loads of the steps between (a pending store only makes the wait longer).
  auto step = [&](uint32_t t0, u32x4 &n, Stage &S) {
    ZC_TICK(4);
    if constexpr (kDepth == 4) asm volatile("s_waitcnt vmcnt(6)" : "+v"(n), "+v"(S.y)::"memory");
    else asm volatile("s_waitcnt vmcnt(2)" : "+v"(n), "+v"(S.y)::"memory");
    ZC_TICK(0);
    const uint32_t p = t0 + tid;
    const bool tail = t0 >= tail0;
    uint4 x = to4(n);
    if (tail) x = fix16(x, p, cbytes);
    const bool find = t0 >= seg0 && p < seg1;  // (prime tiles only insert; tiles past the segment: nothing kept)
    const bool vs = p + 5 <= clen, vl = p + 8 <= clen;
    const uint32_t m5 = mix5(x.x, x.y), m8 = mix8(x.x, x.y);
    const uint32_t hs = m5 >> (32 - HS), hl = m8 >> (32 - HL);
    const uint32_t gs = (m5 >> (32 - HS - 13)) & 0x1FFFu, gl = (m8 >> (32 - HL - 13)) & 0x1FFFu;
    // (both slots read by every lane, the result masked: no exec-mask branch
    // around the LDS reads; a slot index is always in range)
    const uint32_t rs = hts[hs], rl = htl[hl];
    const uint32_t es = find && vs ? rs : 0u, el = find && vl ? rl : 0u;
    verify(S);
    ZC_TICK(1);
    // the candidate: the long key's if its tag matches, else the short key's
    const uint32_t cl = prime0 + (el >> 13) - 1, cs = prime0 + (es >> 13) - 1;
#ifdef MCDC_ZC_NOBAR
    const bool okl = el != 0 && (el & 0x1FFFu) == gl && cl < p && p - cl <= zs::kWindow;
    const bool oks = es != 0 && (es & 0x1FFFu) == gs && cs < p && p - cs <= zs::kWindow;
#else
    // (an entry is an earlier tile's position of this segment or the
    // re-inserted bytes: less than 2^20 back, no window test needed)
    const bool okl = el != 0 && (el & 0x1FFFu) == gl;
    const bool oks = es != 0 && (es & 0x1FFFu) == gs;
#endif
    const uint32_t q = okl ? cl : oks ? cs : p;
    S.v = find;
    S.k = okl || oks;
    S.tail = tail;
    S.p = p;
    S.q = q;
    S.x = x;
#if defined(MCDC_ZC_NOGATHER)  // (A/B timing only: no candidate gathers, every position a literal)
    S.k = false;
    S.y = ald16s(cb, min(p, last16));
#else
    S.y = ald16s(cb, min(q, last16));
#endif
    n = ald16s(cb, min(p + kDepth * kFindTile, last16));
    const uint32_t r = (p - prime0 + 1) << 13;
#ifndef MCDC_ZC_NOBAR  // (A/B timing only: no barriers, racy lookups)
    tile_sync<NT>();  // every lookup of the tile before any insert
#endif
    ZC_TICK(2);
#ifndef MCDC_ZC_NOINS  // (A/B timing only: no inserts, no candidates)
    if (vs) atomicMax(hts + hs, r | gs);
    if (vl) atomicMax(htl + hl, r | gl);
#endif
#ifndef MCDC_ZC_NOBAR
    tile_sync<NT>();  // every insert before the next tile's lookups
#endif
    ZC_TICK(3);
#ifdef MCDC_ZC_TIMING
    ++nsteps;
#endif
  };
  if constexpr (NT > 64) __syncthreads();
  else wave_lds_order();  // (the cleared tables before the first lookups)
  // (both steps unconditional: a tile past the segment keeps nothing, and a
  // join after a conditional step would cost the compiler's own waits)
  for (uint32_t t0 = prime0; t0 < seg1; t0 += kDepth * kFindTile) {
    step(t0, n0, s0);
    step(t0 + kFindTile, n1, s1);
    if constexpr (kDepth == 4) {
      step(t0 + 2 * kFindTile, n2, s2);
      step(t0 + 3 * kFindTile, n3, s3);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3), "+v"(s0.y), "+v"(s1.y), "+v"(s2.y),
               "+v"(s3.y)::"memory");
  verify(s0);
  verify(s1);
  if constexpr (kDepth == 4) {
    verify(s2);
    verify(s3);
  }
#ifdef MCDC_ZC_TIMING
  if (tid == 0 && bi0 % 509 == 0)
    printf("ZCT wg %lu steps %u wait %lu calc %lu bar1 %lu bar2 %lu loop %lu\n", (unsigned long)bi0, nsteps,
           (unsigned long)tm[0], (unsigned long)tm[1], (unsigned long)tm[2], (unsigned long)tm[3], (unsigned long)tm[4]);
#endif
}


// The match finder over the segments of the batch (k_zc_find_t above): the
// 1024-thread form with the full tables for chunks of more than one block.
#define MCDC_ZC_FIND_BIG k_zc_find_t<kFindThreads, kHsLog, kHlLog>
// ---- the probe and the far matches --------------------------------------
// Anchors: positions whose 8-byte key mixes (mix8) to a value with its top
// bits clear, so that a repeated stretch has anchors at the same places in
// both copies.  Slots from the mix's next bits, 13-bit tags from the 5-byte
// key's mix (mix5).  Near anchors (1 position in 32) feed k_zc_probe's repeat
// test, far anchors (1 in 128, a subset) the far tables of k_zc_far.
constexpr uint32_t kNearLog = 14;
__device__ __forceinline__ bool far_anchor(uint32_t m8) { return m8 < (1u << 25); }
__device__ __forceinline__ uint32_t far_slot(uint32_t m8) { return (m8 >> 13) & (kZcSegBlocks * kZcFarSlots - 1u); }
__device__ __forceinline__ uint32_t anchor_tag(uint32_t m5) { return m5 >> 19; }
// The probe's near anchors (high-entropy blocks only, where no byte pattern
// dominates): 1 position in 32 by one 24-bit product of bytes 0..2 (two
// VALU), the slot from its next bits, the tag from a product of bytes 4..6;
// a hit is verified on the 8 bytes.
__device__ __forceinline__ uint32_t near_mix(uint32_t lo) { return mul24(lo & 0xFFFFFFu, 0x9E3779u); }
__device__ __forceinline__ bool near_anchor(uint32_t nm) { return nm < (1u << 27); }
__device__ __forceinline__ uint32_t near_slot(uint32_t nm) { return (nm >> 13) & ((1u << kNearLog) - 1u); }
__device__ __forceinline__ uint32_t near_tag(uint32_t hi) { return mul24(hi & 0xFFFFFFu, 0xC2B2AFu) >> 19; }
static_assert(kZcSegBlocks * kZcFarSlots == 4096, "far slots: bits 13..24 of a far anchor's mix");
// Bits per byte (order 0) at or above which a block without repeats is stored
// raw: Huffman coding could save at most (8 - 7.9) / 8 of it, less its table.
constexpr float kRawEntropy = 7.9f;
constexpr uint32_t kProbeThreads = 1024, kProbeTile = 16 * kProbeThreads;
static_assert(kPrime % kProbeTile == 0 && kZcBlock % kProbeTile == 0, "probe tiles start at segments and blocks");
constexpr uint32_t kFarBack = 256;  // bytes a far match is extended backwards
constexpr uint32_t kFarStride = 4;  // positions between the far words written over a backward extension

// bytes j .. j + 3 of the words w (little endian)
__device__ __forceinline__ uint32_t byte_window(const uint32_t *w, int j) {
  return (j & 3) ? __builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], (uint32_t)(j & 3)) : w[j >> 2];
}
// equal bytes at the end of two 16-byte strings
__device__ __forceinline__ uint32_t suffix16(uint4 x, uint4 y) {
  const uint64_t d0 = (uint64_t)(x.y ^ y.y) << 32 | (x.x ^ y.x), d1 = (uint64_t)(x.w ^ y.w) << 32 | (x.z ^ y.z);
  return d1 ? (uint32_t)__builtin_clzll(d1) >> 3 : d0 ? 8u + ((uint32_t)__builtin_clzll(d0) >> 3) : 16u;
}

// The probe: one workgroup per finder segment (the segments longest first,
// as k_zc_find).  Pass 1 over the segment: a byte histogram of each of its
// blocks (4 of every 16 bytes: an 8 KiB sample, whose plug-in entropy of
// uniform bytes is 7.98 bits; a chunk's last block under 16 KiB whole, the
// threshold lowered by the smaller sample's bias); in a chunk of more than one segment, its far
// anchors into its far table (latest per slot, built in LDS -- repeated keys
// would serialise on one L2 address -- and stored to HBM; not for a chunk's
// last segment: no later segment reads it) and their ballots (a bit per 16
// positions, a word per 1024) for k_zc_far.  Only if a block carries
// kRawEntropy bits per byte or more: pass 2 over the re-inserted bytes and
// the segment up to the last such block, every near anchor into an LDS table
// (earliest per slot) tile by tile; such a block is hopeless if none of its
// near anchors finds an earlier anchor with the same 8 bytes -- kZcRaw,
// stored raw without the finder, the parse or the entropy coders (random,
// compressed or encrypted data).  k_zc_far's rescue mode then clears kZcRaw
// of a block with a far match.
__global__ __launch_bounds__(kProbeThreads) void k_zc_probe(const uint8_t *base, uint64_t nbytes, ZcBlock *blocks,
                                                            uint64_t nblk, const uint32_t *order, uint32_t *ftab,
                                                            uint64_t *fbits) {
  __shared__ uint32_t tab[1u << kNearLog];  // pass 1: the far table (its first slots); passes 2, 3: the near table
  __shared__ uint32_t hist[kZcSegBlocks][256];
  __shared__ uint32_t rep[kZcSegBlocks], high[kZcSegBlocks], nsmp[kZcSegBlocks];
  static_assert(kZcSegBlocks * kZcFarSlots <= (1u << kNearLog), "the far table fits the near table's place");
  MCDC_VGPR_PAD(32);  // (not an exact fill)
  const uint64_t bi0 = order[blockIdx.x];
  if (bi0 >= nblk) return;
  const ZcBlock B0 = blocks[bi0];
  if (B0.b % kZcSegBlocks) return;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / 64;
  const uint64_t csrc = B0.src - (uint64_t)B0.b * kZcBlock;
  const uint32_t clen = (B0.nb - 1) * (uint32_t)kZcBlock + blocks[bi0 + (B0.nb - 1 - B0.b)].len;
  const uint32_t seg0 = B0.b * (uint32_t)kZcBlock;
  const uint32_t seg1 = min(clen, seg0 + kZcSegBlocks * (uint32_t)kZcBlock);
  const uint32_t prime0 = seg0 > kPrime ? seg0 - kPrime : 0u;
  const uint32_t nsb = (seg1 - seg0 + (uint32_t)kZcBlock - 1) / (uint32_t)kZcBlock;
  const bool far_out = seg1 < clen;  // a later segment reads this one's far table
  const bool far_in = seg0 > 0;      // k_zc_far reads this segment's ballots
  const uint8_t *cb = base + csrc;
  const uint64_t cbytes = nbytes - csrc;
  if (clen < 16 || cbytes < 16) return;  // (flags stay 0)
  for (uint32_t k = tid; k < kZcSegBlocks * 256; k += kProbeThreads) (&hist[0][0])[k] = 0;
  if (tid < kZcSegBlocks) rep[tid] = high[tid] = 0;
  if (far_out)
    for (uint32_t k = tid; k < kZcSegBlocks * kZcFarSlots; k += kProbeThreads) tab[k] = 0;
  __syncthreads();
  auto load6 = [&](uint32_t p, uint32_t(&w)[6]) {  // bytes p .. p + 23 (zero past the buffer)
    const uint4 a = fix16(ld16c(cb, p, cbytes), p, cbytes), b = fix16(ld16c(cb, p + 16, cbytes), p + 16, cbytes);
    w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w, w[4] = b.x, w[5] = b.y;
  };
  const bool hash1 = far_out || far_in;
  for (uint32_t t0 = seg0; t0 < seg1; t0 += kProbeTile) {
    const uint32_t p = t0 + 16 * tid;
    uint32_t fm = 0;
    if (p < seg1) {
      uint32_t w[6];
      if (hash1) {
        load6(p, w);
      } else {
        const uint4 a = fix16(ld16c(cb, p, cbytes), p, cbytes);
        w[0] = a.x;
      }
      const uint32_t hb = (p - seg0) >> 15;
      // (a chunk's last block shorter than 16 KiB is counted whole: its
      // sample would be too small to tell random bytes from others)
      const bool whole = seg1 - (seg0 + (hb << 15)) < 16384u;
      if (whole && !hash1) {
        const uint4 a = fix16(ld16c(cb, p, cbytes), p, cbytes);
        w[1] = a.y, w[2] = a.z, w[3] = a.w;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((j < 4 || whole) && p + j < seg1) atomicAdd(&hist[hb][(w[j >> 2] >> (8 * (j & 3))) & 0xFFu], 1u);
      if (hash1) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t q = p + j;
          if (q >= seg1 || q + 8 > clen) continue;
          const uint32_t lo = byte_window(w, j), hi = byte_window(w, j + 4), m8 = mix8(lo, hi);
          if (!far_anchor(m8)) continue;
          fm |= 1u << j;
          // (q - seg0 + 1 takes 18 bits: the segment's very last position, 2^18, is not inserted)
          if (far_out && q - seg0 + 1 < (1u << 18)) atomicMax(&tab[far_slot(m8)], (q - seg0 + 1) << 14 | anchor_tag(mix5(lo, hi)));
        }
      }
    }
    if (far_in) {  // (uniform)
      const uint64_t bal = __ballot(fm != 0);
      const uint32_t qw = t0 + 1024 * wv;
      if (lane == 0 && qw < seg1) fbits[(bi0 - B0.b) * kZcFarBallots + qw / 1024] = bal;
    }
  }
  __syncthreads();
  if (far_out) {
    uint32_t *ft = ftab + bi0 * kZcFarSlots;
    for (uint32_t k = tid; k < kZcSegBlocks * kZcFarSlots; k += kProbeThreads) ft[k] = tab[k];
  }
  if (wv < nsb) {  // order-0 entropy of block wv's sample: n log2 n - sum c log2 c >= kRawEntropy n
    float sc = 0.f;
    uint32_t n = 0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint32_t c = hist[wv][lane + 64 * h];
      sc += c ? (float)c * __log2f((float)c) : 0.f;
      n += c;
    }
    for (int o = 32; o > 0; o >>= 1) {
      sc += __shfl_xor(sc, o);
      n += __shfl_xor(n, o);
    }
    // (the threshold less the plug-in estimate's bias for n samples beyond an
    // 8 KiB sample's, (K - 1) / (2 n ln 2) with K = 256 values: the same
    // margin below uniform bytes at every sample size)
    const float thr = kRawEntropy - 183.9f / (float)max(n, 1u) + 183.9f / 8192.f;
    if (lane == 0) {
      high[wv] = n >= 512 && (float)n * __log2f((float)n) - sc >= thr * (float)n ? 1u : 0u;
      nsmp[wv] = n;
    }
  }
  __syncthreads();
  // (a chunk's last block too short to judge, under 512 bytes, follows the
  // block before it: it would otherwise keep a random segment alive alone)
  if (tid == 0 && nsb > 1 && nsmp[nsb - 1] < 512 && high[nsb - 2]) high[nsb - 1] = 1;
  __syncthreads();
  uint32_t hend = 0;  // the end of the last high-entropy block
  for (uint32_t k = 0; k < nsb; ++k)
    if (high[k]) hend = min(seg1, seg0 + (k + 1) * (uint32_t)kZcBlock);
  if (!hend) return;
  for (uint32_t k = tid; k < (1u << kNearLog); k += kProbeThreads) tab[k] = 0xFFFFFFFFu;
  __syncthreads();
  // one pass, tile by tile: a tile's near anchors into the table (earliest
  // per slot), barrier, then each anchor of a high-entropy block looks for an
  // earlier anchor with its key among the tiles so far (a later tile's
  // inserts only ever fill empty slots with later positions: no second
  // barrier)
  for (uint32_t t0 = prime0; t0 < hend; t0 += kProbeTile) {
    const uint32_t p = t0 + 16 * tid;
    uint32_t w[6] = {0, 0, 0, 0, 0, 0}, am = 0;
    if (p < hend) {
      load6(p, w);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t q = p + j, nm = near_mix(byte_window(w, j));
        if (near_anchor(nm) && q < hend && q + 8 <= clen) {
          am |= 1u << j;
          atomicMin(&tab[near_slot(nm)], (q - prime0 + 1) << 13 | near_tag(byte_window(w, j + 4)));
        }
      }
    }
    __syncthreads();
    if (am && p >= seg0 && high[(p - seg0) >> 15]) {
      bool hit = false;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (!((am >> j) & 1)) continue;
        const uint32_t q = p + j, lo = byte_window(w, j), hi = byte_window(w, j + 4);
        const uint32_t e = tab[near_slot(near_mix(lo))];
        const uint32_t c = prime0 + (e >> 13) - 1;
        if ((e & 0x1FFFu) == near_tag(hi) && c < q) {  // (rare: verify the 8 bytes)
          const uint2 y = *reinterpret_cast<const uint2 *>(cb + c);  // (c + 8 < q + 8 <= clen)
          hit |= y.x == lo && y.y == hi;
        }
      }
      if (hit) rep[(p - seg0) >> 15] = 1;  // (any writer sets it)
    }
  }
  __syncthreads();
  bool all = true;
  for (uint32_t k = 0; k < nsb; ++k) all &= high[k] && !rep[k];
  if (tid < nsb && high[tid] && !rep[tid]) blocks[bi0 + tid].flags = kZcRaw | (tid == 0 && all ? kZcSegRaw : 0u);
}

// The small chunks: every chunk of one block (<= DMAX bytes, the size class
// kZcSmallClass) probed and matched by one workgroup of W waves, with the
// chunk's bytes and its tables in LDS -- k_zc_find's 1024-thread tiles over
// global loads are latency-bound on a chunk of a few KiB (two tiles of loads
// in flight, a CU per chunk), and lose the matches inside a tile.  Here:
//   1. the chunk's bytes into LDS (every load issued at once) and their
//      order-0 histogram (a chunk under 16 KiB whole, else 4 of every 16
//      bytes), in the table space;
//   2. its entropy as k_zc_probe's test (kRawEntropy, the same bias term);
//   3. the match finder over LDS: tiles of 64 W positions (the tables as the
//      earlier tiles left them, then the tile's inserts, LDS max atomics:
//      the latest position per slot), tables of 2^HS / 2^HL 32-bit entries
//      sized to the class (zstd too shrinks its tables to a small source;
//      tools/zc_model4.cpp priced the classes: 97-98 % of level 3 on the
//      kernel-tree files, 94.5 % with k_zc_find), each position's candidate
//      verified on 16 bytes from LDS;
//   4. a chunk of high entropy without a verified match of 8 bytes or more is
//      hopeless (kZcRaw, as k_zc_probe's repeat test), stored raw.
// LDS: the bytes (DMAX) then the tables: exactly 160 KiB / (the class's
// workgroups per CU).
template <uint32_t W, uint32_t HS, uint32_t HL, uint32_t DMAX>
__global__ __launch_bounds__(64 * W) void k_zc_small(const uint8_t *base, uint64_t nbytes, ZcBlock *blocks,
                                                     uint64_t nblk, uint32_t *words, const uint32_t *order) {
  constexpr uint32_t NT = 64 * W;
  static_assert(DMAX % 16 == 0 && (1u << HS) >= 256 && HS + 13 <= 32 && HL + 13 <= 32, "class shape");
  // (one array: the bytes first, so that the reads past a chunk's end land in the tables)
  __shared__ __attribute__((aligned(16))) uint32_t lds[DMAX / 4 + (1u << HS) + (1u << HL)];
  uint32_t *const dat = lds, *const hts = lds + DMAX / 4, *const htl = hts + (1u << HS);
  MCDC_VGPR_PAD(40);  // (not an exact fill)
  const uint64_t bi = order[blockIdx.x];
  if (bi >= nblk) return;
  const ZcBlock B = blocks[bi];
  const uint32_t tid = threadIdx.x, lane = lane_id(), L = B.len;
  if (B.nb != 1 || L > DMAX) return;  // (not this class: the host's counts disagree)
  const uint8_t *cb = base + B.src;
  const uint64_t cbytes = nbytes - B.src;
  uint32_t *const wc = words + B.w0;
  if (L < 16 || cbytes < 16) {  // (too short to match: every position a literal; flags stay 0)
    for (uint32_t p = tid; p < L; p += NT) wc[p] = 0u;
    return;
  }
#ifdef MCDC_ZC_TIMING  // (A/B: clocks per phase of thread 0, some workgroups, printed)
  uint64_t tq[5], tq0 = __builtin_amdgcn_s_memtime();
#define ZQ(k) (tq[k] = __builtin_amdgcn_s_memtime())
#else
#define ZQ(k) ((void)0)
#endif
  // 1. the bytes (16-byte loads at chunk offsets: misaligned global loads;
  // the last 16 readable bytes realigned) and the histogram
  uint32_t *const hist = hts;  // (256 words, cleared with the tables below)
  for (uint32_t k = tid; k < 256; k += NT) hist[k] = 0u;
  const uint32_t nq = (L + 15) / 16;
  constexpr uint32_t kQ = DMAX / 16 / NT;  // quads per thread
  static_assert(kQ * NT * 16 == DMAX, "quads per thread");
  uint4 q[kQ];
#pragma unroll
  for (uint32_t j = 0; j < kQ; ++j) {
    const uint32_t k = tid + j * NT;
    q[j] = k < nq ? fix16(ld16c(cb, 16 * k, cbytes), 16 * k, cbytes) : make_uint4(0, 0, 0, 0);
  }
  tile_sync<NT>();  // (the histogram cleared)
  const bool whole = L < 16384;
#pragma unroll
  for (uint32_t j = 0; j < kQ; ++j) {
    const uint32_t k = tid + j * NT;
    if (k < nq) {
      reinterpret_cast<uint4 *>(dat)[k] = q[j];
      const uint32_t w4[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
      for (int b = 0; b < 16; ++b)
        if ((b < 4 || whole) && 16 * k + b < L) atomicAdd(&hist[(w4[b >> 2] >> (8 * (b & 3))) & 0xFFu], 1u);
    }
  }
  ZQ(0);
  // 2. entropy (wave 0; thread 0 keeps the answer): n log2 n - sum c log2 c
  // >= thr n, thr as k_zc_probe's
  tile_sync<NT>();
  bool high = false;
  if (tid < 64) {
    float sc = 0.f;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint32_t c = hist[lane + 64 * h];
      sc += c ? (float)c * __log2f((float)c) : 0.f;
    }
    for (int o = 32; o > 0; o >>= 1) sc += __shfl_xor(sc, o);
    const uint32_t n = whole ? L : 4 * (L / 16) + min(4u, L % 16);  // (the bytes counted)
    const float thr = kRawEntropy - 183.9f / (float)max(n, 1u) + 183.9f / 8192.f;
    high = n >= 512 && (float)n * __log2f((float)n) - sc >= thr * (float)n;
  }
  tile_sync<NT>();
  ZQ(1);
  for (uint32_t k = tid; k < ((1u << HS) + (1u << HL)) / 4; k += NT) reinterpret_cast<uint4 *>(hts)[k] = make_uint4(0, 0, 0, 0);
  tile_sync<NT>();
  ZQ(2);
  // 3. the finder, NT positions per tile
  auto bytes16 = [&](uint32_t p) {  // chunk bytes p .. p + 15 from LDS (past L: anything)
    const uint32_t i = p >> 2, sh = p & 3;
    const uint32_t d0 = dat[i], d1 = dat[i + 1], d2 = dat[i + 2], d3 = dat[i + 3], d4 = dat[i + 4];
    return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                      __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
  };
  bool rep = false;
  for (uint32_t t0 = 0; t0 < L; t0 += NT) {
    const uint32_t p = t0 + tid;
    const uint4 x = bytes16(min(p, L - 1));
    const bool vs = p + 5 <= L, vl = p + 8 <= L;
    const uint32_t m5 = mix5(x.x, x.y), m8 = mix8(x.x, x.y);
    const uint32_t hs = m5 >> (32 - HS), hl = m8 >> (32 - HL);
    const uint32_t gs = (m5 >> (32 - HS - 13)) & 0x1FFFu, gl = (m8 >> (32 - HL - 13)) & 0x1FFFu;
    const uint32_t es = vs ? hts[hs] : 0u, el = vl ? htl[hl] : 0u;
    const bool okl = el != 0 && (el & 0x1FFFu) == gl, oks = es != 0 && (es & 0x1FFFu) == gs;
    const uint32_t c = okl ? (el >> 13) - 1 : oks ? (es >> 13) - 1 : p;
    const uint4 y = bytes16(min(c, L - 1));
    const uint32_t lim = p < L ? min(kMlCap, L - p) : 0u;
    const uint32_t m = (okl || oks) ? min(prefix16(x, y), lim) : 0u;
    rep |= m >= 8;
    if (p < L) wc[p] = m >= zs::kMinMatch ? (m << 24 | (p - c) | (m == kMlCap ? kZcLocalCap : 0u)) : 0u;
    tile_sync<NT>();  // every lookup of the tile before any insert
    const uint32_t r = (p + 1) << 13;
    if (vs) atomicMax(hts + hs, r | gs);
    if (vl) atomicMax(htl + hl, r | gl);
    tile_sync<NT>();  // every insert before the next tile's lookups
  }
  ZQ(3);
#ifdef MCDC_ZC_TIMING
  if (tid == 0 && blockIdx.x % 397 == 0)
    printf("ZCS W %u L %u tiles %u load %lu ent %lu clear %lu loop %lu per_tile %lu\n", W, L, (L + NT - 1) / NT,
           (unsigned long)(tq[0] - tq0), (unsigned long)(tq[1] - tq[0]), (unsigned long)(tq[2] - tq[1]),
           (unsigned long)(tq[3] - tq[2]), (unsigned long)((tq[3] - tq[2]) / ((L + NT - 1) / NT)));
#endif
#undef ZQ
  // 4. hopeless: high entropy, no repeat (the tables are free: hts[0] is the
  // workgroup's "any repeat")
  bool any = __ballot(rep) != 0;
  if constexpr (W > 1) {
    if (tid == 0) hts[0] = 0u;
    __syncthreads();
    if (any && lane == 0) hts[0] = 1u;  // (any writer)
    __syncthreads();
    any = hts[0] != 0u;
  }
  if (tid == 0 && high && !any) blocks[bi].flags = kZcRaw | kZcSegRaw;
}

// Far matches: the 2^20 window of SecureStorage::compress (storage.rs:74-84)
// beyond the finder's reach (its segment and the kPrime bytes before it).
// One wave per 1024 positions of a block in a chunk's second or later
// segment.  Each far anchor (k_zc_probe's ballots) looks up the far tables of
// the 5 segments before its own, nearest first (the latest anchor per slot of
// each); a tagged entry within the window is verified on 16 bytes, extended
// backwards (up to kFarBack bytes, 16 at a time), and every position from the
// extension's start to the anchor gets the far match's word -- unless the
// finder verified a full match there itself (atomicMax: kZcLocalCap words
// win, then the longer match, then the larger offset, so the result does not
// depend on the order).  k_zc_parse extends the full matches.
//
// Rescue mode (before the finder): the same lookups for the blocks
// k_zc_probe found hopeless (its repeat test sees only the segment and the
// re-inserted bytes); a verified far match clears the block's kZcRaw.
__global__ __launch_bounds__(256) void k_zc_far(const uint8_t *base, uint64_t nbytes, ZcBlock *blocks, uint64_t nblk,
                                                const uint32_t *ftab, const uint64_t *fbits, uint32_t *words,
                                                bool rescue) {
  MCDC_VGPR_PAD(48);  // (not an exact fill)
  const uint64_t g = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const uint64_t bi = g / kZcFarBallots;
  const uint32_t j = (uint32_t)(g % kZcFarBallots), lane = lane_id();
  if (bi >= nblk) return;
  const ZcBlock B = blocks[bi];
  if (B.b < kZcSegBlocks || ((B.flags & kZcRaw) != 0) != rescue || j * 1024 >= B.len) return;
  const uint64_t bal = fbits[bi * kZcFarBallots + j];
  if (!((bal >> lane) & 1)) return;
  const uint64_t rec0 = bi - B.b;
  const uint64_t csrc = B.src - (uint64_t)B.b * kZcBlock;
  const uint32_t clen = (B.nb - 1) * (uint32_t)kZcBlock + blocks[bi + (B.nb - 1 - B.b)].len;
  const uint8_t *cb = base + csrc;
  const uint64_t cbytes = nbytes - csrc;
  uint32_t *wc = chunk_words(words, B);
  const uint32_t s = B.b / kZcSegBlocks;
  const uint32_t p = B.b * (uint32_t)kZcBlock + j * 1024 + 16 * lane;
  const uint32_t bend = min(clen, (B.b + 1) * (uint32_t)kZcBlock);
  uint32_t am = 0;  // far anchors among p .. p + 15
  {
    uint32_t w[6];
    const uint4 a = fix16(ld16c(cb, p, cbytes), p, cbytes), b = fix16(ld16c(cb, p + 16, cbytes), p + 16, cbytes);
    w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w, w[4] = b.x, w[5] = b.y;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj)
      if (p + jj + 8 <= clen && far_anchor(mix8(byte_window(w, jj), byte_window(w, jj + 4)))) am |= 1u << jj;
  }
  while (am) {
    const uint32_t q = p + (uint32_t)__builtin_ctz(am);
    am &= am - 1;
    if (q + kMlCap > bend || (!rescue && (wc[q] & kZcLocalCap))) continue;
    const uint4 x = fix16(ld16c(cb, q, cbytes), q, cbytes);
    const uint32_t m8 = mix8(x.x, x.y), tag = anchor_tag(mix5(x.x, x.y)), slot = far_slot(m8);
    uint32_t e[5];  // (the five tables' entries requested together)
#pragma unroll
    for (uint32_t k = 1; k <= 5; ++k)
      e[k - 1] = k <= s ? ftab[(rec0 + (uint64_t)(s - k) * kZcSegBlocks) * kZcFarSlots + slot] : 0u;
    uint32_t c = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t k = 1; k <= 5; ++k)
      if (c == 0xFFFFFFFFu && e[k - 1] && (e[k - 1] & 0x3FFFu) == tag) {
        const uint32_t cc = (s - k) * kZcSegBlocks * (uint32_t)kZcBlock + (e[k - 1] >> 14) - 1;
        c = q - cc <= zs::kWindow ? cc : 0xFFFFFFFEu;  // (the nearest tagged entry decides)
      }
    if (c >= 0xFFFFFFFEu) continue;
    if (prefix16(x, fix16(ld16c(cb, c, cbytes), c, cbytes)) < kMlCap) continue;
    if (rescue) {
      atomicAnd(&blocks[bi].flags, ~kZcRaw);
      atomicAnd(&blocks[bi - B.b % kZcSegBlocks].flags, ~kZcSegRaw);  // (the segment's first record)
      return;
    }
    uint32_t bk = 0;
    while (bk < kFarBack && c >= bk + 16) {
      const uint32_t sf = suffix16(*reinterpret_cast<const uint4 *>(cb + (q - bk - 16)),
                                   *reinterpret_cast<const uint4 *>(cb + (c - bk - 16)));
      bk += sf;
      if (sf < 16) break;
    }
    // the words of the extension's start and every kFarStride-th position
    // after it up to the anchor (the parse's chain meets one within
    // kFarStride positions of wherever it enters the stretch)
    const uint32_t off = q - c;
    for (uint32_t x0 = q - bk;; x0 += kFarStride) {
      x0 = min(x0, q);
      const uint32_t lim = min(kMlCap, min(clen, (x0 / (uint32_t)kZcBlock + 1) * (uint32_t)kZcBlock) - x0);
      if (lim >= zs::kMinMatch) atomicMax(wc + x0, lim << 24 | off);
      if (x0 == q) break;
    }
  }
}

#ifdef MCDC_ZC_TIMING  // (A/B: cycles per phase of one wave, some blocks, printed)
#define ZT_DECL uint64_t zt_[6] = {0, 0, 0, 0, 0, 0}, zt0_ = __builtin_amdgcn_s_memtime(), zt1_ = 0; uint32_t ztn_[2] = {0, 0}
#define ZT(k) (zt1_ = __builtin_amdgcn_s_memtime(), zt_[k] += zt1_ - zt0_, zt0_ = zt1_)
#define ZTN(k) (++ztn_[k])
#define ZT_PRINT(name, cond)                                                                                      \
  if ((cond) && lane_id() == 0)                                                                                  \
  printf("ZCT %s blk %lu t0 %lu t1 %lu t2 %lu t3 %lu t4 %lu n0 %u n1 %u\n", name, (unsigned long)blockIdx.x,      \
         (unsigned long)zt_[0], (unsigned long)zt_[1], (unsigned long)zt_[2], (unsigned long)zt_[3], (unsigned long)zt_[4], \
         ztn_[0], ztn_[1])
#else
#define ZTN(k) ((void)0)
#define ZT_DECL
#define ZT(k) ((void)0)
#define ZT_PRINT(name, cond)
#endif

// Wave scans with DPP (row shifts within 16-lane rows, then the row
// broadcasts of lanes 15 and 31): VALU operand modifiers, where __shfl_up /
// __shfl_xor go through the LDS crossbar (ds_bpermute) at LDS latency per step.
#define MCDC_DPP(old, v, ctrl, rm) ((uint32_t)__builtin_amdgcn_update_dpp((int)(old), (int)(v), ctrl, rm, 0xf, false))
// Inclusive sum over the wave's 64 lanes (all lanes active).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, uint32_t) {
  v += MCDC_DPP(0, v, 0x111, 0xf);  // row_shr:1
  v += MCDC_DPP(0, v, 0x112, 0xf);  // row_shr:2
  v += MCDC_DPP(0, v, 0x114, 0xf);  // row_shr:4
  v += MCDC_DPP(0, v, 0x118, 0xf);  // row_shr:8
  v += MCDC_DPP(0, v, 0x142, 0xa);  // row_bcast:15 into rows 1, 3
  v += MCDC_DPP(0, v, 0x143, 0xc);  // row_bcast:31 into rows 2, 3
  return v;
}
// Inclusive max over the wave's 64 lanes (values >= -1).
__device__ __forceinline__ int32_t wave_incl_max(int32_t v, uint32_t) {
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x111, 0xf));
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x112, 0xf));
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x114, 0xf));
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x118, 0xf));
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x142, 0xa));
  v = max(v, (int32_t)MCDC_DPP(-1, v, 0x143, 0xc));
  return v;
}
// The value of the lane below (wave_shr:1); lane 0 gets old.
__device__ __forceinline__ int32_t wave_shr1(int32_t v, int32_t old) { return (int32_t)MCDC_DPP(old, v, 0x138, 0xf); }
__device__ __forceinline__ int32_t lane63(int32_t v) { return __builtin_amdgcn_readlane(v, 63); }
__device__ __forceinline__ int32_t wave_max(int32_t v) { return lane63(wave_incl_max(v, 0)); }
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return (uint32_t)lane63((int32_t)wave_incl_sum(v, 0)); }

// The greedy parse of one block over k_zc_find's words, 256 positions per
// window (position i of the window in lane i % 64, slot i / 64), without a
// serial walk: every position's successor (+ its match length, or + 1 for a
// literal) is known from its word, so the chain from the cursor is found by
// pointer doubling in LDS (J_k = the 2^k-th successor, k <= 5; lane m finds
// the chain's node m of each 64 from the cursor by composing J over the bits
// of m), and the chain's matches and literals get their indices from prefix
// counts of ballots, each match its literal length and previous offset from
// the match ranked before it (LDS).
// Capped matches (16 verified bytes) get their true lengths before the walk
// (see the window loop); the first long one on the chain (more than kRunExt
// bytes past the 16) is extended by the wave (2 KiB per step) and ends the
// window.  Offsets repeat as repeat code 1 (the previous
// sequence's offset, literal length > 0: rep[0] is always the previous
// offset when only that code is used) after the block's first sequence.
__global__ __launch_bounds__(64) void k_zc_parse(const uint8_t *base, uint64_t nbytes, ZcBlock *blocks, uint64_t nblk,
                                                 uint32_t *words, uint8_t *stage, const uint32_t *porder) {
  __shared__ uint16_t J[6][257];
  __shared__ uint16_t ends[257], jp[256];
  __shared__ uint8_t mk[260], capl[256];
  __shared__ uint32_t offl[256], wbyt[64], mend[256], moff[256], llen[256];
  __shared__ uint16_t xlist[256];
  if (blockIdx.x >= nblk) return;
  const uint64_t bi = porder[blockIdx.x];  // (the longest blocks first, k_zc_segorder)
  const uint32_t lane = lane_id();
  const ZcBlock B = blocks[bi];
  if (B.flags & kZcRaw) {  // (hopeless, k_zc_probe: stored raw)
    if (lane == 0) blocks[bi].nlit = blocks[bi].nseq = 0;
    return;
  }
  const uint32_t end = B.len;
  const uint8_t *p0 = base + B.src;
  const uint32_t *w = words + (uint32_t)__builtin_amdgcn_readfirstlane((int)B.w0);  // (uniform: an SGPR base)
  uint8_t *lit = blk_slot(stage, B, bi) + zs::kLitHdr;
  uint64_t *sq = blk_seqs(words, B);  // (over the words already read: see blk_span)
  const uint32_t wlast = blk_span(B.len) - 1;  // (the block's last word: reads past the end clamped)
  uint32_t nlit = 0, nseq = 0, lit0 = 0, cur = 0, last_off = 0;  // (last_off 0: no sequence yet)
  if (lane == 0) {
    for (int k = 0; k < 6; ++k) J[k][256] = 256;
    ends[256] = 256;
  }
  // A window's words and source bytes (lane l: bytes [wb + 4 l, + 4)) are
  // requested a window ahead with loads outside the compiler's wait counting
  // (see ald16s: the literal and sequence stores would otherwise drain them),
  // and waited for at the next window's start, used or not.
  const uint64_t lim = nbytes - B.src;                                          // bytes readable at p0
  const bool wide = lim >= 4;                                                   // (else byte loads)
  const uint32_t lim4 = wide ? (uint32_t)min<uint64_t>(lim - 4, 0xFFFFFFFCull) : 0u;
  auto issue = [&](uint32_t wb, uint32_t *v, uint32_t &by) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = min(wb + 64 * j + lane, wlast);
      asm volatile("global_load_dword %0, %1, %2" : "=v"(v[j]) : "v"(4 * q), "s"(w) : "memory");
    }
    asm volatile("global_load_dword %0, %1, %2" : "=v"(by) : "v"(min(wb + 4 * lane, lim4)), "s"(p0) : "memory");
  };
  auto wait_all = [&](uint32_t *v, uint32_t &by) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(by)::"memory");
  };
  uint32_t nwd[4], nby;
  uint32_t nwb = 0;
  ZT_DECL;
  issue(0, nwd, nby);
  while (cur < end) {
    const uint32_t wb = cur & ~63u, s0 = cur - wb;
    ZTN(0);
    ZT(4);
    wait_all(nwd, nby);
    uint32_t wd[4], by;
    if (wb != nwb) {  // (a long match skipped the prefetched window)
      issue(wb, nwd, nby);
      wait_all(nwd, nby);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) wd[j] = wb + 64 * j + lane < end ? nwd[j] : 0u;
    {
      const uint32_t a = wb + 4 * lane, c = min(a, lim4);
      by = a - c < 4 ? nby >> (8 * (a - c)) : 0u;  // (clamped at the end of the input: realigned)
      if (!wide) {  // (fewer than 4 bytes readable)
        by = 0;
        for (uint32_t k = 0; k < 4; ++k)
          if (a + k < lim) by |= (uint32_t)p0[a + k] << (8 * k);
      }
    }
    wbyt[lane] = by;
    ZT(0);
    // Match lengths first.  A word of fewer than kMlCap bytes is exact; a
    // capped word (kMlCap verified bytes) is extended here, all of them at
    // once: consecutive capped positions with the same offset form a run of
    // one repeat, whose positions all end where it ends, so only each run's
    // last position is extended (per lane, up to kRunExt more bytes in one
    // round of loads) and the end is handed back through the run by pointer
    // jumping in LDS (ends[i] = ends[i + 1]).  A run still matching after
    // kRunExt bytes is long: the chain stops at it (J = 256), and the first
    // long match on the chain is extended by the whole wave (2 KiB per step)
    // and ends the window -- short repeats (identifiers, keywords, indents of
    // source code) no longer cost a memory round trip each.
    uint32_t ml[4], cj[4], en[4];
    bool valid[4], cap[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = 64 * j + lane;
      valid[j] = wb + i < end;
      ml[j] = (wd[j] >> 24) & 31u;
      cap[j] = valid[j] && ml[j] == kMlCap;
      offl[i] = wd[j] & 0xFFFFFFu;
      mk[i] = (uint8_t)(i == s0);
      en[j] = valid[j] ? i + (ml[j] ? ml[j] : 1u) : 256u;
    }
    const bool anycap = __ballot(cap[0] || cap[1] || cap[2] || cap[3]) != 0;  // (else every length is exact)
    if (anycap) {
#pragma unroll
      for (int j = 0; j < 4; ++j) capl[64 * j + lane] = (uint8_t)cap[j];
      // the runs' last positions, listed (ballot ranks) and extended one per
      // lane: one round of loads for the window (they were per slot: four
      // dependent memory round trips in a window of source code)
      uint32_t nx = 0;
      bool ext[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = 64 * j + lane;
        const bool same = i < 255 && capl[i + 1] && offl[i + 1] == offl[i];
        ext[j] = cap[j] && !same;
        en[j] = !valid[j] ? 256u : !cap[j] ? i + (ml[j] ? ml[j] : 1u) : same ? kEndNext : 0u;
        const uint64_t bx = __ballot(ext[j]);
        if (ext[j])
          xlist[nx + __builtin_amdgcn_mbcnt_hi((uint32_t)(bx >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bx, 0u))] =
              (uint16_t)i;
        nx += (uint32_t)__builtin_popcountll(bx);
        ends[i] = (uint16_t)en[j];
        jp[i] = (uint16_t)(i + 1);
      }
      lds_sync();  // (the list, written by other lanes)
      for (uint32_t r = lane; r < nx; r += 64) {  // kRunExt bytes after the run's kMlCap
        const uint32_t i = xlist[r], q = wb + i + kMlCap, off = offl[i];
        uint4 x[kRunExt / 16], y[kRunExt / 16];
#pragma unroll
        for (int u = 0; u < (int)(kRunExt / 16); ++u) {
          const uint64_t g = B.src + q + 16 * u;
          x[u] = ld16c(base, g, nbytes);
          y[u] = ld16c(base, g - off, nbytes);
        }
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < (int)(kRunExt / 16); ++u) {
          const uint32_t qu = q + 16 * u;
          const uint64_t g = B.src + qu;
          const uint32_t mu = qu < end ? min(prefix16(fix16(x[u], g, nbytes), fix16(y[u], g - off, nbytes)), end - qu) : 0u;
          m += m == 16 * (uint32_t)u ? mu : 0u;
        }
        ends[i] = (uint16_t)(m == kRunExt ? kEndLong : i + kMlCap + m);
      }
      lds_sync();
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ext[j]) en[j] = ends[64 * j + lane];
    }
    // the next window's words and bytes, in flight meanwhile (requested after
    // the run ends' loads: the compiler's wait for those counts every older
    // load, and would drain this prefetch with them)
    nwb = wb + 256;
    issue(nwb, nwd, nby);
    // the run's end to every position of the run (pointer jumping)
    for (int r = 0; r < 8 && anycap && __ballot(en[0] == kEndNext || en[1] == kEndNext || en[2] == kEndNext ||
                                                en[3] == kEndNext); ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = 64 * j + lane;
        if (en[j] == kEndNext) {
          const uint32_t p = jp[i], e2 = ends[p];
          if (e2 != kEndNext) {
            en[j] = e2;
            ends[i] = (uint16_t)e2;
          } else {
            jp[i] = jp[p];
          }
        }
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = 64 * j + lane;
      cj[j] = en[j] == kEndLong ? 256u : min(en[j], 256u);  // (a long run stops the chain)
      J[0][i] = (uint16_t)cj[j];
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {  // J_{k+1} = J_k(J_k), up to J_5 (32 nodes)
#pragma unroll
      for (int j = 0; j < 4; ++j) cj[j] = J[k][cj[j]];
#pragma unroll
      for (int j = 0; j < 4; ++j) J[k + 1][64 * j + lane] = (uint16_t)cj[j];
    }
    // The chain's nodes 64 at a time: node m of a quarter is J_0..J_5
    // composed over the set bits of m from the quarter's first node (lane m
    // finds it: 6 LDS reads) and is marked (256: past the window or a long
    // match); the next quarter starts one step after node 63.  Most windows
    // of compressible data hold fewer than 64 nodes: one quarter, and the
    // doubling stops at J_5 (it ran to J_7 and marked in 8 rounds before).
    // The chain stops at a long match: the wave extends it (2 KiB per step:
    // lane k compares bytes [.. + 32 k, + 32)) and, if it ends inside the
    // window, marks on from its end (J holds for every position) -- a long
    // match ended the window before, a window reload and recomputation each
    // (source code and binary data: many 48-byte-plus repeats per window).
    ZT(1);
    for (uint32_t st0 = s0;;) {
      for (uint32_t st = st0, qq = 0; qq < 4 && st < 256; ++qq) {
        uint32_t x = st;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          const uint32_t y = J[b][x];
          x = (lane >> b) & 1u ? y : x;
        }
        mk[x] = 1;
        st = (uint32_t)__builtin_amdgcn_readfirstlane((int)J[0][__builtin_amdgcn_readlane((int)x, 63)]);
      }
      int32_t lf = 0x7FFFFFFF;  // the first long match on the chain from st0
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = 64 * j + lane;
        const uint64_t bl = __ballot(i >= st0 && en[j] == kEndLong && mk[i]);
        if (lf == 0x7FFFFFFF && bl) lf = 64 * j + (int32_t)__builtin_ctzll(bl);
      }
      if (lf == 0x7FFFFFFF) break;
      ZTN(1);
      const uint32_t L = (uint32_t)lf, pos = wb + L, off = offl[L];
      uint32_t mlt = kMlCap;
      for (;;) {
        const uint32_t q = pos + mlt + 32 * lane;
        uint32_t m = 0;
        uint4 x[2], y[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // (the source may lie in an earlier block of the chunk: B.src + q - off)
          const uint64_t g = B.src + q + 16 * u;
          x[u] = ld16c(base, g, nbytes);
          y[u] = ld16c(base, g - off, nbytes);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint32_t qu = q + 16 * u;
          const uint64_t g = B.src + qu;
          const uint32_t mu = qu < end ? min(prefix16(fix16(x[u], g, nbytes), fix16(y[u], g - off, nbytes)), end - qu) : 0u;
          m += m == 16 * (uint32_t)u ? mu : 0u;
        }
        const uint64_t brk = __ballot(m < 32);
        if (brk) {
          const uint32_t t = (uint32_t)__builtin_ctzll(brk);
          mlt += 32 * t + (uint32_t)__builtin_amdgcn_readlane((int)m, (int)t);
          break;
        }
        mlt += 2048;
      }
      if (lane == 0) llen[L] = mlt;
      if (L + mlt >= 256) break;  // (the window ends with it)
      st0 = L + mlt;
    }
    bool node[4], mt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = 64 * j + lane;
      node[j] = valid[j] && mk[i];
      mt[j] = node[j] && ml[j] != 0;
    }
    ZT(2);
    // this window's matches and literals, in position order (slot-major).
    // Pass 1: window ranks from ballots; each match's end and offset into LDS
    // at its rank, each literal's byte out.  Pass 2: a match's literal length
    // and the offset it may repeat from the match ranked before it (the
    // block's carried lit0 / last_off for the window's first) -- two LDS reads
    // where a wave max-scan carried them (13 DPP steps per slot before).
    uint32_t mcount = 0, lcount = 0, exit_pos = 0;
    uint32_t mrk[4], mln[4];
    bool mm[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = 64 * j + lane, q = wb + i;
      const bool in = node[j], m = in && mt[j], l = in && !mt[j];
      const uint32_t mlen = en[j] == kEndLong ? llen[i] : cap[j] ? en[j] - i : ml[j];
      const uint64_t bm = __ballot(m), bl = __ballot(l);
      const uint32_t mr = mcount + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      const uint32_t lr = lcount + __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
      if (m) {
        mend[mr] = q + mlen;
        moff[mr] = offl[i];
      }
      if (l) lit[nlit + lr] = reinterpret_cast<const uint8_t *>(wbyt)[i];
      mcount += (uint32_t)__builtin_popcountll(bm);
      lcount += (uint32_t)__builtin_popcountll(bl);
      if (in) exit_pos = max(exit_pos, q + (m ? mlen : 1u));
      mm[j] = m;
      mrk[j] = mr;
      mln[j] = mlen;
    }
    lds_sync();  // (the ranks' ends and offsets written by other lanes)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (mm[j]) {
        const uint32_t i = 64 * j + lane, q = wb + i, mr = mrk[j];
        const uint32_t start = mr ? mend[mr - 1] : lit0, poff = mr ? moff[mr - 1] : last_off;
        const uint32_t ll = q - start, off = offl[i];
        const uint32_t ov = (ll && off == poff) ? 1u : off + 3;
        sq[nseq + mr] = zs::seq_pack_ov(ll, mln[j], ov);
      }
    }
    nseq += mcount;
    nlit += lcount;
    if (mcount) {
      lit0 = mend[mcount - 1];
      last_off = moff[mcount - 1];
    }
    cur = (uint32_t)wave_max((int32_t)exit_pos);
    ZT(3);
  }
  wait_all(nwd, nby);  // (no load may land in a register after its last use)
  MCDC_VGPR_PAD(88);  // (not an exact fill)
  ZT_PRINT("parse", bi % 509 == 0);
  if (lane == 0) {
    blocks[bi].nlit = nlit;
    blocks[bi].nseq = nseq;
  }
}


// huf_build (mcdc_zstd.h) by the wave, from the counts and ranks of the
// lane's four symbols (lane + 64 h): the same code.  Lane 0 runs only the
// two-queue merge (register heads, one LDS read per step); the depths by
// pointer jumping (d += d[anc], anc = anc[anc]: a few rounds for the <= 511
// nodes, 8 per lane); the lengths by rank from the per-depth counts; the
// canonical codes from ballots per length, in symbol order.
__device__ void huf_build_wave(const uint32_t (&c)[4], const uint32_t (&r)[4], uint32_t n, HufCT &ct, HufWork &w,
                               uint32_t lane) {
  __shared__ uint32_t s_maxd;
  uint32_t *const f = w.f, *const bl = w.bl;
#pragma unroll
  for (int h = 0; h < 4; ++h)
    if (c[h]) f[r[h]] = c[h];
  bl[lane] = 0;
  __syncthreads();
  const uint32_t m = 2 * n - 1, root = m - 1;
  if (lane == 0) {
    constexpr uint32_t kInf = 0xFFFFFFFFu;
    uint32_t li = 0, ni = n, fl = f[0], fn = kInf;
    for (uint32_t nn = n; nn < m; ++nn) {
      uint32_t ab[2], wab[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (fl <= fn) {  // (a leaf on a tie: the serial queue's order)
          ab[t] = li++;
          wab[t] = fl;
          fl = li < n ? f[li] : kInf;
        } else {
          ab[t] = ni++;
          wab[t] = fn;
          fn = ni < nn ? f[ni] : kInf;
        }
      }
      const uint32_t sum = wab[0] + wab[1];
      f[nn] = sum;
      w.par[ab[0]] = w.par[ab[1]] = (uint16_t)nn;
      if (fn == kInf) fn = sum;  // (the internal queue was empty: ni == nn)
    }
  }
  __syncthreads();
  // depths: node i = lane + 64 j
  uint32_t an[8], dn[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t i = lane + 64 * j;
    an[j] = i < root ? w.par[i] : root;
    dn[j] = i < root ? 1u : 0u;
  }
  for (;;) {
    bool more = false;
#pragma unroll
    for (int j = 0; j < 8; ++j) more |= lane + 64 * j < m && an[j] != root;
    if (!__ballot(more)) break;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (lane + 64 * j < m) {
        w.par[lane + 64 * j] = (uint16_t)an[j];
        w.dep[lane + 64 * j] = (uint8_t)dn[j];
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (lane + 64 * j < m && an[j] != root) {
        dn[j] += w.dep[an[j]];
        an[j] = w.par[an[j]];
      }
    __syncthreads();
  }
  // leaves 0 .. n - 1 per depth (capped at 63, as huf_build)
  uint32_t maxd = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (lane + 64 * j < n) {
      const uint32_t d = min(dn[j], 63u);
      atomicAdd(&bl[d], 1u);
      maxd = max(maxd, d);
    }
  maxd = (uint32_t)wave_max((int32_t)maxd);
  __syncthreads();
  if (lane == 0) {  // the length limit (huf_build's steps)
    if (maxd > kHufMaxBits) {
      for (uint32_t d = kHufMaxBits + 1; d <= maxd; ++d) {
        bl[kHufMaxBits] += bl[d];
        bl[d] = 0;
      }
      uint64_t kraft = 0;
      for (uint32_t d = 1; d <= kHufMaxBits; ++d) kraft += (uint64_t)bl[d] << (kHufMaxBits - d);
      while (kraft > (1ull << kHufMaxBits)) {
        uint32_t d = kHufMaxBits - 1;
        while (bl[d] == 0) --d;
        --bl[d];
        bl[d + 1] += 2;
        --bl[kHufMaxBits];
        --kraft;
      }
      maxd = kHufMaxBits;
    }
    s_maxd = maxd;
  }
  __syncthreads();
  maxd = s_maxd;
  // lengths: the j-th most frequent symbol (j = n - 1 - rank) takes the
  // shortest depth d with bl[1] + .. + bl[d] > j
  uint32_t L[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    L[h] = 0;
    if (c[h]) {
      const uint32_t j = n - 1 - r[h];
      uint32_t cum = 0;
      for (uint32_t d = 1; d <= maxd; ++d) {
        cum += bl[d];
        if (cum > j) {
          L[h] = d;
          break;
        }
      }
    }
    ct.nb[lane + 64 * h] = (uint8_t)L[h];
  }
  uint32_t last = 0;
#pragma unroll
  for (int h = 0; h < 4; ++h)
    if (c[h]) last = lane + 64 * h;
  last = (uint32_t)wave_max((int32_t)last);
  // canonical codes: per length from the longest down, start 0, next
  // length's start (start + count) >> 1; within a length in symbol order
  uint32_t start[kHufMaxBits + 1];
  {
    uint32_t mn = 0;
#pragma unroll
    for (int d = kHufMaxBits; d >= 1; --d) {
      start[d] = mn;
      if ((uint32_t)d <= maxd) mn = (mn + bl[d]) >> 1;
    }
  }
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int d = 1; d <= (int)kHufMaxBits; ++d) {
    uint32_t base = start[d];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint64_t mk = __ballot(L[h] == (uint32_t)d);
      if (L[h] == (uint32_t)d) ct.code[lane + 64 * h] = (uint16_t)(base + (uint32_t)__builtin_popcountll(mk & lt));
      base += (uint32_t)__builtin_popcountll(mk);
    }
  }
  if (lane == 0) {
    ct.maxb = maxd;
    ct.last = last;
  }
}

// The literals section of a compressed block: Huffman-coded or RLE when that
// is smaller than the raw section (3-byte header + the literals), written
// over the staging slot's raw literals; B.lsize its size, 0 = raw.  The whole
// wave works on every step but the tree and its description (one lane):
//   count    16 bytes per lane per step into 4 LDS histogram copies
//   rank     the 256 symbols by count (ties by symbol), four per lane
//   tree     huf_build on the ranked symbols, the weights' description
//            (direct or FSE-compressed, the shorter; lane 0)
//   sizes    bits per stream (wave sums); give up unless smaller than raw
//   streams  each stream cut into 64 contiguous pieces (in writing order:
//            the last literal first), a lane per piece: its bit count, a
//            wave scan for its offset, then its bits packed in a register
//            and stored a word at a time into the block's match-word
//            scratch's upper half (the sequences fill at most the lower; words shared with a
//            neighbouring piece OR-ed in)
//   store    header, tree, jump table; the section copied to the slot
// (LDS ~9 KiB per wave: 16 waves per CU; the section itself stays in HBM.)
__global__ __launch_bounds__(64) void k_zc_huff(const uint8_t *base, uint64_t nbytes, ZcBlock *blocks, uint64_t nblk,
                                                uint8_t *stage, uint32_t *scratch, const uint32_t *porder) {
  // LDS: the counts (4 copies while counting, merged into the first), then
  // in the place of copies 1-3, one after another: huf_build's work, the
  // description's work, the code table ctw (6.4 KiB in all: 25 waves per CU)
  constexpr uint32_t kRegion = (sizeof(HufWork) > 768 * 4 ? sizeof(HufWork) : 768 * 4) / 4;
  static_assert(sizeof(HufDescWork) <= kRegion * 4 && sizeof(HufWork) % 4 == 0, "huff LDS layout");
  __shared__ __attribute__((aligned(16))) uint32_t pool[256 + kRegion];
  uint32_t(*const hist)[256] = reinterpret_cast<uint32_t(*)[256]>(pool);
  HufWork &hw = *reinterpret_cast<HufWork *>(pool + 256);
  HufDescWork &dw = *reinterpret_cast<HufDescWork *>(pool + 256);
  uint32_t *const ctw = pool + 256;
  __shared__ HufCT ct;
  __shared__ uint8_t tdesc[132];
  __shared__ uint32_t tree_sz;
  if (blockIdx.x >= nblk) return;
  const uint64_t bi = porder[blockIdx.x];  // (the longest blocks first, k_zc_segorder)
  const uint32_t lane = lane_id();
  const ZcBlock B = blocks[bi];
  // a block without sequences: all of it literals, read from the input (k_zc_parse staged nothing)
  const uint32_t n = B.nseq ? B.nlit : B.len;
  if (n < 32 || (B.flags & kZcRaw)) return;  // (lsize stays 0: raw literals; hopeless blocks stored raw)
  uint8_t *st = blk_slot(stage, B, bi);
  const uint8_t *src = B.nseq ? st + kLitHdr : base + B.src;
  ZT_DECL;
  for (uint32_t k = lane; k < 4 * 256; k += 64) (&hist[0][0])[k] = 0;
  __syncthreads();
  // streams: stream k holds literals [k seg, min((k + 1) seg, n)); four of
  // them above 1023 literals
  const bool one = n < 1024;
  const uint32_t seg = one ? n : (n + 3) / 4, ns = one ? 1 : 4;
  // count per stream (hist[k]), 16 bytes per lane per step (misaligned
  // 16-byte loads: gfx950 reads the bytes at the address); a lane's 16 bytes
  // cross at most one stream boundary (seg >= 256)
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
    const uint32_t s0 = one ? 0u : (k >= seg) + (k >= 2 * seg) + (k >= 3 * seg), nb0 = (s0 + 1) * seg;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
      if (j < m) atomicAdd(&hist[s0 + (k + j >= nb0 ? 1u : 0u)][(w[j >> 2] >> (8 * (j & 3))) & 0xFF], 1u);
  }
  __syncthreads();
  uint32_t c[4], cs[3][4];  // totals; streams 0-2's counts (stream 3's = total - the rest)
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const uint32_t k = lane + 64 * h;
    cs[0][h] = hist[0][k];
    cs[1][h] = hist[1][k];
    cs[2][h] = hist[2][k];
    c[h] = cs[0][h] + cs[1][h] + cs[2][h] + hist[3][k];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 4; ++h) hist[0][lane + 64 * h] = c[h];
  // rank: symbols by count ascending, ties by symbol (huf_build's stable order)
  uint64_t pm[4];
  uint32_t distinct = 0;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    pm[h] = __ballot(c[h] != 0);
    distinct += (uint32_t)__builtin_popcountll(pm[h]);
  }
  if (distinct == 1) {  // RLE literals: 3-byte header + the byte
    if (lane == 0) {
      uint32_t sym = 0;
      for (int h = 0; h < 4; ++h)
        if (pm[h]) sym = 64 * h + (uint32_t)__builtin_ctzll(pm[h]);
      put_rle_lit_header(st, n);
      st[3] = (uint8_t)sym;
      blocks[bi].lsize = 4;
    }
    return;
  }
  __syncthreads();
  uint32_t r[4] = {0, 0, 0, 0};
  if (distinct <= 96) {  // (text: a few dozen symbols -- compare against the present ones only)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      for (uint64_t m = pm[g]; m; m &= m - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m), t = 64 * g + l;
        const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)c[g], (int)l);
#pragma unroll
        for (int h = 0; h < 4; ++h) r[h] += (q < c[h] || (q == c[h] && t < lane + 64 * h)) ? 1u : 0u;
      }
  } else {
    for (uint32_t t = 0; t < 256; t += 4) {
      const uint4 q = *reinterpret_cast<const uint4 *>(&hist[0][t]);  // (broadcast)
      const uint32_t qs[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < 4; ++h)
          r[h] += (qs[j] && (qs[j] < c[h] || (qs[j] == c[h] && t + j < lane + 64 * h))) ? 1u : 0u;
    }
  }
  ZT(0);
#if MCDC_ZC_HCUT == 1  // (A/B timing: stop after the counts)
  return;
#endif
  huf_build_wave(c, r, distinct, ct, hw, lane);
  __syncthreads();
  ZT(4);
  if (lane == 0) tree_sz = huf_tree_desc(ct, tdesc, dw);
  __syncthreads();
  ZT(1);
  const uint32_t tree = tree_sz;
  if (!tree) return;  // (no description applies: raw literals)
#if MCDC_ZC_HCUT == 2  // (A/B timing: stop after the tree)
  return;
#endif
  // code | length << 16 per symbol: one LDS read per literal; bits per stream
  // from the per-stream counts
  uint32_t sb[4] = {0, 0, 0, 0};
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const uint32_t x = lane + 64 * h, nb = ct.nb[x];
    ctw[x] = nb ? (uint32_t)ct.code[x] | nb << 16 : 0u;
    sb[0] += cs[0][h] * nb;
    sb[1] += cs[1][h] * nb;
    sb[2] += cs[2][h] * nb;
    sb[3] += (c[h] - cs[0][h] - cs[1][h] - cs[2][h]) * nb;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) sb[k] = wave_sum(sb[k]);
  if (one) sb[0] += sb[1] + sb[2] + sb[3];  // (one stream: every count is stream 0's)
  __syncthreads();
  ZT(2);
  uint32_t ssz[4];
  const uint32_t total = huf_section_size(tree, n, sb, one, ssz);
  if (total >= kLitHdr + n) return;  // not smaller than raw
  const uint32_t csize = tree + (one ? 0 : 6) + ssz[0] + (one ? 0 : ssz[1] + ssz[2] + ssz[3]);
  if (one && csize >= 1024) return;  // (one stream: 10-bit sizes)
  const uint32_t hdr = lit_hdr_size(n, csize, one);
  uint32_t *sw = blk_upper(scratch, B);  // the section under assembly (the words' upper half)
  const uint32_t nq = (total + 3) / 4 + 1;
  for (uint32_t k = lane; k < nq; k += 64) sw[k] = 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // (same wave: agent scope would write back the L2)
  // The streams, 256 literals per step in writing order (the last literal
  // first): lane l takes writing indices 4 l .. 4 l + 3 of the step (one
  // 4-byte load, read from its top byte down), a wave scan of the lanes' bit
  // counts places them, their codes are OR-ed into an LDS ring of 512 words,
  // and the ring's completed words go out with plain stores (a stream's first
  // and last word, shared with its neighbours, OR-ed in).
  uint32_t *const ring = pool + 512;
  constexpr uint32_t kRing = 512;
  static_assert(512 + kRing <= 256 + kRegion, "huff ring in the LDS pool");
  uint32_t o = hdr + tree + (one ? 0 : 6);  // byte offset of stream k in the section
  for (uint32_t k = 0; k < ns; ++k) {
    const uint32_t a = k * seg, e = min(a + seg, n), len = e - a;
    const uint32_t fw = (8 * o) >> 5;  // the stream's first word
    uint32_t bitp = 8 * o, ff = fw;    // next bit; first word not yet flushed
    for (uint32_t u = lane; u < kRing; u += 64) ring[u] = 0;
    auto flush = [&](uint32_t upto) {  // words [ff, upto) out, their ring slots zeroed
      for (uint32_t i = ff + lane; i < upto; i += 64) {
        const uint32_t v = ring[i & (kRing - 1)];
#if MCDC_ZC_HCUT != 3  // (A/B timing: no stores)
        if (i == fw) atomicOr(sw + i, v);
        else sw[i] = v;
#endif
        ring[i & (kRing - 1)] = 0;
      }
      ff = upto;
    };
    // lane's 4 bytes of the step at r0: literals e - 1 - w0 down to e - 4 - w0
    // (w0 = r0 + 4 lane) are the 4 bytes at e - 4 - w0, clamped to the
    // stream's first literal (the bytes below it shifted out); requested a
    // step ahead, outside the compiler's wait counting (see ald16s)
    auto issue = [&](uint32_t r0) {
      const int32_t at = (int32_t)e - 4 - (int32_t)(r0 + 4 * lane);
      const uint8_t *p = src + (at < (int32_t)a ? a : (uint32_t)at);
      uint32_t v;
      asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
      return v;
    };
    // (each step waits for its own bytes, requested two steps back: the
    // step between issued one load after them, so vmcnt(1) -- a flush's
    // stores, which may retire out of order, only make it wait longer)
    auto step = [&](uint32_t r0, uint32_t &q) {
      asm volatile("s_waitcnt vmcnt(1)" : "+v"(q)::"memory");
      const uint32_t w0 = r0 + 4 * lane;
      const uint32_t cnt = w0 < len ? min(len - w0, 4u) : 0u;
      const int32_t at = (int32_t)e - 4 - (int32_t)w0;
      const uint32_t below = at < (int32_t)a ? (uint32_t)((int32_t)a - at) : 0u;  // bytes below the stream (cnt < 4)
      const uint32_t dw = below >= 4 ? 0u : q << (8 * below);
      q = issue(r0 + 512);
      // the lane's 4 codes packed (<= 44 bits), then placed: the first and
      // last word of its span may be shared with the neighbouring lanes (LDS
      // OR), a middle word is its own (plain store)
      uint64_t acc = 0;
      uint32_t lb = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t t = (uint32_t)j < cnt ? ctw[(dw >> (8 * (3 - j))) & 0xFFu] : 0u;
        acc |= (uint64_t)(t & 0xFFFFu) << lb;
        lb += t >> 16;
      }
      const uint32_t incl = wave_incl_sum(lb, lane);
      if (lb) {
        const uint32_t off = bitp + incl - lb, sh = off & 31, wd = off >> 5;
        const uint64_t lo = acc << sh;
        const uint32_t top = sh ? (uint32_t)(acc >> (64 - sh)) : 0u;  // bits 64.. of the shifted span
        const uint32_t nw = (sh + lb + 31) >> 5;                        // words spanned (1..3)
        atomicOr(ring + (wd & (kRing - 1)), (uint32_t)lo);
        if (nw == 2) atomicOr(ring + ((wd + 1) & (kRing - 1)), (uint32_t)(lo >> 32));
        if (nw == 3) {
          ring[(wd + 1) & (kRing - 1)] = (uint32_t)(lo >> 32);
          atomicOr(ring + ((wd + 2) & (kRing - 1)), top);
        }
      }
      bitp += (uint32_t)lane63((int32_t)incl);
      if ((bitp >> 5) - ff >= 128) flush(bitp >> 5);
    };
    uint32_t da = issue(0), db = issue(256);
#if MCDC_ZC_HCUT == 5  // (A/B timing: no stream steps)
    if (len > 0) break;
#endif
    for (uint32_t r0 = 0; r0 < len; r0 += 512) {  // (two registers alternate: no copy of a loading
      step(r0, da);                                 // register; a step at or past len adds nothing)
      step(r0 + 256, db);
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(da), "+v"(db)::"memory");
    // the end mark, then every word the stream touched (the last one OR-ed)
    if (lane == 0) atomicOr(ring + ((bitp >> 5) & (kRing - 1)), 1u << (bitp & 31));
    const uint32_t last = bitp >> 5;
    flush(last);
    if (lane == 0) atomicOr(sw + last, ring[last & (kRing - 1)]);
    o += ssz[k];
  }
#if MCDC_ZC_HCUT == 4  // (A/B timing: stop after the streams)
  return;
#endif
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // (same wave: agent scope would write back the L2)
  if (lane == 0) {
    uint8_t *sec = reinterpret_cast<uint8_t *>(sw);
    put_huf_lit_header(sec, n, csize, one);
    for (uint32_t i = 0; i < tree; ++i) sec[hdr + i] = tdesc[i];
    if (!one)
      for (int k = 0; k < 3; ++k) {
        sec[hdr + tree + 2 * k] = (uint8_t)ssz[k];
        sec[hdr + tree + 2 * k + 1] = (uint8_t)(ssz[k] >> 8);
      }
    blocks[bi].lsize = total;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // (same wave: agent scope would write back the L2)
  // (every read of the staged literals is done: the section replaces them)
  const uint32_t n16 = (total + 15) / 16;
  for (uint32_t k = lane; k < n16; k += 64)
    reinterpret_cast<uint4 *>(st)[k] = reinterpret_cast<const uint4 *>(sw)[k];
  ZT(3);
  ZT_PRINT("huff", bi % 509 == 0);
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

// The sequences section of a block, in three kernels (the serial FSE state
// machines split from the rest, and run for many blocks per wave):
//   k_zc_plan    ONE WAVE PER BLOCK: code histograms (lanes over the
//                sequences, LDS atomics), seq_plan on lane 0 (per symbol type
//                the block's own FSE_Compressed_Mode table or the predefined
//                one), the own tables built by the wave; plan and tables to
//                the upper half of the block's match-word scratch (free
//                after k_zc_huff), the codes to the staging slot after the
//                raw literals (free until k_zc_encode)
//   k_zc_chain   ONE LANE PER STATE MACHINE, 9 blocks x 3 types per wave:
//                the wave's 27 tables in LDS, each lane walks its block's
//                sequences from the last to the first, per sequence the state
//                bits (count | value << 4, 16 bits; one array per symbol type,
//                a batch of 16 stored as 32 contiguous bytes), then the final
//                state; codes prefetched 8 sequences ahead
//   k_zc_encode  ONE WAVE PER BLOCK: per sequence its bits (state bits + extra
//                bits), 64 sequences at a time OR-ed into an LDS buffer at
//                offsets from wave scans in writing order (last sequence
//                first), the buffer's whole words out with plain stores, the
//                partial last word carried; then the final states, the end
//                mark and the header (count, modes, descriptions)
// The block stays raw when the compressed block is not smaller.
struct ZcSeqTab {    // (in the upper half of the block's match-word scratch)
  FseCTL t[3];       // LL, OF, ML: own or predefined
  uint32_t fin[3];   // final states (k_zc_chain)
  uint32_t sbits[3]; // state bits of each machine's sequences (k_zc_chain)
  uint32_t xbits;    // extra bits of the block's sequences (k_zc_plan)
  SeqPlan P;
};
__device__ __forceinline__ ZcSeqTab *seq_tab(uint8_t *extra, uint64_t bi) {
  return reinterpret_cast<ZcSeqTab *>(extra + bi * kZcExtra);
}
// k_zc_chain's state records: three arrays of rec_cap 16-bit words (LL, OF,
// ML), by sequence (a block of len bytes has at most len / 4 sequences), in
// the upper half of the block's words (k_zc_huff's section copied out by
// then), or after the tables in extra[] for blocks under 512 words.
constexpr uint32_t kSeqTabBytes = (sizeof(ZcSeqTab) + 15) / 16 * 16;
constexpr uint32_t kRecsUpper = 512;  // (span >= this: 1.5 span + the 128-byte reads past the end <= 2 span)
static_assert(kSeqTabBytes + 3 * (kRecsUpper - 64) / 2 + 256 <= kZcExtra, "tables and short blocks' records in extra[]");
__device__ __forceinline__ uint32_t rec_cap(const ZcBlock &B) { return blk_span(B.len) / 4; }
__device__ __forceinline__ uint16_t *blk_recs(uint32_t *words, uint8_t *extra, const ZcBlock &B, uint64_t bi) {
  return blk_span(B.len) >= kRecsUpper ? reinterpret_cast<uint16_t *>(blk_upper(words, B))
                                       : reinterpret_cast<uint16_t *>(extra + bi * kZcExtra + kSeqTabBytes);
}
// Per symbol type the sequences' codes, one byte each, the last sequence
// first (k_zc_chain's walking order), + 8 bytes of slack, in the staging slot
// after the raw literals (16-byte aligned): every sequence covers a match of
// at least 4 bytes, so nlit + 4 nseq <= len and the three arrays fit in the
// slot (span + 64 bytes); k_zc_huff's section is shorter than the raw
// literals it replaces, and k_zc_encode writes over the codes only after
// k_zc_chain read them.  (k_zc_chain's prefetches read up to kZcSeqCap + 48
// bytes past a block's codes: the staging buffer carries kZcStagePad more.)
__device__ __forceinline__ uint8_t *seq_codes(uint8_t *stage, const ZcBlock &B, uint64_t bi, uint32_t k) {
  return blk_slot(stage, B, bi) + ((kLitHdr + B.nlit + 15) & ~15u) + k * (B.nseq + 8);
}
static_assert(kLitHdr + 15 + 3 * 8 <= 64, "codes fit the staging slot (nlit + 3 nseq <= len <= span)");
static_assert(kZcSeqCap + 64 <= kZcStagePad, "staging pad covers k_zc_chain's reads past the codes");

// Float sum over the wave's 64 lanes (DPP, as wave_incl_sum), the total in every lane.
__device__ __forceinline__ float wave_sum_f(float v) {
#define MCDC_FADD(ctrl, rm) v += __int_as_float((int)MCDC_DPP(0, __float_as_int(v), ctrl, rm))
  MCDC_FADD(0x111, 0xf);
  MCDC_FADD(0x112, 0xf);
  MCDC_FADD(0x114, 0xf);
  MCDC_FADD(0x118, 0xf);
  MCDC_FADD(0x142, 0xa);
  MCDC_FADD(0x143, 0xc);
#undef MCDC_FADD
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// seq_plan (mcdc_zstd.h) by the whole wave: lane s holds symbol s of a type,
// the normalization, its largest count and both costs by wave reductions;
// only the table description is written by one lane.  (The decisions are
// seq_plan's; a cost sum in another order may round differently, which can
// only move a near tie between two valid encodings.)
__device__ void seq_plan_wave(uint32_t (*cnt)[53], uint32_t nseq, SeqPlan &P, uint32_t lane) {
  const int16_t *pre[3] = {kLLNorm, kOFNorm, kMLNorm};
  const uint32_t npre[3] = {36, 29, 53}, tpre[3] = {6, 5, 6}, shift[3] = {6, 4, 2};
  uint32_t ndesc = 0, modes = 0;
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = lane < kSeqNSym[k] ? cnt[k][lane] : 0u;
    const uint64_t nz = __ballot(c != 0);
    const uint32_t distinct = (uint32_t)__builtin_popcountll(nz), maxsym = nz ? 63u - (uint32_t)__builtin_clzll(nz) : 0u;
    bool own = false;
    uint32_t tl = tpre[k], nd = 0;
    if (nseq >= 32 && distinct >= 2) {
      tl = fse_table_log(nseq, maxsym, kSeqMaxLog[k]);
      const uint32_t scale = 1u << tl;
      uint32_t v = c ? (c * scale + nseq / 2) / nseq : 0u;
      if (c && v == 0) v = 1;
      const uint32_t sum = wave_sum(v);
      const uint32_t bc = (uint32_t)wave_max((int32_t)c);
      const uint32_t big = (uint32_t)__builtin_ctzll(__ballot(c == bc));  // (the first largest count)
      const int32_t fixed = (int32_t)__builtin_amdgcn_readlane((int)v, (int)big) + (int32_t)scale - (int32_t)sum;
      if (fixed >= 1) {
        const int32_t nrm = lane == big ? fixed : (int32_t)v;
        if (lane < 53) P.norm[k][lane] = (int16_t)(lane <= maxsym ? nrm : 0);
        __syncthreads();
        if (lane == 0) nd = fse_write_ncount(P.norm[k], maxsym + 1, tl, P.desc + ndesc);
        nd = (uint32_t)__builtin_amdgcn_readlane((int)nd, 0);
        const int32_t pn0 = lane < npre[k] ? pre[k][lane] : 0, pn = pn0 == -1 ? 1 : pn0;
        const float oc = c ? (float)c * ((float)tl - log2f((float)nrm)) : 0.0f;
        const float pc = c ? (pn <= 0 ? 1e30f : (float)c * ((float)tpre[k] - log2f((float)pn))) : 0.0f;
        const float ownc = wave_sum_f(oc) + 8.0f * (float)nd, predc = wave_sum_f(pc);
        own = ownc < predc;
      }
    }
    if (lane == 0) {
      P.own[k] = own ? 1u : 0u;
      P.tl[k] = own ? tl : tpre[k];
      P.doff[k] = ndesc;
      P.dlen[k] = own ? nd : 0u;
    }
    if (own) {
      ndesc += nd;
      modes |= 2u << shift[k];
    }
    __syncthreads();
  }
  if (lane == 0) {
    P.ndesc = ndesc;
    P.modes = modes;
  }
}

__global__ __launch_bounds__(64) void k_zc_plan(const ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                uint32_t *words, uint8_t *extra, ZTables T, const uint32_t *porder) {
  __shared__ FseCTL tb[3];
  __shared__ SeqPlan P;
  __shared__ uint32_t hist[3][53], cum[54], seen[54];
  const uint32_t lane = lane_id();
  if (blockIdx.x >= nblk) return;
  const uint64_t bi = porder[blockIdx.x];  // (the longest blocks first, k_zc_segorder)
  const ZcBlock B = blocks[bi];
  const uint32_t ns = B.nseq;
  if (ns == 0) return;
  const uint64_t *sq = blk_seqs(words, B);
  ZT_DECL;
  for (uint32_t k = lane; k < 3 * 53; k += 64) (&hist[0][0])[k] = 0;
  __syncthreads();
  uint8_t *cd0 = seq_codes(stage, B, bi, 0), *cd1 = seq_codes(stage, B, bi, 1), *cd2 = seq_codes(stage, B, bi, 2);
  uint32_t xb = 0;  // extra bits
  // (64 sequences per step, the next step's requested meanwhile outside the
  // compiler's wait counting: see ald16s)
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto issue = [&](uint32_t i) {
    u32x2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(sq + min(i, ns - 1)) : "memory");
    return v;
  };
  u32x2 qv = issue(lane);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(qv)::"memory");
  for (uint32_t i0 = 0; i0 < ns; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint64_t q = (uint64_t)qv.y << 32 | qv.x;
    qv = issue(i + 64);
    if (i < ns) {
      const uint32_t c0 = ll_code(seq_ll(q)), c1 = highbit(seq_ov(q)), c2 = ml_code(seq_ml(q) - 3);
      xb += ll_bits(c0) + c1 + ml_bits(c2);
      atomicAdd(&hist[0][c0], 1u);
      atomicAdd(&hist[1][c1], 1u);
      atomicAdd(&hist[2][c2], 1u);
      cd0[ns - 1 - i] = (uint8_t)c0;
      cd1[ns - 1 - i] = (uint8_t)c1;
      cd2[ns - 1 - i] = (uint8_t)c2;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(qv)::"memory");
  }
  __syncthreads();
  ZT(3);
  seq_plan_wave(hist, ns, P, lane);
  __syncthreads();
  ZT(4);
  const FseCT *pre[3] = {&T.ll, &T.of, &T.ml};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (P.own[k]) {
      fse_build_wave(P.norm[k], P.tl[k], tb[k], cum, seen, lane);
    } else {
      tb[k].state[lane] = pre[k]->state[lane];
      if (lane < 53) {
        tb[k].dfs[lane] = pre[k]->dfs[lane];
        tb[k].dnb[lane] = pre[k]->dnb[lane];
      }
      if (lane == 0) tb[k].log = pre[k]->log;
    }
    __syncthreads();
  }
  ZcSeqTab *tab = seq_tab(extra, bi);
  xb = wave_sum(xb);
  if (lane == 0) tab->xbits = xb;
#pragma unroll
  for (int k = 0; k < 3; ++k) {  // (the states in use, then dfs, dnb, log)
    const uint32_t nst = 1u << tb[k].log;
    for (uint32_t u = lane; u < nst; u += 64) tab->t[k].state[u] = tb[k].state[u];
    if (lane < 53) {
      tab->t[k].dfs[lane] = tb[k].dfs[lane];
      tab->t[k].dnb[lane] = tb[k].dnb[lane];
    }
    if (lane == 0) tab->t[k].log = tb[k].log;
  }
  constexpr uint32_t kPw = sizeof(SeqPlan) / 4;
  static_assert(sizeof(SeqPlan) % 4 == 0, "SeqPlan copy by words");
  for (uint32_t u = lane; u < kPw; u += 64) reinterpret_cast<uint32_t *>(&tab->P)[u] = reinterpret_cast<const uint32_t *>(&P)[u];
  ZT(0);
  ZT_PRINT("plan", bi % 509 == 0);
}

// Blocks per wave: 27 state machines, one per lane; 39 KiB of tables, 4
// waves per CU, so that a batch of 8192 blocks is one round of waves on 256
// CUs.  The machines are VALU-bound (one wave per SIMD): k_zc_plan hands
// them their codes, one byte per sequence, in walking order.
constexpr uint32_t kChainBlocks = 9;
constexpr uint32_t kChainSplit = 64;  // blocks with at least this many sequences: two lanes per state machine
__global__ __launch_bounds__(64) void k_zc_chain(const ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                 uint32_t *words, uint8_t *extra) {
  __shared__ FseCTL tb[3 * kChainBlocks];
  const uint32_t lane = lane_id();
  const uint64_t g0 = (uint64_t)blockIdx.x * kChainBlocks;
  ZT_DECL;
  for (uint32_t j = 0; j < kChainBlocks && g0 + j < nblk; ++j) {
    const uint64_t b = g0 + j;
    if (blocks[b].nseq == 0) continue;
    const ZcSeqTab *tab = seq_tab(extra, b);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      FseCTL &d = tb[3 * j + k];
      const uint32_t lg = tab->t[k].log, nst = 1u << lg;
      for (uint32_t u = lane; u < nst / 2; u += 64)
        reinterpret_cast<uint32_t *>(d.state)[u] = reinterpret_cast<const uint32_t *>(tab->t[k].state)[u];
      if (lane < 53) {
        d.dfs[lane] = tab->t[k].dfs[lane];
        d.dnb[lane] = tab->t[k].dnb[lane];
      }
    }
  }
  __syncthreads();
  ZT(0);
  // Two lanes per state machine: lane jk (< 27) walks the first half of its
  // block's sequences from the true initial state, lane 27 + jk the second
  // half from a guessed one (the initial state of the half's first code, as
  // if the stream began there), so the wave's dependent LDS chain is half as
  // long.  The second lane then re-walks its half from the true state beside
  // the guessed walk until the two states agree (an encoder's state map is
  // many-to-one: they agree within a few codes), rewriting those records.
  const uint32_t half = lane >= 3 * kChainBlocks ? 1u : 0u, jk = lane - half * 3 * kChainBlocks;
  const uint32_t j = min(jk / 3, kChainBlocks - 1), k = jk % 3;
  const uint64_t b = g0 + j;
  const bool act = lane < 6 * kChainBlocks && b < nblk;
  const uint64_t bq = act ? b : 0;  // (inactive lanes: block 0's addresses, nothing stored)
  const ZcBlock Bq = blocks[bq];
  const uint32_t ns = act ? Bq.nseq : 0u;
  const bool split = ns >= kChainSplit;
  const uint32_t h = split ? ns / 2 : ns;                       // half 0: codes [1, h), half 1: [h, ns)
  const uint32_t m_lo = half ? h : 1u, m_hi = half ? (split ? ns : h) : h;
  const uint32_t nsl = m_hi > m_lo ? m_hi - m_lo : 0u;
  const FseCTL &ct = tb[3 * j + k];
  // type k's state records, one 16-bit word per sequence (sequence order)
  uint16_t *rec = blk_recs(words, extra, Bq, bq) + k * rec_cap(Bq);
  const uint8_t *cd = seq_codes(stage, Bq, bq, k);  // codes in walking order: cd[m] = sequence ns - 1 - m
  const uint8_t *cdl = cd + m_lo;
  // 16 sequences per batch: codes of batch t in a register quad, of batch
  // t + 1 in flight (a load outside the compiler's wait counting, waited
  // for after the batch's steps, before its records are stored; 16 steps of
  // the chain cover the load's latency, 8 did not)
  auto issue = [&](uint32_t m0) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(cdl + m0) : "memory");
    return v;
  };
  auto init_state = [&](uint32_t c) {  // the state after a stream's first code (no bits)
    const uint32_t dnb = ct.dnb[c], nb = (dnb + (1u << 15)) >> 16;
    return (uint32_t)ct.state[((((nb << 16) - dnb)) >> nb) + ct.dfs[c]];
  };
  const int32_t top = wave_max((int32_t)nsl);  // (the wave's longest half sets the batch count)
  uint32_t state = 0, guess = 0;
  if (ns && (half == 0 || split)) {
    state = init_state(cd[half ? h - 1 : 0]);
    guess = state;
    if (half == 0) rec[ns - 1] = 0;  // the last sequence: the initial state (no bits)
  }
  // one batch: the codes in cq (waited for), the next batch's requested into
  // nq; the loop alternates two register quads, so that no register with a
  // load in flight is ever copied
  uint32_t sbits = 0;
  auto batch = [&](int32_t m0, u32x4 &cq, u32x4 &nq) {
    uint32_t dn[16];
    int32_t df[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t c = (cq[u >> 2] >> (8 * (u & 3))) & 63u;
      dn[u] = ct.dnb[c];
      df[u] = ct.dfs[c];
    }
    nq = issue((uint32_t)m0 + 16);
    uint32_t r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t nb = (state + dn[u]) >> 16;
      r[u] = nb | (state & ((1u << nb) - 1u)) << 4;
      const uint32_t nxt = ct.state[((state >> nb) + (uint32_t)df[u]) & 511u];
      const bool in = m0 + u < (int32_t)nsl;
      state = in ? nxt : state;
      sbits += in ? nb : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(nq)::"memory");
    if (m0 + 16 <= (int32_t)nsl) {  // a whole batch: its 16 records are 32 contiguous bytes (r[15] first)
      const u32x4 v0 = {r[15] | r[14] << 16, r[13] | r[12] << 16, r[11] | r[10] << 16, r[9] | r[8] << 16};
      const u32x4 v1 = {r[7] | r[6] << 16, r[5] | r[4] << 16, r[3] | r[2] << 16, r[1] | r[0] << 16};
      uint16_t *d = rec + (ns - 1 - (m_lo + (uint32_t)m0 + 15));  // (2-byte aligned: gfx950 stores a
      asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(d), "v"(v0) : "memory");  // misaligned
      asm volatile("global_store_dwordx4 %0, %1, off offset:16" ::"v"(d), "v"(v1) : "memory");  // quad as is)
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (m0 + u < (int32_t)nsl) rec[ns - 1 - (m_lo + (uint32_t)(m0 + u))] = (uint16_t)r[u];
    }
  };
  u32x4 qa = issue(0), qb;
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(qa)::"memory");
  for (int32_t m0 = 0; m0 < top; m0 += 32) {
    batch(m0, qa, qb);
    batch(m0 + 16, qb, qa);
  }
  // the first half's final state and bits to the second half's lane
  const uint32_t src = (half ? jk : lane) * 4;
  const uint32_t s_true = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)state);
  const uint32_t bits0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)sbits);
  if (act && half && split) {
    // re-walk from the true state beside the guessed walk until they agree
    uint32_t st = s_true, sg = guess;
    for (uint32_t m = h; m < ns && st != sg;) {
      const u32x4 q = *reinterpret_cast<const u32x4 *>(cd + m);  // (16 codes; the slack covers the end)
      for (int u = 0; u < 16 && m < ns && st != sg; ++u, ++m) {
        const uint32_t c = (q[u >> 2] >> (8 * (u & 3))) & 63u, dn = ct.dnb[c], df = (uint32_t)ct.dfs[c];
        const uint32_t nt = (st + dn) >> 16, ng = (sg + dn) >> 16;
        rec[ns - 1 - m] = (uint16_t)(nt | (st & ((1u << nt) - 1u)) << 4);
        sbits += nt - ng;
        st = ct.state[((st >> nt) + df) & 511u];
        sg = ct.state[((sg >> ng) + df) & 511u];
      }
    }
    if (st != sg) state = st;  // (never agreed: the true walk ran to the end)
  }
  if (act && ns && (half ? split : !split)) {  // the walk that ends at the block's last code
    seq_tab(extra, b)->fin[k] = state;
    seq_tab(extra, b)->sbits[k] = sbits + (half ? bits0 : 0u);
  }
  ZT(1);
  ZT_PRINT("chain", blockIdx.x % 97 == 0);
}

__device__ __forceinline__ void or_bits(uint32_t *w, uint32_t bit, uint64_t lo, uint64_t hi, uint32_t nbits) {
  // bits [bit, bit + nbits) of a little-endian stream of 32-bit words = the
  // low nbits of hi:lo (nbits <= 96)
  const uint32_t sh = (uint32_t)(bit & 31);
  uint32_t *q = w + (bit >> 5);
  const uint64_t a = lo << sh, b = (hi << sh) | (sh ? lo >> (64 - sh) : 0), c = sh ? hi >> (64 - sh) : 0;
  const uint32_t words = (sh + nbits + 31) >> 5;
  const uint32_t v[4] = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < words && v[k]) atomicOr(q + k, v[k]);
  if (words > 4 && (uint32_t)c) atomicOr(q + 4, (uint32_t)c);
}

__global__ __launch_bounds__(64) void k_zc_encode(ZcBlock *blocks, uint64_t nblk, uint8_t *stage,
                                                  uint32_t *words, uint8_t *extra, uint64_t *piece) {
  MCDC_VGPR_PAD(40);  // (not an exact fill)
  constexpr uint32_t kWbWords = 512 + 64 * 96 / 32 + 8;  // 512 words + a batch's bits + slack
  __shared__ uint32_t wb[kWbWords];
  const uint32_t lane = lane_id();
  const uint64_t bi = blockIdx.x;
  if (bi == 0 && lane == 0) piece[nblk] = 0;
  if (bi >= nblk) return;
  const ZcBlock B = blocks[bi];
  const uint32_t ns = B.nseq;
  const uint64_t *sq = blk_seqs(words, B);
  // the state records: three arrays of rec_cap 16-bit words (LL, OF, ML), by sequence
  const uint16_t *rec = blk_recs(words, extra, B, bi);
  const uint32_t rcap = rec_cap(B);
  uint8_t *st = blk_slot(stage, B, bi);
  uint32_t csize = 0;
  if (ns || B.lsize) {  // (no sequences but a Huffman / RLE section: a literals-only block)
    const uint32_t at = B.lsize ? B.lsize : kLitHdr + B.nlit;  // the literals section (k_zc_huff / raw)
    if (!B.lsize && lane == 0) put_raw_lit_header(st, B.nlit);
    if (ns == 0) {
      if (lane == 0) st[at] = 0;  // Number_of_Sequences 0
      csize = at + 1 < B.len ? at + 1 : 0;
    } else {
      ZT_DECL;
      const ZcSeqTab *tab = seq_tab(extra, bi);
      const uint32_t ndesc = tab->P.ndesc;
      // the section: header, then the bitstream from a 4-byte aligned word base
      const uint32_t cnt = ns < 128 ? 1u : ns < 0x7F00 ? 2u : 3u;
      const uint32_t hsz = cnt + 1 + ndesc;
      uint8_t *bs0 = st + at + hsz;
      const uint32_t pre_bits = (uint32_t)((uintptr_t)bs0 & 3) * 8;  // stream bit 0 inside the first word
      uint32_t *w0 = reinterpret_cast<uint32_t *>((uintptr_t)bs0 & ~(uintptr_t)3);
      // bits per sequence and offsets (writing order: the last sequence first)
      const uint32_t tl0 = tab->t[0].log, tl1 = tab->t[1].log, tl2 = tab->t[2].log;
      // the total (state bits from k_zc_chain, extra bits from k_zc_plan), to
      // size the stream and choose raw or compressed
      const uint64_t tot = (uint64_t)tab->xbits + tab->sbits[0] + tab->sbits[1] + tab->sbits[2];
      const uint64_t all_bits = tot + tl0 + tl1 + tl2 + 1;  // + final states + end mark
      const uint32_t nbytes = (uint32_t)((all_bits + 7) / 8);
      const uint32_t total = at + hsz + nbytes;
      if (total < B.len) {
        // The bitstream, 64 sequences at a time: their bits OR-ed into an LDS
        // buffer at offsets from a wave scan (a batch is at most 64 x 96
        // bits); when the buffer holds 512 words they go out with plain
        // stores and the partial last word moves to its front.  The first
        // word keeps the bytes before the stream (the header's, written
        // last, or the literals' when the header is short).  A batch's
        // sequences and records are requested during the batch before,
        // outside the compiler's wait counting (see ald16s).
        for (uint32_t k = lane; k < kWbWords; k += 64) wb[k] = 0;
        __syncthreads();
        if (lane == 0) wb[0] = w0[0] & (pre_bits ? (1u << pre_bits) - 1u : 0u);
        uint32_t cb = pre_bits, wi = 0;  // bits in the buffer; the buffer's first word in the slot
        auto flush = [&](bool all) {     // whole words out (all: the partial last one too)
          const uint32_t nwords = all ? (cb + 31) >> 5 : cb >> 5;
          __syncthreads();
          for (uint32_t k = lane; k < nwords; k += 64) w0[wi + k] = wb[k];
          if (all) return;
          const uint32_t part = wb[nwords];
          __syncthreads();
          for (uint32_t k = lane; k <= nwords; k += 64) wb[k] = 0;
          __syncthreads();
          if (lane == 0) wb[0] = part;
          cb &= 31;
          wi += nwords;
        };
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        auto issue = [&](int32_t b1, u32x2 &q, uint32_t &r0, uint32_t &r1, uint32_t &r2) {
          const int32_t i = b1 - 1 - (int32_t)lane, ic = i >= 0 ? i : 0;
          asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(q) : "v"(sq + ic) : "memory");
          asm volatile("global_load_ushort %0, %1, off" : "=v"(r0) : "v"(rec + ic) : "memory");
          asm volatile("global_load_ushort %0, %1, off" : "=v"(r1) : "v"(rec + rcap + ic) : "memory");
          asm volatile("global_load_ushort %0, %1, off" : "=v"(r2) : "v"(rec + 2 * rcap + ic) : "memory");
        };
        auto batch = [&](int32_t b1, u32x2 &qv, uint32_t &r0, uint32_t &r1, uint32_t &r2) {
          const int32_t b0 = b1 > 64 ? b1 - 64 : 0;
          const int32_t i = b1 - 1 - (int32_t)lane;  // lane 0 the batch's last sequence (written first)
          const uint64_t q = (uint64_t)qv.y << 32 | qv.x, rr = (uint64_t)r2 << 32 | r1 << 16 | r0;
          issue(b1 - 64, qv, r0, r1, r2);  // the next batch's, waited for at this one's end
          uint64_t lo = 0, hi = 0;
          uint32_t nb = 0;
          if (i >= b0) {
            const uint32_t ll = seq_ll(q), mb = seq_ml(q) - 3, ob = seq_ov(q);
            const uint32_t llc = ll_code(ll), mlc = ml_code(mb), ofc = highbit(ob);
            auto put = [&](uint64_t v, uint32_t n) {  // append n bits (n <= 32)
              v &= n >= 64 ? ~0ull : ((1ull << n) - 1);
              if (nb < 64) {
                lo |= v << nb;
                if (nb + n > 64) hi |= v >> (64 - nb);
              } else {
                hi |= v << (nb - 64);
              }
              nb += n;
            };
            // states in writing order OF, ML, LL (none for the last sequence)
            put((rr >> 20) & 0xFFF, (uint32_t)((rr >> 16) & 15));
            put((rr >> 36) & 0xFFF, (uint32_t)((rr >> 32) & 15));
            put((rr >> 4) & 0xFFF, (uint32_t)(rr & 15));
            put(ll, ll_bits(llc));
            put(mb, ml_bits(mlc));
            put(ob, ofc);
          }
          const uint32_t incl = wave_incl_sum(nb, lane);  // inclusive prefix in lane order = writing order
          if (nb) or_bits(wb, cb + incl - nb, lo, hi, nb);
          cb += (uint32_t)lane63((int32_t)incl);
          if (cb >= 512 * 32) flush(false);
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(qv), "+v"(r0), "+v"(r1), "+v"(r2)::"memory");
        };
        u32x2 qa;
        uint32_t ra0, ra1, ra2;
        issue((int32_t)ns, qa, ra0, ra1, ra2);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(qa), "+v"(ra0), "+v"(ra1), "+v"(ra2)::"memory");
        for (int32_t b1 = (int32_t)ns; b1 > 0; b1 -= 64) batch(b1, qa, ra0, ra1, ra2);
        // final states (ML, OF, LL: log bits each), the end mark, the last words
        const uint32_t f0 = tab->fin[0], f1 = tab->fin[1], f2 = tab->fin[2];  // final states of LL, OF, ML
        {
          const uint32_t fb = tl2 + tl1 + tl0 + 1;
          const uint64_t v = (uint64_t)(f2 & ((1u << tl2) - 1)) | (uint64_t)(f1 & ((1u << tl1) - 1)) << tl2 |
                             (uint64_t)(f0 & ((1u << tl0) - 1)) << (tl2 + tl1) | 1ull << (tl2 + tl1 + tl0);
          __syncthreads();
          if (lane == 0) or_bits(wb, cb, v, 0, fb);
          cb += fb;
          flush(true);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // (same wave: agent scope would write back the L2)
        if (lane == 0) {
          uint8_t *h = st + at;  // Number_of_Sequences, Symbol_Compression_Modes, descriptions
          if (cnt == 1) {
            h[0] = (uint8_t)ns;
          } else if (cnt == 2) {
            h[0] = (uint8_t)((ns >> 8) + 0x80);
            h[1] = (uint8_t)ns;
          } else {
            h[0] = 0xFF;
            h[1] = (uint8_t)(ns - 0x7F00);
            h[2] = (uint8_t)((ns - 0x7F00) >> 8);
          }
          h[cnt] = (uint8_t)tab->P.modes;
          for (uint32_t k = 0; k < ndesc; ++k) h[cnt + 1 + k] = tab->P.desc[k];
        }
        csize = total;
      }
      ZT(2);
      ZT_PRINT("encode", bi % 509 == 0);
    }
  }
  if (lane == 0) {
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
  const uint8_t *s = comp ? blk_slot(const_cast<uint8_t *>(stage), B, bi) : base + B.src;
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
                       uint64_t *wcnt, uint64_t *wfirst, uint32_t *err, uint64_t *bound, uint8_t *cls, void *tmp,
                       size_t tmp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(k_zc_nblocks, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, chunks, n, nbytes, cnt,
                     wcnt, err, bound, cls);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, cnt, first, (int)n + 1, st);
  b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, wcnt, wfirst, (int)n + 1, st);
}

void launch_zc_batch(const uint8_t *base, uint64_t nbytes, const DevChunk *chunks, const uint64_t *first,
                     const uint64_t *wfirst, uint64_t c0, uint64_t c1, uint64_t b0, uint64_t nblk, ZcBlock *blocks,
                     uint8_t *stage, uint32_t *words, uint8_t *extra, const zs::ZTables &T, uint64_t *piece, uint64_t *poff,
                     uint64_t *obase,
                     uint8_t *out, uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st, bool huf,
                     hipEvent_t final_after, hipEvent_t final_done, bool far, uint64_t nseg, const uint64_t *nsmall) {
  if (nblk == 0) return;
  if (nseg == 0 || nseg > nblk) nseg = nblk, nsmall = nullptr;  // (every segment's first record is in order[0, nseg))
  hipLaunchKernelGGL(k_zc_blocks, dim3((unsigned)((c1 - c0 + 255) / 256)), dim3(256), 0, st, chunks, first, wfirst,
                     c0, c1, b0, blocks);
  // (piece, nblk + 1 words of 8 bytes, is free until k_zc_encode: the
  // finder's segment order and the parse's block order)
  uint32_t *order = reinterpret_cast<uint32_t *>(piece), *porder = order + nblk;
  hipLaunchKernelGGL(k_zc_segorder, dim3(1), dim3(1024), 0, st, blocks, nblk, order, porder);
  // (the far tables and ballots live in extra[], free until k_zc_plan)
  static_assert(kZcFarSlots * 4 + kZcFarBallots * 8 <= kZcExtra, "far tables in extra[]");
  uint32_t *ftab = reinterpret_cast<uint32_t *>(extra);
  uint64_t *fbits = reinterpret_cast<uint64_t *>(ftab + nblk * kZcFarSlots);
  // the probe over the segments of longer chunks (the front of the order),
  // the small chunks (one block) by k_zc_small per size class (then the
  // order's back, longest first: kZcSmallClass)
  const uint64_t *ns_ = nsmall;
  const uint64_t nsmall_all = ns_ ? ns_[0] + ns_[1] + ns_[2] + ns_[3] : 0;
  const uint64_t nprobe = nsmall_all <= nseg ? nseg - nsmall_all : nseg;
  if (nprobe)
    hipLaunchKernelGGL(k_zc_probe, dim3((unsigned)nprobe), dim3(kProbeThreads), 0, st, base, nbytes, blocks, nblk,
                       order, ftab, fbits);
  if (nsmall_all && nsmall_all <= nseg) {
    const uint32_t *os = order + nprobe;
    if (ns_[0])
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_zc_small<4, 13, 12, 32768>), dim3((unsigned)ns_[0]), dim3(256), 0, st, base,
                         nbytes, blocks, nblk, words, os);
    if (ns_[1])
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_zc_small<4, 12, 11, 16384>), dim3((unsigned)ns_[1]), dim3(256), 0, st, base,
                         nbytes, blocks, nblk, words, os + ns_[0]);
    if (ns_[2])
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_zc_small<2, 12, 11, 8192>), dim3((unsigned)ns_[2]), dim3(128), 0, st, base,
                         nbytes, blocks, nblk, words, os + ns_[0] + ns_[1]);
    if (ns_[3])
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_zc_small<1, 11, 10, 4096>), dim3((unsigned)ns_[3]), dim3(64), 0, st, base,
                         nbytes, blocks, nblk, words, os + ns_[0] + ns_[1] + ns_[2]);
  }
  const dim3 gfar((unsigned)((nblk * kZcFarBallots + 3) / 4));
  if (far)
    hipLaunchKernelGGL(k_zc_far, gfar, dim3(256), 0, st, base, nbytes, blocks, nblk, ftab, fbits, words, true);
  // the finder over the segments of chunks of more than one block (the small
  // chunks' words are k_zc_small's); segments and blocks k_zc_probe /
  // k_zc_small found hopeless return at once, here and in every kernel after
  const uint64_t nbig = nprobe, nwork = nblk;
  if (nbig)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(MCDC_ZC_FIND_BIG), dim3((unsigned)nbig), dim3(kFindThreads), 0, st, base, nbytes,
                       blocks, nblk, words, order);
  if (far && nwork)
    hipLaunchKernelGGL(k_zc_far, gfar, dim3(256), 0, st, base, nbytes, blocks, nblk, ftab, fbits, words, false);
  if (nwork) {
    hipLaunchKernelGGL(k_zc_parse, dim3((unsigned)nwork), dim3(64), 0, st, base, nbytes, blocks, nblk, words, stage,
                       porder);
    if (huf)
      hipLaunchKernelGGL(k_zc_huff, dim3((unsigned)nwork), dim3(64), 0, st, base, nbytes, blocks, nblk, stage, words,
                         porder);
    hipLaunchKernelGGL(k_zc_plan, dim3((unsigned)nwork), dim3(64), 0, st, blocks, nblk, stage, words, extra, T, porder);
  }
  hipLaunchKernelGGL(k_zc_chain, dim3((unsigned)((nblk + kChainBlocks - 1) / kChainBlocks)), dim3(64), 0, st, blocks,
                     nblk, stage, words, extra);
  hipLaunchKernelGGL(k_zc_encode, dim3((unsigned)nblk), dim3(64), 0, st, blocks, nblk, stage, words, extra, piece);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, piece, poff, (int)nblk + 1, st);
  if (final_after) (void)hipStreamWaitEvent(st, final_after, 0);
  hipLaunchKernelGGL(k_zc_final, dim3((unsigned)nblk), dim3(64), 0, st, base, blocks, nblk, stage, poff, obase, out,
                     ext);
  hipLaunchKernelGGL(k_zc_advance, dim3(1), dim3(64), 0, st, obase, poff, nblk);
  if (final_done) (void)hipEventRecord(final_done, st);
}

}  // namespace mcdc
