// mcdc_zcomp.h — launch wrappers of the GPU zstd compressor (mcdc_zcomp.hip),
// used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcdc_internal.h"
#include "mcdc_zstd.h"

namespace mcdc {

constexpr uint64_t kZcBlock = 32768;               // zstd block: 32 KiB of one chunk
constexpr uint32_t kZcSeqCap = kZcBlock / 4;       // sequences per block: every match is >= 4 bytes
constexpr uint64_t kZcStagePad = 16384;            // staging bytes after a batch's last slot (k_zc_chain's prefetch)
constexpr uint64_t kZcExtra = 6144;                // per block: far tables, then the FSE tables (+ short blocks' records)
// A block's scratch span in words (= bytes of its staging slot, + 64): its
// length rounded up to 64, at least 64; a chunk's span (the sum over its
// blocks: every block but the last is kZcBlock) is zc_span of its length.
__host__ __device__ inline uint64_t zc_span(uint64_t len) { return len > 64 ? (len + 63) & ~63ull : 64ull; }
constexpr uint32_t kZcSegBlocks = 8;               // blocks of a chunk one match-finder workgroup covers
constexpr uint32_t kZcPrime = 65536;               // bytes before a segment the finder re-inserts

struct ZcBlock {
  uint64_t src;                 // chunk bytes [src, src + len) of the input
  uint32_t len, chunk, b, nb;   // block b of nb of chunk
  uint32_t nlit, nseq, csize;   // parse result; csize 0 = stored raw
  uint32_t lsize;               // literals section already in the staging slot (Huffman / RLE), 0 = raw literals
  uint32_t flags;               // kZcRaw: k_zc_probe found the block hopeless (stored raw, no finder / parse)
  uint32_t w0;                  // its first word in the batch's words; its staging slot at w0 + 64 x its index
};
static_assert(sizeof(ZcBlock) == 48, "block record");
constexpr uint32_t kZcRaw = 1u;
constexpr uint32_t kZcSegRaw = 2u;  // (on a segment's first record) every block of the segment is kZcRaw
// Far matches (k_zc_probe / k_zc_far): per block record kZcFarSlots table
// entries (a segment of kZcSegBlocks records owns kZcSegBlocks x kZcFarSlots
// slots) and kZcBlock / 1024 anchor ballots, carved from the batch's extra[]
// (free until k_zc_plan).
constexpr uint32_t kZcFarSlots = 512;
constexpr uint32_t kZcFarBallots = (uint32_t)(kZcBlock / 1024);

size_t zc_tmp_bytes(uint64_t n);
// cnt[i] = blocks of chunk i (n + 1 entries), first = exclusive prefix;
// wcnt[i] = its words (zc_span), wfirst = exclusive prefix; chunks outside
// [0, nbytes) or of 2 GiB or more set *err; bound[0] += sum of the raw frame
// sizes (the output capacity that always suffices); cls[i] = the k_zc_small
// class of a chunk of one block (zc_small_class), 4 for longer.
void launch_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint64_t *first,
                       uint64_t *wcnt, uint64_t *wfirst, uint32_t *err, uint64_t *bound, uint8_t *cls, void *tmp,
                       size_t tmp_bytes, hipStream_t st);
// Scratch per batch of nblk blocks spanning nw words (bytes), all device
// memory of the context, packed by the blocks' lengths (zc_span):
//   blocks nblk x sizeof(ZcBlock); match words (nw + 1024) x 4 (also the
//   sequences, k_zc_huff's section and the state records after
//   k_zc_parse); stage nw + 64 nblk + kZcStagePad (literals, the sequence
//   codes, the encoded block); extra nblk x kZcExtra (far tables, then the
//   FSE tables); piece / poff (nblk + 1) x 8.  ~5 bytes per input byte, and
//   blocks shorter than 32 KiB cost in proportion.  Batches are whole chunks
//   within the context's "zc_batch_blocks" x 32 KiB of words and twice that
//   many blocks (two sets of half each on two streams), unless one chunk is
//   longer (mcdc_api.hip: zc_batches).
// one batch: the chunks [c0, c1), blocks [b0, b0 + nblk)
void launch_zc_batch(const uint8_t *base, uint64_t nbytes, const DevChunk *chunks, const uint64_t *first,
                     const uint64_t *wfirst, uint64_t c0, uint64_t c1, uint64_t b0, uint64_t nblk, ZcBlock *blocks,
                     uint8_t *stage, uint32_t *words, uint8_t *extra, const zs::ZTables &T, uint64_t *piece, uint64_t *poff, uint64_t *obase, uint8_t *out,
                     uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st, bool huf = true,
                     hipEvent_t final_after = nullptr, hipEvent_t final_done = nullptr, bool far = true,
                     uint64_t nseg = 0, const uint64_t *nsmall = nullptr);
// Chunks of one block (<= 32 KiB) are probed and matched by k_zc_small, one
// workgroup per chunk with the chunk's bytes and its tables in LDS, in four
// size classes: chunks of up to kZcSmallClass[k] bytes and more than
// kZcSmallClass[k + 1] (k = 0 the longest).  nsmall[k]: the batch's chunks
// of class k (the host counts them from the chunk lengths).
constexpr uint32_t kZcSmallClass[5] = {32768, 16384, 8192, 4096, 0};
__host__ __device__ inline int zc_small_class(uint64_t len) {
  return len > 16384 ? 0 : len > 8192 ? 1 : len > 4096 ? 2 : 3;
}
// (final_after: the output offsets' previous update, on another stream, is
// waited for before this batch's final copy; final_done: recorded after it;
// far: some chunk is longer than one finder segment, k_zc_far runs; nseg:
// the batch's finder segments, sum of ceil(blocks / kZcSegBlocks) over its
// chunks -- the probe's and the finder's grids; 0 = one workgroup per block.
// nsmall: the batch's chunks of one block per k_zc_small class
// (kZcSmallClass), or null = every chunk through k_zc_probe and k_zc_find.
// Nothing is read back: segments and blocks found hopeless return at once in
// every later kernel, so the host never waits inside a batch)

}  // namespace mcdc
