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
constexpr uint64_t kZcSlot = kZcBlock + 64;        // staging bytes per block
constexpr uint64_t kZcStagePad = 16384;            // staging bytes after a batch's last slot (k_zc_chain's prefetch)
constexpr uint32_t kZcSegBlocks = 8;               // blocks of a chunk one match-finder workgroup covers
constexpr uint32_t kZcPrime = 65536;               // bytes before a segment the finder re-inserts

struct ZcBlock {
  uint64_t src;                 // chunk bytes [src, src + len) of the input
  uint32_t len, chunk, b, nb;   // block b of nb of chunk
  uint32_t nlit, nseq, csize;   // parse result; csize 0 = stored raw
  uint32_t lsize;               // literals section already in the staging slot (Huffman / RLE), 0 = raw literals
  uint32_t flags;               // kZcRaw: k_zc_probe found the block hopeless (stored raw, no finder / parse)
};
constexpr uint32_t kZcRaw = 1u;
constexpr uint32_t kZcSegRaw = 2u;  // (on a segment's first record) every block of the segment is kZcRaw
// Far matches (k_zc_probe / k_zc_far): per block record kZcFarSlots table
// entries (a segment of kZcSegBlocks records owns kZcSegBlocks x kZcFarSlots
// slots) and kZcBlock / 1024 anchor ballots, carved from the batch's staging
// slots (free until k_zc_parse).
constexpr uint32_t kZcFarSlots = 512;
constexpr uint32_t kZcFarBallots = (uint32_t)(kZcBlock / 1024);

size_t zc_tmp_bytes(uint64_t n);
// cnt[i] = blocks of chunk i (n + 1 entries), first = exclusive prefix; chunks
// outside [0, nbytes) or of 2 GiB or more set *err; bound[0] += sum of the raw
// frame sizes (the output capacity that always suffices); cls[i] = the
// k_zc_small class of a chunk of one block (zc_small_class), 4 for longer.
void launch_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint64_t *first,
                       uint32_t *err, uint64_t *bound, uint8_t *cls, void *tmp, size_t tmp_bytes, hipStream_t st);
// Scratch per batch of nblk blocks (bytes), all device memory of the context:
//   blocks nblk x sizeof(ZcBlock), stage nblk x kZcSlot + kZcStagePad (also
//   the far tables until k_zc_parse, and the sequence codes), match words
//   (nblk x kZcBlock + 1024) x 4 (also the sequences, k_zc_huff's section,
//   the FSE tables and the state records after k_zc_parse), piece / poff
//   (nblk + 1) x 8: ~5 x the batch's input in all, 2.5 GiB for a batch set of
//   16384 blocks.  A batch holds whole chunks, at most the context's
//   "zc_batch_blocks" (two sets of half that on two streams) unless one
//   chunk is longer (1 GiB: 7 x 2^18 words).
// one batch: the chunks [c0, c1), blocks [b0, b0 + nblk)
void launch_zc_batch(const uint8_t *base, uint64_t nbytes, const DevChunk *chunks, const uint64_t *first, uint64_t c0,
                     uint64_t c1, uint64_t b0, uint64_t nblk, ZcBlock *blocks, uint8_t *stage,
                     uint32_t *words, const zs::ZTables &T, uint64_t *piece, uint64_t *poff, uint64_t *obase, uint8_t *out,
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
