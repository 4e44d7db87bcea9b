// mcdc_zcomp.h — launch wrappers of the GPU zstd compressor (mcdc_zcomp.hip),
// used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcdc_internal.h"
#include "mcdc_zstd.h"

namespace mcdc {

constexpr uint64_t kZcBlock = 16384;               // zstd block: 16 KiB of one chunk
constexpr uint32_t kZcSeqCap = 4096;               // sequences per block: a 16 KiB block of 4-byte matches
constexpr uint64_t kZcSlot = kZcBlock + 64;        // staging bytes per block
#ifndef MCDC_ZC_RUN
#define MCDC_ZC_RUN 2  // (compile-time A/B knob; tools/build_variants.py)
#endif
constexpr uint32_t kZcRun = MCDC_ZC_RUN;           // blocks parsed in a row by one wave (table kept)
constexpr uint64_t kZcBatchBlocks = 65536;         // blocks per batch (1 GiB; more for a longer chunk)

struct ZcBlock {
  uint64_t src;                 // chunk bytes [src, src + len) of the input
  uint32_t len, chunk, b, nb;   // block b of nb of chunk
  uint32_t nlit, nseq, csize;   // parse result; csize 0 = stored raw
  uint32_t lsize;               // literals section already in the staging slot (Huffman / RLE), 0 = raw literals
};

size_t zc_tmp_bytes(uint64_t n);
// cnt[i] = blocks of chunk i (n + 1 entries), first = exclusive prefix; chunks
// outside [0, nbytes) or of 2 GiB or more set *err; bound[0] += sum of the raw
// frame sizes (the output capacity that always suffices).
void launch_zc_nblocks(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *cnt, uint64_t *first,
                       uint32_t *err, uint64_t *bound, void *tmp, size_t tmp_bytes, hipStream_t st);
// one batch: the chunks [c0, c1), blocks [b0, b0 + nblk)
void launch_zc_batch(const uint8_t *base, const DevChunk *chunks, const uint64_t *first, uint64_t c0, uint64_t c1,
                     uint64_t b0, uint64_t nblk, ZcBlock *blocks, uint8_t *stage, uint64_t *seqs,
                     const zs::ZTables &T, uint64_t *piece, uint64_t *poff, uint64_t *obase, uint8_t *out,
                     uint64_t *ext, void *tmp, size_t tmp_bytes, hipStream_t st, bool huf = true);

}  // namespace mcdc
