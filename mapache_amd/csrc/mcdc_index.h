// mcdc_index.h — launch wrappers of the GPU blob dedup index (which chunk IDs
// of a batch are new), used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcdc_internal.h"

namespace mcdc {

// The index: n IDs sorted by their first 8 bytes (little-endian u64).
struct IdxIndexView {
  const uint64_t *pfx;
  const uint8_t *ids;
  uint64_t size;
};

// Per-call scratch (n = batch size): keys/pos n entries each, skeys/spos n,
// sflag n, count 2 words, tmp idx_tmp_bytes(n).
struct IdxScratch {
  uint64_t *keys, *skeys;
  uint32_t *pos, *spos;
  uint8_t *sflag;
  uint64_t *count;  // [0] new IDs (keys), [1] the same (positions)
  void *tmp;
  size_t tmp_bytes;
};

size_t idx_tmp_bytes(uint64_t n);
// is_new[i] = 1 iff ids[32 i, +32) is neither in the index nor equal to an
// earlier ID of the batch; afterwards s.keys / s.pos hold the new IDs'
// prefixes / batch positions in prefix order and s.count[0] their number.
void launch_idx_mark(const uint8_t *ids, uint64_t n, const IdxIndexView &ix, const IdxScratch &s, uint8_t *is_new,
                     hipStream_t st);
// opfx / oids (ix.size + m entries) = the index merged with the m new IDs.
void launch_idx_merge(const uint8_t *ids, uint64_t m, const IdxIndexView &ix, const IdxScratch &s, uint64_t *opfx,
                      uint8_t *oids, hipStream_t st);
// out = the chunks whose is_new flag is set, in order; *count their number.
void launch_idx_compact_chunks(const DevChunk *chunks, const uint8_t *is_new, uint64_t n, DevChunk *out,
                               uint64_t *count, void *tmp, size_t tmp_bytes, hipStream_t st);

}  // namespace mcdc
