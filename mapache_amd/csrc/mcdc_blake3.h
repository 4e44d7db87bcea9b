// mcdc_blake3.h — launch wrappers of the GPU chunk-ID kernels (BLAKE3 of
// every chunk of a boundary list), used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcdc_internal.h"

namespace mcdc {

// device temp bytes of the group-offset scan over nchunks + 1 entries
size_t b3_tmp_bytes(uint64_t nchunks);
// upper bound of the 16-KiB leaf groups of a boundary list covering total_bytes
uint64_t b3_group_bound(uint64_t total_bytes, uint64_t nchunks);
// device words of the tail-group histogram and bin cursors (hist argument)
constexpr size_t kB3HistWords = 520;  // tail bins, bin cursors, wide-tree list count and draw counter
// gcnt[0..n] (n + 1 entries), goff[0..n] = exclusive prefix of the packed
// counts (low 32 bits full groups, high 32 bits tail groups);
// b3_groups_total(goff[n]) = groups.  Chunks outside [0, nbytes) set *err and
// get no groups.  hist: kB3HistWords device words.
void launch_b3_prepare(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *gcnt, uint64_t *goff,
                       uint32_t *hist, uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t stream);
// groups of a packed count / offset
uint64_t b3_groups_total(uint64_t packed);
// ids[32 * i] = BLAKE3(base[chunks[i].offset, + chunks[i].length)); group_bound
// sizes the grid (b3_group_bound, exact for disjoint chunks).  When the group
// total exceeds it (overlapping or repeated chunks) the kernels write nothing
// and the caller re-runs with group_bound = the total.  hist: as prepared.
// gcnt: the prepare step's count buffer (free after its scan; reused for the
// list of chunks the wave-parallel tree takes).
void launch_b3_hash(const uint8_t *base, const DevChunk *chunks, uint64_t n, const uint64_t *goff,
                    uint64_t group_bound, uint32_t *hist, uint32_t *owner, uint32_t *nodes, uint8_t *ids,
                    uint64_t *gcnt, hipStream_t stream);

}  // namespace mcdc
