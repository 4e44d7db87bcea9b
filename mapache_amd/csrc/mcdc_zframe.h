// mcdc_zframe.h — launch wrappers of the GPU zstd raw-block frame writer,
// used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcdc_internal.h"

namespace mcdc {

size_t zframe_tmp_bytes(uint64_t n);
// sz[i] = frame i's size rounded up to 16 bytes (n + 1 entries), off = their
// exclusive prefix (off[n] = output bytes); chunks outside [0, nbytes) set *err.
void launch_zframe_sizes(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *sz, uint64_t *off,
                         uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t st);
// frames into out at off[i]; ext[2 i], ext[2 i + 1] = (offset, length) of frame i
void launch_zframe_write(const uint8_t *base, const DevChunk *chunks, uint64_t n, const uint64_t *off, uint8_t *out,
                         uint64_t *ext, hipStream_t st);

// Gather: segment i = src[ext[3 i], + ext[3 i + 2]) to dst + ext[3 i + 1]
// (dst + ext[3 i + 1] congruent to src + ext[3 i] modulo 16: whole 16-byte
// loads and stores between a byte head and tail).  One workgroup per segment.
void launch_gather(const uint8_t *src, const uint64_t *ext, uint64_t n, uint8_t *dst, hipStream_t st);

}  // namespace mcdc
