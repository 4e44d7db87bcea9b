/*
 * fastcdc_oracle.h — CPU restatement of FastCDC v2020 as mapache calls it.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the MI355X chunker
 * in mapache_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / timed CPU
 * baseline — never as the product path.
 *
 * What it restates
 *   The reference (jLantxa/mapache @ 2025-07-18) does not contain the
 *   chunking arithmetic: it calls the external crate `fastcdc` 3.2.1
 *   (/root/reference/Cargo.toml:23, Cargo.lock:449-452, checksum
 *   bf51ceb4...f2ce6bc), module `v2020`, which is NOT vendored and cannot be
 *   built here (no rustc/cargo, no network).  This file restates the crate's
 *   published algorithm:
 *     - call site: StreamCDC::with_level(reader, MIN, AVG, MAX,
 *       Normalization::Level1)  — /root/reference/src/archiver/processor.rs:173-179
 *     - parameters: 512 KiB / 1 MiB / 8 MiB — src/global/defaults.rs:35-40
 *     - small-file gate (no CDC below MIN) — src/archiver/processor.rs:144-156
 *     - cut_gear / tables / StreamCDC buffer semantics — SURVEY.md Appendix A
 *
 * Provenance / pinning ("parity unpinned" by the reference itself)
 *   No test in /root/reference reaches the chunker (every fixture file is
 *   <= 11 B, below the 512 KiB gate).  What pins this
 *   restatement:
 *     (1) GEAR[i] = BE-u64(MD5([i]*64)[0:8]) — derived here by our own MD5,
 *         checked against sha256 91a30610...0f028f88 and four entries
 *         recalled from the crate source;
 *     (2) popcount(MASKS[k]) == k;
 *     (3) the crate's own `test_all_zeros` KAT, recalled (the crate's test
 *         file is not in the container): 10240 zero bytes at 64/256/1024
 *         give 10 chunks of 1024 with hash 14169102344523991076 — this
 *         restatement reproduces it (tests/test_oracle.py);
 *     (4) 1-byte vs 2-byte loop equivalence, StreamCDC == slice semantics.
 *   Until a real `fastcdc 3.2.1` run diffs tests/golden/, parity is stated
 *   as "vs this restatement" (DESIGN.md §Parity).
 */
#ifndef MAPACHE_FASTCDC_ORACLE_H
#define MAPACHE_FASTCDC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* crate v2020 bounds (asserts in StreamCDC::with_level / FastCDC::with_level) */
#define OC_MINIMUM_MIN 64u
#define OC_MINIMUM_MAX 1048576u
#define OC_AVERAGE_MIN 256u
#define OC_AVERAGE_MAX 4194304u
#define OC_MAXIMUM_MIN 1024u
#define OC_MAXIMUM_MAX 16777216u

typedef struct {
  uint32_t min_size, avg_size, max_size, level;
  uint64_t mask_s, mask_l, mask_s_ls, mask_l_ls;
} oc_params;

typedef struct {
  uint64_t offset, length, hash;
} oc_chunk;

/* Tables.  GEAR is derived with MD5 at first use. */
void oc_gear(uint64_t out[256]);
void oc_gear_ls(uint64_t out[256]);
void oc_masks(uint64_t out[26]);
uint32_t oc_logarithm2(uint32_t v); /* f64::log2().round() */

/* with_level: 0 on success, -1 if a crate assert would panic. */
int oc_params_init(oc_params *p, uint32_t min_size, uint32_t avg_size,
                   uint32_t max_size, uint32_t level);

/* cut_gear, the crate's 2-byte loop, literally. */
void oc_cut_gear(const oc_params *p, const uint8_t *src, size_t len,
                 uint64_t *hash, size_t *count);
/* Equivalent 1-byte formulation; same count, same hash. */
void oc_cut_gear_1byte(const oc_params *p, const uint8_t *src, size_t len,
                       uint64_t *hash, size_t *count);

/* FastCDC iterator over a whole slice.  Writes up to cap chunks, returns the
 * total number of chunks (may exceed cap: then only cap were written). */
size_t oc_chunk_slice(const oc_params *p, const uint8_t *data, size_t n,
                      oc_chunk *out, size_t cap);
/* Same, 1-byte loop. */
size_t oc_chunk_slice_1byte(const oc_params *p, const uint8_t *data, size_t n,
                            oc_chunk *out, size_t cap);

/* StreamCDC semantics: a max-sized buffer refilled from a reader that hands
 * out at most `read_quantum` bytes per read() (crate fill_buffer/drain). */
size_t oc_chunk_stream(const oc_params *p, const uint8_t *data, size_t n,
                       size_t read_quantum, oc_chunk *out, size_t cap);

/* Many independent files, each chunked from offset 0, `threads` pthreads
 * (files in parallel; the CPU baseline).  out gets each file's chunks
 * concatenated (offsets relative to the file); counts[i] per file.
 * Returns total chunk count, or (size_t)-1 if cap is too small. */
size_t oc_chunk_files(const oc_params *p, const uint8_t *const *bufs,
                      const size_t *lens, size_t nfiles, int threads,
                      oc_chunk *out, size_t cap, size_t *counts);

/* Chunk count + order-sensitive digest only (no output array; for big
 * samples).  Returns number of chunks. */
size_t oc_chunk_digest(const oc_params *p, const uint8_t *data, size_t n,
                       uint64_t *digest);

/* The counter-based stream [0, n) of `seed` (oc_fill_random) chunked as one
 * file, regenerated slab by slab (memory O(slab + max)): count, digest, and
 * the sum of lengths.  For full-size (64 GiB) parity checks. */
size_t oc_random_stream_digest(const oc_params *p, uint64_t seed, uint64_t n, size_t slab, uint64_t *digest,
                               uint64_t *sum);
/* Same, plus *hdigest = oc_hash_digest of the chunks' ChunkData.hash values. */
size_t oc_random_stream_digest_h(const oc_params *p, uint64_t seed, uint64_t n, size_t slab, uint64_t *digest,
                                 uint64_t *sum, uint64_t *hdigest);
/* Order-sensitive digest of a list of chunk hashes: fold of
 * oc_digest_step(d, index, hash). */
uint64_t oc_hash_digest(const uint64_t *hashes, size_t n);

/* Many files of counter-based streams (file i = [pos[i], pos[i] + len[i]) of
 * the stream of seeds[i]), each chunked as one file on `threads` threads:
 * per-file count, oc_chunk_digest-style boundary digest (file-relative
 * offsets) and hash digest (hdigests may be NULL).  0 ok, -1 allocation. */
int oc_random_files_digest(const oc_params *p, const uint64_t *seeds, const uint64_t *pos,
                           const uint64_t *len, size_t nfiles, int threads, uint64_t *counts,
                           uint64_t *digests, uint64_t *hdigests);

/* Counter-based byte generator shared with the device fill kernel and the
 * bench: byte i = (splitmix64_at(seed, i/8) >> 8*(i%8)) & 0xff. */
void oc_fill_random(uint8_t *dst, uint64_t pos, size_t n, uint64_t seed);
uint64_t oc_file_seed(uint64_t seed, uint64_t file_index);

/* Digest of a boundary list (order-sensitive): matches mcdc's digest. */
uint64_t oc_digest_step(uint64_t d, uint64_t offset, uint64_t length);

#ifdef __cplusplus
}
#endif
#endif
