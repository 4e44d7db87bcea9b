/*
 * mcdc.h — C ABI of the MI355X-native FastCDC v2020 chunker (libmcdc.so).
 *
 * This is the drop-in boundary for mapache's Archiver chunker.  The reference
 * has no in-tree FFI for this path: it calls the Rust crate `fastcdc` 3.2.1
 * directly at
 *     /root/reference/src/archiver/processor.rs:173-179
 *         StreamCDC::with_level(reader, MIN_CHUNK_SIZE as u32,
 *                               AVG_CHUNK_SIZE as u32, MAX_CHUNK_SIZE as u32,
 *                               Normalization::Level1)
 *     /root/reference/src/archiver/processor.rs:181-202  (`for result in chunker`)
 * with parameters from /root/reference/src/global/defaults.rs:35-40.  Each
 * entry point below states which piece of that interface it replaces; the
 * Rust-side binding a maintainer would add is in INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns an int status: MCDC_OK (0) or a negative code.
 *     No exception, panic or abort crosses this boundary; the message of the
 *     last failure on the calling thread is returned by mcdc_last_error().
 *   - The caller owns every buffer.  Output arrays are caller-allocated with a
 *     capacity; MCDC_E_CAPACITY reports the required count in *n_out.
 *   - A context (mcdc_ctx) owns one HIP device, one stream and its device
 *     workspace.  Contexts are independent (the library is re-entrant across
 *     contexts); one context must not be used by two threads at once.
 *   - Chunk boundaries are bit-identical to fastcdc::v2020 (the crate's
 *     cut_gear loop restated in oracle/), including ChunkData.hash.
 */
#ifndef MCDC_H
#define MCDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCDC_ABI_VERSION 5

/* status codes */
#define MCDC_OK 0
#define MCDC_E_INVALID (-1)  /* null pointer / bad argument                         */
#define MCDC_E_PARAMS (-2)   /* min/avg/max/level outside the crate's asserts       */
#define MCDC_E_CAPACITY (-3) /* output array too small; *n_out = required count      */
#define MCDC_E_DEVICE (-4)   /* HIP runtime error (message in mcdc_last_error)      */
#define MCDC_E_NOMEM (-5)    /* device or pinned host allocation failed              */
#define MCDC_E_TOOBIG (-6)   /* input larger than the context was created for       */
#define MCDC_E_INTERNAL (-7) /* internal consistency check failed                  */
#define MCDC_E_AUTH (-8)     /* mcdc_open_device: a blob failed authentication     */

/* fastcdc::v2020::Normalization (crate enum; Level1 is what mapache uses,
 * processor.rs:178). */
typedef enum {
  MCDC_LEVEL0 = 0,
  MCDC_LEVEL1 = 1,
  MCDC_LEVEL2 = 2,
  MCDC_LEVEL3 = 3
} mcdc_normalization;

/* The arguments of StreamCDC::with_level(source, min_size, avg_size,
 * max_size, level) — processor.rs:173-179. */
typedef struct {
  uint32_t min_size;
  uint32_t avg_size;
  uint32_t max_size;
  uint32_t level; /* mcdc_normalization */
} mcdc_params;

/* One yielded chunk: the crate's ChunkData{hash, offset, length, data} minus
 * the owned `data` Vec (the caller slices its own buffer).  `offset` is
 * relative to the start of the buffer/file it belongs to. */
typedef struct {
  uint64_t offset;
  uint64_t length;
  uint64_t hash;
} mcdc_chunk;

/* Device time of the last call on a context (HIP events on the context
 * stream).  device_ms covers the first scan kernel to the last boundary
 * written (the device-resident metric); the copies are timed separately. */
typedef struct {
  double scan_ms;      /* candidate scan kernel(s) only                  */
  double resolve_ms;   /* chain resolution + boundary emission kernels   */
  double device_ms;    /* scan_ms + resolve_ms, one event pair           */
  double h2d_ms;       /* host->device input copies (host entry points)  */
  double d2h_ms;       /* boundary list device->host                     */
  double total_ms;     /* host wall time of the whole call               */
  uint64_t bytes;      /* input bytes chunked                            */
  uint64_t chunks;     /* chunks produced                                */
  uint64_t scan_launches; /* number of scan kernel launches             */
  uint64_t fallback_files; /* files resolved by the serial fallback     */
  double ids_ms;       /* chunk-ID (BLAKE3) kernels of mcdc_chunk_ids_device */
  double aead_ms;      /* sealing kernels of mcdc_seal_device / mcdc_open_device */
  uint64_t lane_walk;  /* 1: the chains were walked one lane per chain */
  uint64_t handed_back; /* lane walk: segments handed to the group walk (spec + link) */
  double host_pre_ms;  /* host time from the call's entry to the first kernel enqueued */
  double host_post_ms; /* host time from the last device event to the return (results, copies) */
} mcdc_timing;

/* ------------------------------------------------------------------ API -- */

/* Validate params exactly as the crate's with_level asserts do
 * (MINIMUM_MIN 64 <= min <= 1 MiB, 256 <= avg <= 4 MiB, 1 KiB <= max <=
 * 16 MiB, level <= 3).  Where the crate panics this returns MCDC_E_PARAMS.
 * Optionally returns the normalised masks mask_s = MASKS[bits+level],
 * mask_l = MASKS[bits-level] (either pointer may be NULL). */
int mcdc_params_check(const mcdc_params *params, uint64_t *mask_s, uint64_t *mask_l);

/* Create a context on HIP device `device` able to chunk inputs up to
 * max_bytes per call (workspace is sized lazily up to that bound). */
int mcdc_ctx_create(int device, size_t max_bytes, struct mcdc_ctx **out);
void mcdc_ctx_destroy(struct mcdc_ctx *ctx);

/* Chunk one device-resident buffer (the device-resident GiB/s metric).
 * Replaces one StreamCDC::with_level(..) + its full iteration over a file
 * whose bytes already sit in HBM (processor.rs:173-202).  d_data is a device
 * pointer on the context's device (any alignment).
 * `out` may be host memory (pageable: one D2H copy; pinned: written directly
 * over PCIe) or a device pointer on the context's device, in which case the
 * boundary list stays in HBM for a device-side consumer (the next pipeline
 * stage, chunk IDs) and nothing crosses PCIe but the count.  The same holds
 * for `out` of every entry point below. */
int mcdc_chunk_device(struct mcdc_ctx *ctx, const mcdc_params *params, const void *d_data,
                      size_t n, mcdc_chunk *out, size_t cap, size_t *n_out);

/* Chunk one host buffer (end-to-end: H2D copy, kernels, D2H of boundaries).
 * This is what the Archiver adapter calls per file (processor.rs:165-202):
 * the file's bytes are read into host memory, chunked here, and each
 * ChunkData is the caller's slice [offset, offset+length). */
int mcdc_chunk_host(struct mcdc_ctx *ctx, const mcdc_params *params, const void *h_data,
                    size_t n, mcdc_chunk *out, size_t cap, size_t *n_out);

/* Chunk many independent host buffers in one batch (the many-buffer path:
 * one StreamCDC per file, processor.rs:173; chains restart at every buffer).
 * Chunks of buffer i are written contiguously in buffer order; counts[i]
 * receives buffer i's chunk count (may be NULL).  Offsets are relative to
 * each buffer. */
int mcdc_chunk_batch(struct mcdc_ctx *ctx, const mcdc_params *params,
                     const uint8_t *const *bufs, const size_t *lens, size_t nbufs,
                     mcdc_chunk *out, size_t cap, size_t *counts, size_t *n_out);

/* Same, but the buffers already sit back to back in one device arena:
 * buffer i is d_arena[offsets[i], offsets[i] + lens[i]).  offsets/lens are
 * host arrays, in any order; overlapping non-empty ranges -> MCDC_E_INVALID,
 * an arena span max(offsets[i] + lens[i]) above the context's max_bytes ->
 * MCDC_E_TOOBIG. */
int mcdc_chunk_batch_device(struct mcdc_ctx *ctx, const mcdc_params *params,
                            const void *d_arena, const uint64_t *offsets, const uint64_t *lens,
                            size_t nbufs, mcdc_chunk *out, size_t cap, size_t *counts,
                            size_t *n_out);

/* Chunk IDs of a boundary list: ids[32*i .. 32*i+32) = BLAKE3 (unkeyed,
 * 32-byte output) of the chunk's bytes.  Replaces the per-chunk
 * ID::from_content(&chunk.data) of chunk_and_save_blobs
 * (/root/reference/src/archiver/processor.rs:184 -> src/global/mod.rs:86-88
 * -> src/utils/mod.rs:62-68, crate blake3 1.8.2).  d_data: the device buffer
 * the chunks index (n bytes, any alignment); chunks: nchunks records as
 * produced by mcdc_chunk_device (offset/length relative to d_data; the hash
 * field is ignored), either a device pointer on the context's device (the
 * boundary list stays in HBM) or host memory; ids: 32 * nchunks bytes,
 * device pointer or host memory.  Chunks may overlap or repeat (each is hashed
 * on its own).  A chunk outside [0, n) -> MCDC_E_INVALID. */
int mcdc_chunk_ids_device(struct mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks,
                          size_t nchunks, uint8_t *ids);

/* ------------------------------------------------------ SecureStorage sealing
 * mapache encodes every blob it stores as zstd, then AES-256-GCM-SIV
 * (/root/reference/src/repository/storage.rs:61-65 encode; :97-118
 * encrypt_with_key, crate aes-gcm-siv 0.11.1): a 32-byte key, a fresh random
 * 12-byte nonce per blob, no associated data, and the stored bytes
 *     nonce (12) || ciphertext (= plaintext length) || tag (16).
 * These entry points run that encryption for many blobs at once on the GPU
 * (RFC 8452; bit-identical to the crate).  The nonce is an argument: the
 * caller draws it from its CSPRNG (OsRng in storage.rs:103) exactly as before.
 *
 * d_in: device buffer of n_in bytes (any alignment); blob i is
 * d_in[blobs[i].offset, + blobs[i].length) — for sealing, the compressed
 * blobs; extents may overlap; one outside [0, n_in) -> MCDC_E_INVALID.
 * Output: the results packed back to back from d_out in blob order;
 * out_offsets (optional, nblobs + 1 entries, host or device memory) receives
 * each result's offset and, last, the total; a total above out_cap ->
 * MCDC_E_CAPACITY (nothing written; *out_offsets still filled when given).
 * blobs, nonces: host or device memory. */
#define MCDC_NONCE_BYTES 12
#define MCDC_TAG_BYTES 16
#define MCDC_SEAL_OVERHEAD 28

typedef struct {
  uint64_t offset;
  uint64_t length;
} mcdc_blob;

/* encrypt_with_key for every blob: result i = nonces[12 i, + 12) ||
 * ciphertext || tag, length blobs[i].length + 28. */
int mcdc_seal_device(struct mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in,
                     const mcdc_blob *blobs, size_t nblobs, const uint8_t *nonces, void *d_out,
                     size_t out_cap, uint64_t *out_offsets);

/* Same, with the blob extents given as a boundary list (mcdc_chunk records,
 * the hash field ignored; host memory or a device pointer on the context's
 * device, e.g. the device-resident `out` of mcdc_chunk_device), so that chunk
 * -> IDs -> seal stays in HBM.  mapache compresses each chunk before sealing
 * it; this entry serves blobs that are the chunks themselves (data that the
 * caller stores uncompressed, or a measurement of the sealing stage). */
int mcdc_seal_chunks_device(struct mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in,
                            const mcdc_chunk *chunks, size_t nchunks, const uint8_t *nonces, void *d_out,
                            size_t out_cap, uint64_t *out_offsets);

/* decrypt_with_key (storage.rs:128-144) for every sealed extent: result i is
 * the plaintext (length - 28 bytes).  status (optional, host or device, nblobs
 * entries): 0 authentic, -1 not (tag mismatch, or an extent shorter than 28
 * bytes, where the crate errors too); a failed blob's result bytes are zero.
 * Returns MCDC_E_AUTH when any blob failed, MCDC_OK otherwise. */
int mcdc_open_device(struct mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in,
                     const mcdc_blob *sealed, size_t nblobs, void *d_out, size_t out_cap,
                     uint64_t *out_offsets, int32_t *status);

/* SecureStorage::encode / decode for many blobs held in host memory
 * (storage.rs:61-69): zstd (level 3, window log 20 = log2(AVG_CHUNK_SIZE), no
 * checksum: :31, :74-84) on host threads with the system libzstd.so.1, then
 * encrypt_with_key on the GPU (as mcdc_seal_device); decode = decrypt on the
 * GPU, then zstd decompression with window_log_max 20 (:87-94).
 * encode: blob i = h_in[blobs[i].offset, + length); result i = nonce ||
 * AES-256-GCM-SIV(zstd(blob i)) || tag, packed back to back into h_out in
 * blob order; out_offsets (optional, nblobs + 1): offsets and total.
 * decode: sealed extents of h_in -> the original blobs packed into h_out;
 * status (optional): 0, -1 (authentication failed) or -2 (not a zstd frame
 * within the window); any failure -> MCDC_E_AUTH.  Too small an out_cap ->
 * MCDC_E_CAPACITY (out_offsets still filled).  The compressed bytes depend on
 * the libzstd version; decoding is what is compatible.  No libzstd.so.1 ->
 * MCDC_E_INTERNAL.  Frames carry no content size (the crate's streaming
 * encoder pledges none), so their header is magic || 0x00 || window byte.
 * key == NULL is SecureStorage::build() (storage.rs:40-46: no key; level 0 =
 * zstd's default 3): encode only compresses, decode only decompresses
 * (encrypt / decrypt are the identity, :120-125, :146-151) and nonces may be
 * NULL.  Host memory: encode keeps, per context, a buffer of the blobs'
 * zstd bounds and a pinned one of the frames (about 1.1 and 0.4 x the
 * input for text), grown and reused by later calls (decode reuses the
 * pinned one for the opened frames); mcdc_save_files in host-zstd mode from
 * device input also keeps a pinned copy of the new blobs and of their
 * encoded form.  All are freed by mcdc_ctx_destroy. */
int mcdc_encode_blobs(struct mcdc_ctx *ctx, const uint8_t key[32], const void *h_in, size_t n_in,
                      const mcdc_blob *blobs, size_t nblobs, const uint8_t *nonces, void *h_out,
                      size_t out_cap, uint64_t *out_offsets);
int mcdc_decode_blobs(struct mcdc_ctx *ctx, const uint8_t key[32], const void *h_in, size_t n_in,
                      const mcdc_blob *sealed, size_t nblobs, void *h_out, size_t out_cap,
                      uint64_t *out_offsets, int32_t *status);

/* zstd frames of every chunk of a boundary list, in HBM, in raw-block
 * ("store") mode: the format of SecureStorage::compress (storage.rs:74-84;
 * window 2^20, no checksum) without entropy coding — what zstd itself emits
 * for incompressible data — so chunk -> frame -> seal stays on the GPU and the
 * blobs stay readable by mapache's decoder (storage.rs:87-94).  d_out must be
 * 16-byte aligned (else MCDC_E_INVALID).  Frame i is
 * written at a 16-byte aligned offset of d_out; frames[i] (host or device)
 * receives its (offset, length), ready for mcdc_seal_device.  *out_bytes: the
 * output span (also on MCDC_E_CAPACITY).  chunks: host or device; a chunk
 * outside [0, n) or of 2 GiB or more -> MCDC_E_INVALID. */
int mcdc_zstd_frames_device(struct mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks,
                            size_t nchunks, void *d_out, size_t out_cap, size_t *out_bytes,
                            mcdc_blob *frames);

/* SecureStorage::compress (storage.rs:74-84) of every chunk of a boundary
 * list on the GPU: frame i is a zstd frame of chunk i in the crate's layout
 * (magic, Frame_Header_Descriptor 0x00: no content size, no checksum; window
 * 2^20 = storage.rs:31) of 32 KiB blocks, each compressed (Huffman / RLE /
 * raw literals; sequences with per-block or predefined FSE tables) or raw
 * when that is not smaller.
 * mapache's decoder (zstd, window_log_max 20, :87-94) reads them; the bytes
 * differ from libzstd's level 3 (parity = decode-equality, ratio reported by
 * the bench).  Frames are written back to back from d_out (no alignment);
 * frames[i] (host or device) receives (offset, length).  *out_bytes: the bytes
 * written; on MCDC_E_CAPACITY the capacity that always suffices (the raw
 * frames: sum of length + 6 + 3 per 32 KiB block).  chunks: host or device;
 * a chunk outside [0, n) or of 2 GiB or more -> MCDC_E_INVALID.
 * Scratch: device memory of the context, grown on first use and kept (not
 * counted against max_bytes): about 9 bytes per byte of a batch of whole
 * chunks, a batch holding up to 16384 blocks of 32 KiB (4.5 GiB), two batch
 * sets once the input exceeds one (9 GiB); a chunk longer than a batch
 * takes a batch of its own size.  mcdc_zstd_compress_scratch reports the
 * exact amount for a chunk list before the call. */
int mcdc_zstd_compress_device(struct mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks,
                              size_t nchunks, void *d_out, size_t out_cap, size_t *out_bytes,
                              mcdc_blob *frames);
/* The device scratch (bytes) mcdc_zstd_compress_device allocates on this
 * context for the chunk list `chunks` (host memory, nchunks records; only
 * the lengths are read), with the context's batch settings: a caller sizing
 * HBM adds it to max_bytes.  The context keeps the scratch until it is
 * destroyed (a later call with a smaller list allocates nothing). */
int mcdc_zstd_compress_scratch(struct mcdc_ctx *ctx, const mcdc_chunk *chunks, size_t nchunks, size_t *bytes);

/* Packer::add_blob + flush (/root/reference/src/repository/packer.rs:101-186;
 * flushed when the packer holds more than max_pack_size bytes,
 * repository_v1.rs:185-193, and once more at the end) over a run of encoded
 * blobs in host memory: pack = blobs back to back || encode(header) ||
 * le32(len(encode(header))); header = per blob ID (32 B) || le32 length ||
 * type (1 B: 0 data, 1 tree), padded to a multiple of 64 entries with entries
 * of 36 random bytes + type 0xff (generate_header).  The randomness is the
 * caller's (OsRng in the crate): header_nonces (12 B per pack) and padding (36
 * B per padding entry, npadding entries; at most 63 per pack are used).
 * The header is encoded with mcdc_encode_blobs (key == NULL: compressed only,
 * as with SecureStorage::build() in packer.rs's own tests; no header nonces
 * needed); the pack ID is BLAKE3 of the
 * pack (utils::calculate_hash), computed on the GPU.  Output: the packs back
 * to back in h_out; *out_bytes their total and *npacks their number (also on
 * MCDC_E_CAPACITY); packs[k] = {offset, length, blobs, meta_size (encoded
 * header + 4), id}. */
typedef struct {
  uint64_t offset;
  uint64_t length;
  uint64_t nblobs;
  uint64_t meta_size;
  uint8_t id[32];
} mcdc_pack;
int mcdc_pack_blobs(struct mcdc_ctx *ctx, const uint8_t key[32], const void *h_blobs, size_t n_in,
                    const mcdc_blob *blobs, const uint8_t *ids, const uint8_t *types, size_t nblobs,
                    uint64_t max_pack_size, const uint8_t *header_nonces, size_t nnonces,
                    const uint8_t *padding, size_t npadding, void *h_out, size_t out_cap,
                    size_t *out_bytes, mcdc_pack *packs, size_t packs_cap, size_t *npacks);

/* ------------------------------------------------------------ save path
 * The Archiver's save path for a run of files in one call -- what
 * processor::save_file / chunk_and_save_blobs do per file
 * (/root/reference/src/archiver/processor.rs:138-205) and
 * Repository::save_blob per blob (repository_v1.rs:155-195), in file order:
 *   - a file smaller than store->gate_bytes (default MIN_CHUNK_SIZE = 512 KiB,
 *     :144, independent of the chunker's params) is one blob whose ID is
 *     ID::from_content of the whole file (SaveID::CalculateID);
 *     any other file is chunked (StreamCDC, :173-179) and each chunk is a
 *     blob with ID::from_content (:184);
 *   - each blob is stored unless its ID is in the index or already pending
 *     (:173-180: the dedup index `ix`, which keeps the IDs across calls);
 *   - a stored blob is SecureStorage::encode'd (:182; store->key NULL =
 *     SecureStorage::build()) and added to the packer, which is flushed once
 *     it holds more than store->max_pack_size bytes (:185-192) and once at the
 *     end of the call (the end of the snapshot: Repository::flush);
 *     with store->gpu_compress the compression runs on the GPU: the packs'
 *     blobs decode to the same bytes, IDs, dedup decisions and the storing
 *     order are unchanged, but the encoded sizes are the GPU compressor's, so
 *     pack boundaries (the flush rule runs on encoded sizes), the pack count
 *     and the header padding follow those sizes.
 * data: host memory or a device pointer (n bytes); files: extents in it (the
 * chunked ones must not overlap).  Randomness is the caller's (OsRng in the
 * crate): store->nonces, 12 bytes per stored blob in storing order (unused
 * without a key), header_nonces per pack, padding (36 bytes per padding
 * header entry, drawn in order).
 * Outputs (host memory): file_blobs[nfiles + 1], the blob index where each
 * file's ID list starts (the Vec<ID> save_file returns is ids[32 *
 * file_blobs[f], 32 * file_blobs[f + 1])); ids (32 B per blob, blobs_cap
 * entries); is_new (optional, 1 B per blob: stored by this call); the packs
 * back to back in packs_out and their records (as mcdc_pack_blobs).  Too
 * small a blobs_cap / packs_out_cap / packs_cap -> MCDC_E_CAPACITY with
 * *nblobs / *packs_bytes / *npacks set and the index unchanged: call again
 * with larger outputs.  Any failure after the dedup step (capacity, nonces,
 * a device error) leaves the index exactly as before the call.  Input larger
 * than the context's max_bytes -> MCDC_E_TOOBIG. */
typedef struct {
  const uint8_t *key;           /* 32-byte key, or NULL (SecureStorage::build()) */
  uint64_t max_pack_size;       /* the repository's max_packer_size (16 MiB) */
  const uint8_t *nonces;        /* 12 B per stored blob */
  size_t nnonces;
  const uint8_t *header_nonces; /* 12 B per pack */
  size_t nheader_nonces;
  const uint8_t *padding;       /* 36 B per padding header entry */
  size_t npadding;
  uint32_t gpu_compress;        /* 0: zstd level 3 on host threads (the crate's bytes);
                                   1: mcdc_zstd_compress_device in HBM (frames mapache's
                                   decoder reads, not byte-equal to level 3), the seal
                                   straight into the packs' layout and the pack IDs in
                                   HBM, the packs copied out while later blobs compress:
                                   the whole save path on the GPU.  The pack headers'
                                   zstd frames hold raw blocks (decode-equal; so their
                                   size, and the layout, are known before the seal) */
  uint64_t gate_bytes;          /* processor::save_file's size gate (:144): a file shorter
                                   than this is one blob, never chunked; 0 = the
                                   reference's MIN_CHUNK_SIZE (512 KiB, defaults.rs:35),
                                   whatever params->min_size is */
} mcdc_store;
struct mcdc_index;
int mcdc_save_files(struct mcdc_ctx *ctx, const mcdc_params *params, struct mcdc_index *ix,
                    const mcdc_store *store, const void *data, size_t n, const mcdc_blob *files,
                    size_t nfiles, uint64_t *file_blobs, uint8_t *ids, uint8_t *is_new, size_t blobs_cap,
                    size_t *nblobs, void *packs_out, size_t packs_out_cap, size_t *packs_bytes,
                    mcdc_pack *packs, size_t packs_cap, size_t *npacks);

/* ------------------------------------------------------------- dedup index
 * Repository::save_blob stores a blob only when its ID is neither in the
 * index nor already pending (/root/reference/src/repository/repository_v1.rs:
 * 169-180: index.contains(&id) || !index.add_pending_blob(id)), so of equal
 * IDs the first in processing order is encoded and packed and the others
 * only referenced.  An mcdc_index is a device-resident set of the IDs stored
 * or pending so far (sorted in HBM on the context's device); mcdc_index_add
 * answers that check for a whole batch of chunk IDs at once and adds the new
 * ones.  The index belongs to the device of the context that created it and is
 * used through any context of that device (one call at a time). */
struct mcdc_index;
int mcdc_index_create(struct mcdc_ctx *ctx, struct mcdc_index **out);
void mcdc_index_destroy(struct mcdc_index *ix);
/* IDs held */
size_t mcdc_index_size(const struct mcdc_index *ix);
/* ids: n IDs (32 bytes each, processing order), host or device memory.
 * is_new (optional, n bytes, host or device): 1 for every ID to store (not in
 * the index, not equal to an earlier ID of the batch), else 0.
 * chunks / new_chunks (optional, both or neither; n records each, host or
 * device): the records of the new IDs, compacted in order — e.g. the boundary
 * list whose chunks go on to be sealed.  *n_new (optional): their number.
 * The new IDs are added to the index. */
int mcdc_index_add(struct mcdc_ctx *ctx, struct mcdc_index *ix, const uint8_t *ids, size_t n,
                   uint8_t *is_new, const mcdc_chunk *chunks, mcdc_chunk *new_chunks, size_t *n_new);

/* ---------------------------------------------------------------- batching
 * Cross-worker batching front-end.  mapache chunks files on read_concurrency
 * rayon workers at once (/root/reference/src/archiver/mod.rs:162-215, default
 * 4: src/global/defaults.rs:22), each with its own StreamCDC per file
 * (src/archiver/processor.rs:173).  A batcher lets every worker submit its
 * file and returns that file's chunks, while one mcdc_chunk_batch call serves
 * all files submitted together (group commit: the first submitter waits up to
 * gather_us for others, or until max_batch_files / max_batch_bytes is
 * reached; files arriving while a batch runs form the next one).  Per file the
 * result is exactly mcdc_chunk_host's (chains restart at the file's first
 * byte); statuses are per caller (MCDC_E_CAPACITY reports the file's count).
 * A file larger than max_batch_bytes -> MCDC_E_TOOBIG (chunk it with
 * mcdc_chunk_host or in StreamCDC windows).  mcdc_batcher_chunk is
 * thread-safe; the batcher owns one context on `device`. */
typedef struct mcdc_batcher mcdc_batcher;

typedef struct {
  uint64_t batches;         /* batch calls run                      */
  uint64_t files;           /* files chunked                        */
  uint64_t bytes;           /* bytes chunked                        */
  uint64_t max_batch_files; /* most files served by one batch call  */
} mcdc_batcher_counters;

int mcdc_batcher_create(int device, const mcdc_params *params, size_t max_batch_bytes, size_t max_batch_files,
                        uint32_t gather_us, mcdc_batcher **out);
void mcdc_batcher_destroy(mcdc_batcher *b);
int mcdc_batcher_chunk(mcdc_batcher *b, const void *data, size_t n, mcdc_chunk *out, size_t cap, size_t *n_out);
int mcdc_batcher_stats(const mcdc_batcher *b, mcdc_batcher_counters *out);

/* Timing of the last call on ctx. */
int mcdc_ctx_timing(const struct mcdc_ctx *ctx, mcdc_timing *out);

/* Message of the last failing call on this thread ("" if none). */
const char *mcdc_last_error(void);

/* ---------------------------------------------- utilities (not reference
 * interface: benchmark / test plumbing) -- */

/* Device / pinned-host allocation on the context's device. */
int mcdc_device_alloc(struct mcdc_ctx *ctx, size_t bytes, void **d_ptr);
int mcdc_device_free(struct mcdc_ctx *ctx, void *d_ptr);
/* Wait until all work enqueued by this context has finished: its streams
 * and the null stream; other contexts' work is not waited for (the timed
 * region's device-side bracket in bench.py: the bench never initialises a
 * second HIP runtime, e.g. torch's, in the libmcdc process). */
int mcdc_ctx_synchronize(struct mcdc_ctx *ctx);
/* Per-context settings for tests and tuning (not reference interface):
 *   "zc_batch_blocks"        blocks per GPU compressor batch (default 16384,
 *                            512 MiB; two streams take half each; ~5 bytes
 *                            of scratch per byte of a batch), >= 8
 *   "zc_two"                 0: compressor batches on one stream
 *   "save_group_blocks"      GPU save path: 32 KiB blocks per compression
 *                            group (0, the default: "zc_batch_blocks" or
 *                            32768, the larger: a group ends with a host
 *                            wait, fewer groups wait less); the
 *                            packs a group closes are copied out while the
 *                            next group compresses
 *   "zc_small"               0: chunks of one block (<= 32 KiB) through the
 *                            long chunks' probe and match finder instead of
 *                            the small-chunk kernel (A/B and tests)
 *   "test_fail_after_index"  1: mcdc_save_files fails after its index add
 *                            (exercises the rollback)
 * Unknown name -> MCDC_E_INVALID. */
int mcdc_ctx_set_option(struct mcdc_ctx *ctx, const char *name, long long value);
int mcdc_host_alloc(struct mcdc_ctx *ctx, size_t bytes, void **h_ptr);
int mcdc_host_free(struct mcdc_ctx *ctx, void *h_ptr);
int mcdc_memcpy_h2d(struct mcdc_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int mcdc_memcpy_d2h(struct mcdc_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);

/* Fill d_dst[0, n) with the counter-based synthetic stream used by the bench
 * and tests: byte at stream position p = pos + i is
 *   (mix64(seed + (p/8 + 1) * 0x9e3779b97f4a7c15) >> 8*(p%8)) & 0xff
 * where mix64 is the SplitMix64 finaliser (also in oracle/). */
int mcdc_fill_random_device(struct mcdc_ctx *ctx, void *d_dst, uint64_t pos, size_t n,
                            uint64_t seed);

/* Order-sensitive digest of a boundary list (offset, length pairs), the same
 * function as the oracle's; used to compare full-size runs cheaply. */
uint64_t mcdc_digest(const mcdc_chunk *chunks, size_t n);

/* Library/ABI version. */
int mcdc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MCDC_H */
