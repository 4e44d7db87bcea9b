// mcdc_aead.h — launch wrappers of the GPU SecureStorage sealing kernels
// (AES-256-GCM-SIV, RFC 8452), used by the C ABI in mcdc_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcdc {

constexpr uint32_t kAeadNonce = 12, kAeadTag = 16, kAeadOverhead = kAeadNonce + kAeadTag;
// A tile is one wave's work: up to 64 rows of 64 16-byte blocks (64 KiB).
constexpr uint32_t kAeadRows = 64, kAeadTileBlocks = 64 * kAeadRows;

// Per-blob record built by k_aead_prep (absolute device addresses).
struct AeadRec {
  uint64_t src;       // data bytes read by the CTR pass (seal: plaintext; open: ciphertext)
  uint64_t dst;       // data bytes written by the CTR pass
  uint64_t pv;        // the plaintext POLYVAL reads (seal: src; open: dst after the CTR pass)
  uint64_t ext;       // first output byte (seal: the nonce; open: = dst)
  uint64_t len;       // plaintext bytes
  uint64_t tile0;     // the blob's first tile
  uint32_t nonce[3];
  uint32_t ptiles;    // POLYVAL tiles (the blob's first ptiles tiles)
  uint32_t tag[4];    // seal: computed by k_aead_tag; open: the stored tag
  uint32_t ok;        // open: the extent holds nonce + tag (>= 28 bytes)
  uint32_t pad_[3];
};

// Per-blob key material (RFC 8452 §4) and POLYVAL powers.
struct AeadKeys {
  uint32_t rk[60];     // message-encryption key schedule (AES-256)
  uint32_t h[4];       // message-authentication key H
  uint32_t h4096[4];   // H^4096 (dot powers): tile combination
  uint32_t w[64][4];   // w[i] = H^(64 - i); w[0] = H^64 steps the row Horner
  uint32_t bas[128][4];  // bas[j] = dot(x^j, w[0]) = x^j G x^-128: basis of the row step's nibble tables
};

// AES-256 key schedule on the host: 60 little-endian words (FIPS-197 §5.2 bytes).
void aead_expand_key256(const uint8_t key[32], uint32_t rk[60]);

size_t aead_scan_tmp_bytes(uint64_t n);

// ext[2 i], ext[2 i + 1] = offset, length of boundary record i (24-byte records, device)
void launch_aead_from_chunks(const void *chunks, uint64_t n, uint64_t *ext, hipStream_t stream);

// Sizes: olen[i] (output bytes of blob i), tcnt[i] (tiles), exclusive scans
// into ooff / toff (n + 1 entries; [n] = totals).  An extent outside
// [0, n_in) sets err bit 0.  open: an extent shorter than 28 bytes gets no
// output and no tiles (it fails authentication).
void launch_aead_sizes(int open, const uint64_t *ext, uint64_t n, uint64_t n_in, uint64_t *olen, uint64_t *tcnt,
                       uint64_t *ooff, uint64_t *toff, uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t stream);

struct AeadMaster {
  uint32_t rk[60];  // key-generating key schedule
};

// seal: nonces = 12 * n bytes (device, 4-aligned); open: nonces from the extents.
// ctr: 2 words of device scratch (the persistent launches' tile counters).
void launch_aead_seal(const AeadMaster &mk, const uint8_t *in, const uint64_t *ext, const uint32_t *nonces,
                      uint64_t n, uint8_t *out, const uint64_t *ooff, const uint64_t *toff, uint64_t ntiles,
                      AeadRec *rec, AeadKeys *keys, uint32_t *owner, uint4 *tsum, uint32_t *ctr, int num_cus,
                      hipStream_t stream);
void launch_aead_open(const AeadMaster &mk, const uint8_t *in, const uint64_t *ext, uint64_t n, uint8_t *out,
                      const uint64_t *ooff, const uint64_t *toff, uint64_t ntiles, AeadRec *rec, AeadKeys *keys,
                      uint32_t *owner, uint4 *tsum, int32_t *status, uint32_t *ctr, int num_cus, hipStream_t stream);

}  // namespace mcdc
