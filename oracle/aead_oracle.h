/* aead_oracle.h -- AES-GCM-SIV CPU restatement (RFC 8452 over FIPS-197).
 * TEST INFRASTRUCTURE ONLY: see aead_oracle.c for provenance and pinning. */
#ifndef MAPACHE_AMD_AEAD_ORACLE_H
#define MAPACHE_AMD_AEAD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void oa_sbox(uint8_t out[256]);
/* returns the number of rounds (10 or 14), -1 for a bad key length */
int oa_aes_expand(const uint8_t *key, int key_bytes, uint8_t rk[240]);
void oa_aes_encrypt_rk(const uint8_t *rk, int nr, const uint8_t in[16], uint8_t out[16]);
int oa_aes_encrypt_block(const uint8_t *key, int key_bytes, const uint8_t in[16], uint8_t out[16]);

void oa_dot(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]);
void oa_polyval(const uint8_t h[16], const uint8_t *x, size_t nblocks, uint8_t out[16]);

/* per-nonce message-authentication key (16 B) and message-encryption key (32 B) */
void oa_siv_derive(const uint8_t key[32], const uint8_t nonce[12], uint8_t auth[16], uint8_t enc[32]);
/* ct_tag receives np + 16 bytes */
int oa_siv_encrypt(const uint8_t *key, int key_bytes, const uint8_t nonce[12], const uint8_t *aad, size_t na,
                   const uint8_t *pt, size_t np, uint8_t *ct_tag);
/* 0 and the plaintext, or -1 (tag mismatch; pt zeroed) */
int oa_siv_decrypt(const uint8_t *key, int key_bytes, const uint8_t nonce[12], const uint8_t *aad, size_t na,
                   const uint8_t *ct_tag, size_t nct, uint8_t *pt);

/* storage.rs encrypt_with_key over n blobs: out[out_off[i]..] = nonce_i || ct_i || tag_i */
void oa_seal_blobs(const uint8_t key[32], const uint8_t *data, const uint64_t *off, const uint64_t *len, size_t n,
                   const uint8_t *nonces, uint8_t *out, const uint64_t *out_off, int threads);

#ifdef __cplusplus
}
#endif
#endif
