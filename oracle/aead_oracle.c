/* aead_oracle.c -- CPU restatement of the SecureStorage encryption step.
 *
 * TEST INFRASTRUCTURE ONLY (the parity checker for the GPU AEAD kernels and
 * the CPU baseline); nothing in mapache_amd/ links or loads it.
 *
 * mapache encrypts every blob with AES-256-GCM-SIV (crate aes-gcm-siv 0.11.1,
 * /root/reference/Cargo.toml:13, not vendored), no associated data, a fresh
 * random 12-byte nonce, output nonce || ciphertext || tag
 * (/root/reference/src/repository/storage.rs:97-118, encrypt_with_key; the
 * blob is zstd-compressed first, :61-65).  Restated here from the published
 * algorithm (RFC 8452: key derivation §4, POLYVAL §3, encryption §4, decryption
 * §5) over a byte-oriented AES (FIPS-197).  Pinned by known answers in
 * tests/test_aead_oracle.py: the FIPS-197 AES-128/256 example vectors, the RFC
 * 8452 POLYVAL example and recalled RFC 8452 appendix C vectors, and by AES
 * blocks cross-checked against the system OpenSSL (libcrypto) on the CPU.
 */
#include "aead_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------- AES --- */
static uint8_t sbox[256];
static pthread_once_t sbox_once = PTHREAD_ONCE_INIT;

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return r;
}

/* S-box from its definition: multiplicative inverse in GF(2^8), then the affine map */
static void sbox_init(void) {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x)
      for (int y = 1; y < 256; ++y)
        if (gmul((uint8_t)x, (uint8_t)y) == 1) {
          inv = (uint8_t)y;
          break;
        }
    uint8_t s = inv;
    for (int k = 1; k <= 4; ++k) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    sbox[x] = s ^ 0x63;
  }
}

void oa_sbox(uint8_t out[256]) {
  pthread_once(&sbox_once, sbox_init);
  memcpy(out, sbox, 256);
}

/* key expansion (FIPS-197 §5.2): nk = 4 or 8 words, nr = nk + 6 rounds */
int oa_aes_expand(const uint8_t *key, int key_bytes, uint8_t rk[240]) {
  pthread_once(&sbox_once, sbox_init);
  if (key_bytes != 16 && key_bytes != 32) return -1;
  const int nk = key_bytes / 4, nr = nk + 6, total = 4 * (nr + 1);
  memcpy(rk, key, (size_t)key_bytes);
  uint8_t rcon = 1;
  for (int i = nk; i < total; ++i) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % nk == 0) {
      const uint8_t t0 = t[0];
      t[0] = (uint8_t)(sbox[t[1]] ^ rcon);
      t[1] = sbox[t[2]];
      t[2] = sbox[t[3]];
      t[3] = sbox[t0];
      rcon = xtime(rcon);
    } else if (nk > 6 && i % nk == 4) {
      for (int k = 0; k < 4; ++k) t[k] = sbox[t[k]];
    }
    for (int k = 0; k < 4; ++k) rk[4 * i + k] = (uint8_t)(rk[4 * (i - nk) + k] ^ t[k]);
  }
  return nr;
}

void oa_aes_encrypt_rk(const uint8_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
  for (int r = 1; r <= nr; ++r) {
    uint8_t t[16];
    for (int i = 0; i < 16; ++i) t[i] = sbox[s[i]];  /* SubBytes */
    for (int c = 0; c < 4; ++c)                      /* ShiftRows: row i moves left by i */
      for (int i = 0; i < 4; ++i) s[4 * c + i] = t[4 * ((c + i) % 4) + i];
    if (r != nr)
      for (int c = 0; c < 4; ++c) { /* MixColumns */
        const uint8_t a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
        s[4 * c] = (uint8_t)(xtime(a0) ^ (xtime(a1) ^ a1) ^ a2 ^ a3);
        s[4 * c + 1] = (uint8_t)(a0 ^ xtime(a1) ^ (xtime(a2) ^ a2) ^ a3);
        s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xtime(a2) ^ (xtime(a3) ^ a3));
        s[4 * c + 3] = (uint8_t)((xtime(a0) ^ a0) ^ a1 ^ a2 ^ xtime(a3));
      }
    for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];  /* AddRoundKey */
  }
  memcpy(out, s, 16);
}

int oa_aes_encrypt_block(const uint8_t *key, int key_bytes, const uint8_t in[16], uint8_t out[16]) {
  uint8_t rk[240];
  const int nr = oa_aes_expand(key, key_bytes, rk);
  if (nr < 0) return -1;
  oa_aes_encrypt_rk(rk, nr, in, out);
  return 0;
}

/* --------------------------------------------------------- POLYVAL --- */
/* A field element is the 16-byte string read as a little-endian 128-bit
 * integer: bit i = coefficient of x^i.  Modulus x^128 + x^127 + x^126 +
 * x^121 + 1.  dot(a, b) = a * b * x^-128 (RFC 8452 §3). */
typedef struct {
  uint64_t lo, hi;
} u128;

static u128 load_le(const uint8_t b[16]) {
  u128 r = {0, 0};
  for (int i = 7; i >= 0; --i) {
    r.lo = (r.lo << 8) | b[i];
    r.hi = (r.hi << 8) | b[8 + i];
  }
  return r;
}

static void store_le(u128 v, uint8_t b[16]) {
  for (int i = 0; i < 8; ++i) {
    b[i] = (uint8_t)(v.lo >> (8 * i));
    b[8 + i] = (uint8_t)(v.hi >> (8 * i));
  }
}

static u128 dot(u128 a, u128 b) {
  /* r = a * b mod P: MSB-first shift-and-add over b's bits */
  u128 r = {0, 0};
  for (int i = 127; i >= 0; --i) {
    const uint64_t top = r.hi >> 63;
    r.hi = (r.hi << 1) | (r.lo >> 63);
    r.lo <<= 1;
    if (top) { /* x^128 = x^127 + x^126 + x^121 + 1 */
      r.hi ^= 0xc200000000000000ull;
      r.lo ^= 1ull;
    }
    const uint64_t bit = i >= 64 ? (b.hi >> (i - 64)) & 1 : (b.lo >> i) & 1;
    if (bit) {
      r.lo ^= a.lo;
      r.hi ^= a.hi;
    }
  }
  /* times x^-128: 128 times r = r / x (adding P first when r is odd) */
  for (int i = 0; i < 128; ++i) {
    const uint64_t odd = r.lo & 1;
    r.lo = (r.lo >> 1) | (r.hi << 63);
    r.hi >>= 1;
    if (odd) { /* (r + P) / x: P / x = x^127 + x^126 + x^125 + x^120 (+ x^-1 from the 1, absorbed) */
      r.hi ^= 0xe100000000000000ull;
    }
  }
  return r;
}

void oa_dot(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]) {
  store_le(dot(load_le(a), load_le(b)), out);
}

void oa_polyval(const uint8_t h[16], const uint8_t *x, size_t nblocks, uint8_t out[16]) {
  const u128 H = load_le(h);
  u128 s = {0, 0};
  for (size_t j = 0; j < nblocks; ++j) {
    const u128 xj = load_le(x + 16 * j);
    s.lo ^= xj.lo;
    s.hi ^= xj.hi;
    s = dot(s, H);
  }
  store_le(s, out);
}

/* ---------------------------------------------------- AES-GCM-SIV --- */
/* RFC 8452 §4: per-nonce keys from the key-generating key */
static void derive_keys(const uint8_t *key, int key_bytes, const uint8_t nonce[12], uint8_t auth[16],
                        uint8_t enc[32]) {
  uint8_t rk[240];
  const int nr = oa_aes_expand(key, key_bytes, rk);
  const int nblk = key_bytes == 32 ? 6 : 4;
  for (int i = 0; i < nblk; ++i) {
    uint8_t in[16] = {(uint8_t)i, 0, 0, 0}, out[16];
    memcpy(in + 4, nonce, 12);
    oa_aes_encrypt_rk(rk, nr, in, out);
    if (i < 2) memcpy(auth + 8 * i, out, 8);
    else memcpy(enc + 8 * (i - 2), out, 8);
  }
}

void oa_siv_derive(const uint8_t key[32], const uint8_t nonce[12], uint8_t auth[16], uint8_t enc[32]) {
  derive_keys(key, 32, nonce, auth, enc);
}

static void polyval_msg(const uint8_t h[16], const uint8_t *aad, size_t na, const uint8_t *pt, size_t np,
                        uint8_t s_out[16]) {
  const u128 H = load_le(h);
  u128 s = {0, 0};
  uint8_t blk[16];
  for (int part = 0; part < 2; ++part) {
    const uint8_t *p = part ? pt : aad;
    const size_t n = part ? np : na;
    for (size_t off = 0; off < n; off += 16) {
      const size_t k = n - off < 16 ? n - off : 16;
      memset(blk, 0, 16);
      memcpy(blk, p + off, k);
      const u128 x = load_le(blk);
      s.lo ^= x.lo;
      s.hi ^= x.hi;
      s = dot(s, H);
    }
  }
  u128 len = {(uint64_t)na * 8, (uint64_t)np * 8}; /* le64(bitlen(AAD)) || le64(bitlen(P)) */
  s.lo ^= len.lo;
  s.hi ^= len.hi;
  s = dot(s, H);
  store_le(s, s_out);
}

static void ctr_xor(const uint8_t *rk, int nr, const uint8_t tag[16], const uint8_t *in, size_t n,
                    uint8_t *out) {
  uint8_t ctr[16], ks[16];
  memcpy(ctr, tag, 16);
  ctr[15] |= 0x80;
  uint32_t c = (uint32_t)ctr[0] | (uint32_t)ctr[1] << 8 | (uint32_t)ctr[2] << 16 | (uint32_t)ctr[3] << 24;
  for (size_t off = 0; off < n; off += 16) {
    ctr[0] = (uint8_t)c;
    ctr[1] = (uint8_t)(c >> 8);
    ctr[2] = (uint8_t)(c >> 16);
    ctr[3] = (uint8_t)(c >> 24);
    oa_aes_encrypt_rk(rk, nr, ctr, ks);
    const size_t k = n - off < 16 ? n - off : 16;
    for (size_t i = 0; i < k; ++i) out[off + i] = (uint8_t)(in[off + i] ^ ks[i]);
    ++c; /* le32 counter, wrapping */
  }
}

int oa_siv_encrypt(const uint8_t *key, int key_bytes, const uint8_t nonce[12], const uint8_t *aad, size_t na,
                   const uint8_t *pt, size_t np, uint8_t *ct_tag) {
  if (key_bytes != 16 && key_bytes != 32) return -1;
  uint8_t auth[16], enc[32], s[16], tag[16], rk[240];
  derive_keys(key, key_bytes, nonce, auth, enc);
  polyval_msg(auth, aad, na, pt, np, s);
  for (int i = 0; i < 12; ++i) s[i] ^= nonce[i];
  s[15] &= 0x7f;
  const int nr = oa_aes_expand(enc, key_bytes, rk);
  oa_aes_encrypt_rk(rk, nr, s, tag);
  ctr_xor(rk, nr, tag, pt, np, ct_tag);
  memcpy(ct_tag + np, tag, 16);
  return 0;
}

int oa_siv_decrypt(const uint8_t *key, int key_bytes, const uint8_t nonce[12], const uint8_t *aad, size_t na,
                   const uint8_t *ct_tag, size_t nct, uint8_t *pt) {
  if ((key_bytes != 16 && key_bytes != 32) || nct < 16) return -1;
  const size_t np = nct - 16;
  uint8_t auth[16], enc[32], s[16], tag[16], rk[240];
  derive_keys(key, key_bytes, nonce, auth, enc);
  const int nr = oa_aes_expand(enc, key_bytes, rk);
  ctr_xor(rk, nr, ct_tag + np, ct_tag, np, pt);
  polyval_msg(auth, aad, na, pt, np, s);
  for (int i = 0; i < 12; ++i) s[i] ^= nonce[i];
  s[15] &= 0x7f;
  oa_aes_encrypt_rk(rk, nr, s, tag);
  uint8_t diff = 0;
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ ct_tag[np + i]);
  if (diff) {
    memset(pt, 0, np);
    return -1;
  }
  return 0;
}

/* ------------------------------------------------------------ blobs --- */
/* storage.rs encrypt_with_key for many blobs: out[out_off[i] ..] = nonce_i ||
 * AES-256-GCM-SIV(key, nonce_i, blob_i) || tag_i, out_off[i] = off_i + 28 i
 * when the blobs are packed back to back. */
typedef struct {
  const uint8_t *key, *data, *nonces;
  const uint64_t *off, *len, *out_off;
  uint8_t *out;
  size_t n;
  int t, nt;
} blob_job;

static void *blob_worker(void *arg) {
  blob_job *j = (blob_job *)arg;
  for (size_t i = (size_t)j->t; i < j->n; i += (size_t)j->nt) {
    uint8_t *o = j->out + j->out_off[i];
    memcpy(o, j->nonces + 12 * i, 12);
    oa_siv_encrypt(j->key, 32, j->nonces + 12 * i, NULL, 0, j->data + j->off[i], j->len[i], o + 12);
  }
  return NULL;
}

void oa_seal_blobs(const uint8_t key[32], const uint8_t *data, const uint64_t *off, const uint64_t *len, size_t n,
                   const uint8_t *nonces, uint8_t *out, const uint64_t *out_off, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  blob_job jobs[256];
  for (int t = 0; t < threads; ++t) {
    blob_job j = {key, data, nonces, off, len, out_off, out, n, t, threads};
    jobs[t] = j;
    if (threads > 1) pthread_create(&th[t], NULL, blob_worker, &jobs[t]);
  }
  if (threads == 1) blob_worker(&jobs[0]);
  else
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}
