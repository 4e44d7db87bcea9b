/*
 * blake3_oracle.c — CPU restatement of BLAKE3 (unkeyed hash, 32-byte output)
 * as mapache computes chunk IDs.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker of the GPU chunk-ID kernels
 * (mapache_amd/csrc/mcdc_blake3.hip) and the timed CPU baseline.  Never the
 * product path.
 *
 * Reference call sites: ID::from_content -> utils::calculate_hash
 *   /root/reference/src/global/mod.rs:86-88, src/utils/mod.rs:62-68
 *   (blake3::Hasher::new(); update(data); finalize()), used per chunk at
 *   src/archiver/processor.rs:184.  The arithmetic is the external crate
 *   `blake3` 1.8.2 (/root/reference/Cargo.toml:17, Cargo.lock:170), not
 *   vendored; this file restates the published BLAKE3 specification:
 *   compression function (7 rounds of the G mixing function, message word
 *   permutation), 1024-byte chunks of 16 blocks with CHUNK_START/CHUNK_END,
 *   parent nodes over two chaining values, ROOT on the final compression.
 *
 * The tree is built the way the specification's reference implementation
 * does it: a stack of subtree chaining values merged while the number of
 * completed chunks has trailing zero bits (the GPU uses the equivalent
 * level-by-level pairing instead — two independent statements of the tree
 * rule).  Pinned by the reference's own KAT (src/utils/mod.rs:426-441,
 * tests/golden/blake3_kat.json) and the published BLAKE3("") / BLAKE3("abc").
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

/* compress(cv, block words, counter, block_len, flags) -> first 8 output words */
static void compress(const uint32_t cv[8], const uint32_t m_in[16], uint64_t counter, uint32_t block_len,
                     uint32_t flags, uint32_t out[8]) {
  uint32_t s[16], m[16], t[16];
  memcpy(s, cv, 32);
  memcpy(s + 8, IV, 16);
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  memcpy(m, m_in, 64);
  for (int r = 0; r < 7; ++r) {
    g(s, 0, 4, 8, 12, m[0], m[1]);
    g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);
    g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);
    g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]);
    g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      for (int i = 0; i < 16; ++i) t[i] = m[PERM[i]];
      memcpy(m, t, 64);
    }
  }
  for (int i = 0; i < 8; ++i) out[i] = s[i] ^ s[i + 8];
}

static void load_block(const uint8_t *p, size_t len, uint32_t m[16]) {
  uint8_t buf[64] = {0};
  memcpy(buf, p, len);
  for (int i = 0; i < 16; ++i)
    m[i] = (uint32_t)buf[4 * i] | (uint32_t)buf[4 * i + 1] << 8 | (uint32_t)buf[4 * i + 2] << 16 |
           (uint32_t)buf[4 * i + 3] << 24;
}

/* Chaining value (or root output when is_root) of one <=1024-byte chunk. */
static void chunk_cv(const uint8_t *p, size_t len, uint64_t counter, int is_root, uint32_t out[8]) {
  uint32_t cv[8], m[16];
  memcpy(cv, IV, 32);
  const size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; ++b) {
    const size_t bl = (b + 1 < nblocks) ? 64 : len - 64 * b;
    load_block(p + 64 * b, bl, m);
    uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b + 1 == nblocks ? CHUNK_END : 0);
    if (is_root && b + 1 == nblocks) flags |= ROOT;
    compress(cv, m, counter, (uint32_t)bl, flags, cv);
  }
  memcpy(out, cv, 32);
}

static void parent_cv(const uint32_t l[8], const uint32_t r[8], int is_root, uint32_t out[8]) {
  uint32_t m[16];
  memcpy(m, l, 32);
  memcpy(m + 8, r, 32);
  compress(IV, m, 0, 64, PARENT | (is_root ? ROOT : 0), out);
}

void ob_hash(const uint8_t *data, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  const size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
  if (nchunks == 1) {
    chunk_cv(data, len, 0, 1, h);
  } else {
    uint32_t stack[64][8];
    int sp = 0;
    for (size_t c = 0; c + 1 < nchunks; ++c) {  // every chunk but the last
      uint32_t cv[8];
      chunk_cv(data + 1024 * c, 1024, c, 0, cv);
      uint64_t total = c + 1;  // completed chunks
      while ((total & 1) == 0) {  // merge completed subtrees
        parent_cv(stack[--sp], cv, 0, cv);
        total >>= 1;
      }
      memcpy(stack[sp++], cv, 32);
    }
    const size_t last = nchunks - 1;
    chunk_cv(data + 1024 * last, len - 1024 * last, last, 0, h);
    while (sp > 0) {  // fold the right edge; the last parent is the root
      --sp;
      parent_cv(stack[sp], h, sp == 0, h);
    }
  }
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)h[i];
    out[4 * i + 1] = (uint8_t)(h[i] >> 8);
    out[4 * i + 2] = (uint8_t)(h[i] >> 16);
    out[4 * i + 3] = (uint8_t)(h[i] >> 24);
  }
}

/* IDs of a boundary list over one buffer: ids[i] = BLAKE3(data[off_i, off_i+len_i)). */
typedef struct {
  const uint8_t *data;
  const uint64_t *off, *len;
  uint8_t *ids;
  size_t n, next;
  pthread_mutex_t mu;
} ids_job;

static void *ids_worker(void *arg) {
  ids_job *j = (ids_job *)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const size_t i0 = j->next;
    j->next += 64;
    pthread_mutex_unlock(&j->mu);
    if (i0 >= j->n) break;
    const size_t i1 = i0 + 64 < j->n ? i0 + 64 : j->n;
    for (size_t i = i0; i < i1; ++i) ob_hash(j->data + j->off[i], (size_t)j->len[i], j->ids + 32 * i);
  }
  return NULL;
}

void ob_chunk_ids(const uint8_t *data, const uint64_t *off, const uint64_t *len, size_t n, int threads,
                  uint8_t *ids) {
  ids_job j = {data, off, len, ids, n, 0, PTHREAD_MUTEX_INITIALIZER};
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, ids_worker, &j);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
}
