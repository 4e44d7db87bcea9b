/*
 * fastcdc_oracle.c — CPU restatement of fastcdc 3.2.1 `v2020` (TEST
 * INFRASTRUCTURE ONLY; see fastcdc_oracle.h for provenance and the rule that
 * only tests/, smoke() and bench.py's cpu_baseline leg may use it).
 *
 * Reference anchors:
 *   call site + Level1 + per-file restart ... /root/reference/src/archiver/processor.rs:160-205
 *   parameters ............................... /root/reference/src/global/defaults.rs:35-40
 *   crate pin ................................ /root/reference/Cargo.lock:449-452
 *   algorithm restatement .................... SURVEY.md Appendix A.2-A.5
 */
#include "fastcdc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- MD5 ---- */
/* RFC 1321, used only to derive the GEAR table. */
static uint32_t md5_rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

static void md5_64x(uint8_t byte, uint8_t digest[16]) {
  static const uint32_t K[64] = {
      0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
      0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
      0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
      0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
      0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
      0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
      0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
      0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
      0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
      0xeb86d391};
  static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                            5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                            4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                            6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
  /* message = 64 copies of `byte` -> two 64-byte blocks after padding */
  uint8_t blocks[128];
  memset(blocks, byte, 64);
  memset(blocks + 64, 0, 64);
  blocks[64] = 0x80;
  const uint64_t bitlen = 64 * 8;
  for (int i = 0; i < 8; ++i) blocks[120 + i] = (uint8_t)(bitlen >> (8 * i));
  uint32_t h0 = 0x67452301, h1 = 0xefcdab89, h2 = 0x98badcfe, h3 = 0x10325476;
  for (int blk = 0; blk < 2; ++blk) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) {
      const uint8_t *q = blocks + blk * 64 + 4 * i;
      w[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    uint32_t a = h0, b = h1, c = h2, d = h3;
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
      else { f = c ^ (b | ~d); g = (7 * i) % 16; }
      uint32_t tmp = d;
      d = c;
      c = b;
      b = b + md5_rotl(a + f + K[i] + w[g], R[i]);
      a = tmp;
    }
    h0 += a; h1 += b; h2 += c; h3 += d;
  }
  uint32_t hs[4] = {h0, h1, h2, h3};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) digest[4 * i + j] = (uint8_t)(hs[i] >> (8 * j));
}

/* ------------------------------------------------------------- tables ---- */
static uint64_t GEAR[256], GEAR_LS[256];
static pthread_once_t gear_once = PTHREAD_ONCE_INIT;

static void gear_init(void) {
  for (int i = 0; i < 256; ++i) {
    uint8_t d[16];
    md5_64x((uint8_t)i, d);
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | d[j]; /* from_be_bytes(d[0..8]) */
    GEAR[i] = v;
    GEAR_LS[i] = v << 1; /* crate GEAR_LS = GEAR << 1 (wrapping) */
  }
}

/* MASKS[k] has k set bits, SURVEY.md A.2 (recalled from the crate, popcount
 * checked in tests/test_oracle.py). */
static const uint64_t MASKS[26] = {
    0, 0, 0, 0, 0,
    0x0000000001804110ULL, 0x0000000001803110ULL, 0x0000000018035100ULL,
    0x0000001800035300ULL, 0x0000019000353000ULL, 0x0000590003530000ULL,
    0x0000d90003530000ULL, 0x0000d90103530000ULL, 0x0000d90303530000ULL,
    0x0000d90313530000ULL, 0x0000d90f03530000ULL, 0x0000d90303537000ULL,
    0x0000d90703537000ULL, 0x0000d90707537000ULL, 0x0000d91707537000ULL,
    0x0000d91747537000ULL, 0x0000d91767537000ULL, 0x0000d93767537000ULL,
    0x0000d93777537000ULL, 0x0000d93777577000ULL, 0x0000db3777577000ULL};

void oc_gear(uint64_t out[256]) { pthread_once(&gear_once, gear_init); memcpy(out, GEAR, sizeof GEAR); }
void oc_gear_ls(uint64_t out[256]) { pthread_once(&gear_once, gear_init); memcpy(out, GEAR_LS, sizeof GEAR_LS); }
void oc_masks(uint64_t out[26]) { memcpy(out, MASKS, sizeof MASKS); }

uint32_t oc_logarithm2(uint32_t v) { return (uint32_t)round(log2((double)v)); }

int oc_params_init(oc_params *p, uint32_t min_size, uint32_t avg_size, uint32_t max_size,
                   uint32_t level) {
  pthread_once(&gear_once, gear_init);
  if (min_size < OC_MINIMUM_MIN || min_size > OC_MINIMUM_MAX) return -1;
  if (avg_size < OC_AVERAGE_MIN || avg_size > OC_AVERAGE_MAX) return -1;
  if (max_size < OC_MAXIMUM_MIN || max_size > OC_MAXIMUM_MAX) return -1;
  if (level > 3) return -1;
  const uint32_t bits = oc_logarithm2(avg_size);
  p->min_size = min_size;
  p->avg_size = avg_size;
  p->max_size = max_size;
  p->level = level;
  p->mask_s = MASKS[bits + level];
  p->mask_l = MASKS[bits - level];
  p->mask_s_ls = p->mask_s << 1;
  p->mask_l_ls = p->mask_l << 1;
  return 0;
}

/* --------------------------------------------------------- cut_gear ---- */
void oc_cut_gear(const oc_params *p, const uint8_t *src, size_t len, uint64_t *hash_out,
                 size_t *count_out) {
  size_t remaining = len;
  if (remaining <= p->min_size) { *hash_out = 0; *count_out = remaining; return; }
  size_t center = p->avg_size;
  if (remaining > p->max_size) remaining = p->max_size;
  else if (remaining < center) center = remaining;
  size_t index = p->min_size / 2;
  uint64_t hash = 0;
  while (index < center / 2) {
    const size_t a = index * 2;
    hash = (hash << 2) + GEAR_LS[src[a]];
    if ((hash & p->mask_s_ls) == 0) { *hash_out = hash; *count_out = a; return; }
    hash = hash + GEAR[src[a + 1]];
    if ((hash & p->mask_s) == 0) { *hash_out = hash; *count_out = a + 1; return; }
    index += 1;
  }
  while (index < remaining / 2) {
    const size_t a = index * 2;
    hash = (hash << 2) + GEAR_LS[src[a]];
    if ((hash & p->mask_l_ls) == 0) { *hash_out = hash; *count_out = a; return; }
    hash = hash + GEAR[src[a + 1]];
    if ((hash & p->mask_l) == 0) { *hash_out = hash; *count_out = a + 1; return; }
    index += 1;
  }
  *hash_out = hash;
  *count_out = remaining;
}

/* 1-byte form (SURVEY.md A.3 "Equivalent 1-byte form").  The hash returned
 * at an even position is doubled to match the 2-byte loop's `_ls` state. */
void oc_cut_gear_1byte(const oc_params *p, const uint8_t *src, size_t len, uint64_t *hash_out,
                       size_t *count_out) {
  size_t remaining = len;
  if (remaining <= p->min_size) { *hash_out = 0; *count_out = remaining; return; }
  size_t center = p->avg_size;
  if (remaining > p->max_size) remaining = p->max_size;
  else if (remaining < center) center = remaining;
  const size_t t0 = 2 * (p->min_size / 2), ce = 2 * (center / 2), re = 2 * (remaining / 2);
  uint64_t h = 0;
  for (size_t pos = t0; pos < re; ++pos) {
    h = (h << 1) + GEAR[src[pos]];
    const uint64_t m = pos < ce ? p->mask_s : p->mask_l;
    if ((h & m) == 0) {
      *hash_out = (pos & 1) ? h : (h << 1);
      *count_out = pos;
      return;
    }
  }
  *hash_out = h; /* last processed position re-1 is odd: un-doubled */
  *count_out = remaining;
}

typedef void (*cut_fn)(const oc_params *, const uint8_t *, size_t, uint64_t *, size_t *);

static size_t chunk_slice_with(cut_fn fn, const oc_params *p, const uint8_t *data, size_t n,
                               oc_chunk *out, size_t cap) {
  pthread_once(&gear_once, gear_init);
  size_t off = 0, k = 0;
  while (off < n) { /* FastCDC::next: remaining > 0 */
    uint64_t h;
    size_t c;
    fn(p, data + off, n - off, &h, &c);
    if (c == 0) break;
    if (k < cap) { out[k].offset = off; out[k].length = c; out[k].hash = h; }
    ++k;
    off += c;
  }
  return k;
}

size_t oc_chunk_slice(const oc_params *p, const uint8_t *data, size_t n, oc_chunk *out, size_t cap) {
  return chunk_slice_with(oc_cut_gear, p, data, n, out, cap);
}
size_t oc_chunk_slice_1byte(const oc_params *p, const uint8_t *data, size_t n, oc_chunk *out,
                            size_t cap) {
  return chunk_slice_with(oc_cut_gear_1byte, p, data, n, out, cap);
}

/* StreamCDC: buffer = vec![0; max]; fill_buffer loops read() until full or
 * EOF; cut_gear(&buffer[..length]); drain(..count). */
size_t oc_chunk_stream(const oc_params *p, const uint8_t *data, size_t n, size_t read_quantum,
                       oc_chunk *out, size_t cap) {
  pthread_once(&gear_once, gear_init);
  const size_t capacity = p->max_size;
  uint8_t *buffer = (uint8_t *)calloc(capacity, 1);
  if (!buffer) return 0;
  size_t length = 0, src_pos = 0, processed = 0, k = 0;
  int eof = 0;
  if (read_quantum == 0) read_quantum = 1;
  for (;;) {
    while (!eof && length < capacity) { /* fill_buffer */
      size_t want = capacity - length;
      if (want > read_quantum) want = read_quantum;
      if (want > n - src_pos) want = n - src_pos;
      if (want == 0) { eof = 1; break; }
      memcpy(buffer + length, data + src_pos, want);
      src_pos += want;
      length += want;
    }
    if (length == 0) break; /* Err(Empty) ends the iterator */
    uint64_t h;
    size_t c;
    oc_cut_gear(p, buffer, length, &h, &c);
    if (c == 0) break;
    if (k < cap) { out[k].offset = processed; out[k].length = c; out[k].hash = h; }
    ++k;
    processed += c;
    memmove(buffer, buffer + c, length - c); /* drain_bytes */
    length -= c;
  }
  free(buffer);
  return k;
}

/* ------------------------------------------------------ many files ---- */
typedef struct {
  const oc_params *p;
  const uint8_t *const *bufs;
  const size_t *lens;
  size_t nfiles;
  size_t next; /* guarded by mu */
  pthread_mutex_t mu;
  oc_chunk **res;
  size_t *cnt;
  int failed;
} files_job;

static void *files_worker(void *arg) {
  files_job *j = (files_job *)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->nfiles) break;
    const size_t n = j->lens[i];
    const size_t ub = n / (j->p->min_size - 1) + 2;
    oc_chunk *buf = (oc_chunk *)malloc(ub * sizeof(oc_chunk));
    if (!buf) { j->failed = 1; continue; }
    j->cnt[i] = oc_chunk_slice(j->p, j->bufs[i], n, buf, ub);
    j->res[i] = buf;
  }
  return NULL;
}

size_t oc_chunk_files(const oc_params *p, const uint8_t *const *bufs, const size_t *lens,
                      size_t nfiles, int threads, oc_chunk *out, size_t cap, size_t *counts) {
  pthread_once(&gear_once, gear_init);
  files_job j;
  memset(&j, 0, sizeof j);
  j.p = p; j.bufs = bufs; j.lens = lens; j.nfiles = nfiles;
  pthread_mutex_init(&j.mu, NULL);
  j.res = (oc_chunk **)calloc(nfiles ? nfiles : 1, sizeof(oc_chunk *));
  j.cnt = counts;
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, files_worker, &j);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  size_t total = 0;
  int too_small = 0;
  for (size_t i = 0; i < nfiles; ++i) {
    if (!j.res[i]) { too_small = 1; continue; }
    if (out && total + counts[i] <= cap) memcpy(out + total, j.res[i], counts[i] * sizeof(oc_chunk));
    else if (out) too_small = 1;
    total += counts[i];
    free(j.res[i]);
  }
  free(j.res);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return (too_small || j.failed) ? (size_t)-1 : total;
}

/* ------------------------------------------------------ utilities ---- */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

uint64_t oc_digest_step(uint64_t d, uint64_t offset, uint64_t length) {
  d = mix64(d ^ (offset + 0x9e3779b97f4a7c15ULL + (d << 6) + (d >> 2)));
  d = mix64(d ^ (length + 0x9e3779b97f4a7c15ULL + (d << 6) + (d >> 2)));
  return d;
}

size_t oc_chunk_digest(const oc_params *p, const uint8_t *data, size_t n, uint64_t *digest) {
  pthread_once(&gear_once, gear_init);
  size_t off = 0, k = 0;
  uint64_t d = 0;
  while (off < n) {
    uint64_t h;
    size_t c;
    oc_cut_gear(p, data + off, n - off, &h, &c);
    if (c == 0) break;
    d = oc_digest_step(d, off, c);
    ++k;
    off += c;
  }
  *digest = d;
  return k;
}

/* The counter-based stream [0, n) of `seed` chunked as one file, without
 * holding it: slabs are regenerated with oc_fill_random and the unfinished
 * window carried into the next slab.  A cut is taken only with >= max bytes
 * ahead (or at the end of the stream), so each cut_gear sees what it would see
 * over the whole slice (StreamCDC's refill rule).  Returns the
 * chunk count; *digest as oc_chunk_digest, *sum = sum of lengths. */
size_t oc_random_stream_digest(const oc_params *p, uint64_t seed, uint64_t n, size_t slab, uint64_t *digest,
                               uint64_t *sum) {
  return oc_random_stream_digest_h(p, seed, n, slab, digest, sum, NULL);
}

uint64_t oc_hash_digest(const uint64_t *hashes, size_t n) {
  uint64_t d = 0;
  for (size_t i = 0; i < n; ++i) d = oc_digest_step(d, i, hashes[i]);
  return d;
}

size_t oc_random_stream_digest_h(const oc_params *p, uint64_t seed, uint64_t n, size_t slab, uint64_t *digest,
                                 uint64_t *sum, uint64_t *hdigest) {
  pthread_once(&gear_once, gear_init);
  if (slab < 4096) slab = 4096;
  const size_t cap = slab + p->max_size;
  uint8_t *buf = (uint8_t *)malloc(cap);
  if (!buf) return 0;
  size_t s = 0, e = 0, k = 0;  /* valid bytes buf[s, e) */
  uint64_t gen = 0, off = 0, d = 0, hd = 0;
  for (;;) {
    if (e - s < p->max_size && gen < n) { /* refill */
      memmove(buf, buf + s, e - s);
      e -= s;
      s = 0;
      size_t take = cap - e;
      if (take > n - gen) take = (size_t)(n - gen);
      oc_fill_random(buf + e, gen, take, seed);
      gen += take;
      e += take;
      continue;
    }
    if (e == s) break;
    uint64_t h;
    size_t c;
    oc_cut_gear(p, buf + s, e - s, &h, &c);
    if (c == 0) break;
    d = oc_digest_step(d, off, c);
    hd = oc_digest_step(hd, k, h);
    ++k;
    off += c;
    s += c;
  }
  free(buf);
  *digest = d;
  if (sum) *sum = off;
  if (hdigest) *hdigest = hd;
  return k;
}

void oc_fill_random(uint8_t *dst, uint64_t pos, size_t n, uint64_t seed) {
  size_t i = 0;
  if ((pos & 7) == 0) { /* word-aligned fast path (little-endian host) */
    for (; i + 8 <= n; i += 8) {
      const uint64_t w = mix64(seed + (((pos + i) >> 3) + 1) * 0x9e3779b97f4a7c15ULL);
      memcpy(dst + i, &w, 8);
    }
  }
  while (i < n) {
    const uint64_t at = pos + i;
    const uint64_t w = mix64(seed + ((at >> 3) + 1) * 0x9e3779b97f4a7c15ULL);
    const unsigned b0 = (unsigned)(at & 7);
    for (unsigned b = b0; b < 8 && i < n; ++b, ++i) dst[i] = (uint8_t)(w >> (8 * b));
  }
}

uint64_t oc_file_seed(uint64_t seed, uint64_t file_index) {
  return mix64(seed ^ ((file_index + 1) * 0xd1b54a32d192ed03ULL));
}

/* Many files of the counter-based streams, each regenerated in its own buffer
 * and chunked as one file (a new StreamCDC per file, processor.rs:173), on
 * `threads` threads: file i = bytes [pos[i], pos[i] + len[i]) of the stream of
 * seeds[i].  Per file: its chunk count, oc_chunk_digest of its boundary list
 * (offsets relative to the file) and oc_hash_digest of its hashes.  The host
 * never holds more than threads x max(len) bytes: full-size parity for the
 * many-file configs.  Returns 0, or -1 on allocation failure. */
typedef struct {
  const oc_params *p;
  const uint64_t *seeds, *pos, *len;
  size_t nfiles, next;
  pthread_mutex_t mu;
  uint64_t *counts, *digests, *hdigests;
  int failed;
} rfiles_job;

static void *rfiles_worker(void *arg) {
  rfiles_job *j = (rfiles_job *)arg;
  uint8_t *buf = NULL;
  size_t bcap = 0;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->nfiles) break;
    const size_t n = (size_t)j->len[i];
    if (n > bcap) {
      free(buf);
      buf = (uint8_t *)malloc(n ? n : 1);
      bcap = buf ? n : 0;
      if (!buf) { j->failed = 1; continue; }
    }
    oc_fill_random(buf, j->pos[i], n, j->seeds[i]);
    size_t off = 0, k = 0;
    uint64_t d = 0, hd = 0;
    while (off < n) {
      uint64_t h;
      size_t c;
      oc_cut_gear(j->p, buf + off, n - off, &h, &c);
      if (c == 0) break;
      d = oc_digest_step(d, off, c);
      hd = oc_digest_step(hd, k, h);
      ++k;
      off += c;
    }
    j->counts[i] = k;
    j->digests[i] = d;
    if (j->hdigests) j->hdigests[i] = hd;
  }
  free(buf);
  return NULL;
}

int oc_random_files_digest(const oc_params *p, const uint64_t *seeds, const uint64_t *pos, const uint64_t *len,
                           size_t nfiles, int threads, uint64_t *counts, uint64_t *digests, uint64_t *hdigests) {
  pthread_once(&gear_once, gear_init);
  rfiles_job j;
  memset(&j, 0, sizeof j);
  j.p = p; j.seeds = seeds; j.pos = pos; j.len = len; j.nfiles = nfiles;
  j.counts = counts; j.digests = digests; j.hdigests = hdigests;
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  if (!th) return -1;
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, rfiles_worker, &j);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return j.failed ? -1 : 0;
}
