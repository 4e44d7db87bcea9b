// mcdc_zstd.h — zstd (RFC 8878) compressed-block format pieces shared by the
// GPU compressor (mcdc_zstd.hip) and its CPU format test
// (tests/cpp/test_zstd_format.cpp, built with hipcc, run on the host).
//
// What mapache stores is SecureStorage::compress's output
// (/root/reference/src/repository/storage.rs:74-84): one zstd frame per blob,
// level 3, window log 20 (log2 AVG_CHUNK_SIZE, :31), no checksum, written by the
// crate's streaming encoder (no content size).  The GPU writes the same frame
// header (magic, descriptor 0x00, window descriptor 0x50) and blocks that are
// either raw or compressed with
//   * Raw_Literals_Block literals (3-byte header, Size_Format 11),
//   * sequences coded per symbol type (literal lengths, offsets, match
//     lengths) with the predefined FSE distributions of RFC 8878
//     §3.1.1.3.2.2 (Predefined_Mode) or with the block's own distribution
//     (FSE_Compressed_Mode: normalized counts, table description), whichever
//     is estimated smaller,
//   * offsets as Offset_Value = offset + 3, or a repeat code (1-3) where the
//     offset equals a repeat offset the block itself set (rep_code_block);
//   * literals raw, RLE (one distinct byte) or Huffman-coded (Compressed_
//     Literals_Block: a length-limited canonical code over all 256 byte
//     values, weights in the direct representation or FSE-compressed,
//     whichever is shorter; one stream below 1024 literals, four above),
//     whichever section is smallest.
// Any conforming decoder (mapache's: zstd with window_log_max 20,
// storage.rs:87-94) reads them; the compressed bytes differ from libzstd's,
// so parity is decode-equality.
#pragma once
#include <math.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace mcdc {
namespace zs {

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr uint8_t kFhd = 0x00, kWd = 0x50;  // no content size / checksum; window 2^20
constexpr uint32_t kWindow = 1u << 20;
constexpr uint32_t kMinMatch = 4;           // the GPU parse's shortest match
constexpr uint32_t kFrameHdr = 6, kBlockHdr = 3, kLitHdr = 3;

// ---- sequence codes (RFC 8878 §3.1.1.3.2.1) -------------------------------
__host__ __device__ inline uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

__host__ __device__ inline uint32_t ll_code(uint32_t ll) {
  if (ll < 16) return ll;
  if (ll < 64) {
    // 16,18,20,22 (1 bit) 24,28 (2) 32,40 (3) 48 (4)
    if (ll < 24) return 16 + ((ll - 16) >> 1);
    if (ll < 32) return 20 + ((ll - 24) >> 2);
    if (ll < 48) return 22 + ((ll - 32) >> 3);
    return 24;
  }
  return highbit(ll) + 19;  // 64: code 25 (6 bits), 128: 26 (7 bits), ...
}
__host__ __device__ inline uint32_t ll_bits(uint32_t code) {
  if (code < 16) return 0;
  if (code < 20) return 1;
  if (code < 22) return 2;
  if (code < 24) return 3;
  if (code == 24) return 4;
  return code - 19;  // 25: 6 ... 35: 16
}
// mb = match length - 3
__host__ __device__ inline uint32_t ml_code(uint32_t mb) {
  if (mb < 32) return mb;
  if (mb < 128) {
    // 32,34,36,38 (1 bit) 40,44 (2) 48,56 (3) 64,80 (4) 96 (5)
    if (mb < 40) return 32 + ((mb - 32) >> 1);
    if (mb < 48) return 36 + ((mb - 40) >> 2);
    if (mb < 64) return 38 + ((mb - 48) >> 3);
    if (mb < 96) return 40 + ((mb - 64) >> 4);
    return 42;
  }
  return highbit(mb) + 36;  // 128: code 43 (7 bits) ...
}
__host__ __device__ inline uint32_t ml_bits(uint32_t code) {
  if (code < 32) return 0;
  if (code < 36) return 1;
  if (code < 38) return 2;
  if (code < 40) return 3;
  if (code < 42) return 4;
  if (code == 42) return 5;
  return code - 36;  // 43: 7 ... 52: 16
}

// ---- FSE compression tables for the predefined distributions --------------
// Built exactly as the decoder's spread (RFC 8878 §4.1.1) defines the states,
// in the encoder form of zstd's FSE_buildCTable: per symbol deltaNbBits /
// deltaFindState, and the next-state table sorted by symbol.
template <uint32_t S>
struct FseCTN {
  uint16_t state[S];
  int32_t dfs[53];
  uint32_t dnb[53];
  uint32_t log;
};
using FseCT = FseCTN<64>;    // the predefined distributions (accuracy log <= 6)
using FseCTL = FseCTN<512>;  // a block's own table (FSE_Compressed_Mode, log <= 9)
struct ZTables {
  FseCT ll, ml, of;
};

// Predefined normalized distributions (RFC 8878 §3.1.1.3.2.2).
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1,
                                 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
                                 -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1,
                                 -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// (sym: S bytes, cumul: 54 entries of workspace; the GPU passes LDS, since a
// dynamically indexed local array would live in scratch memory)
template <uint32_t S>
__host__ __device__ inline void fse_build(const int16_t *norm, int nsym, uint32_t tlog, FseCTN<S> &ct, uint8_t *sym,
                                          uint32_t *cumul) {
  const uint32_t size = 1u << tlog;
  uint32_t high = size - 1;
  cumul[0] = 0;
  for (int u = 1; u <= nsym; ++u) {
    if (norm[u - 1] == -1) {
      cumul[u] = cumul[u - 1] + 1;
      sym[high--] = (uint8_t)(u - 1);
    } else {
      cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  uint32_t pos = 0;
  for (int s = 0; s < nsym; ++s)
    for (int i = 0; i < norm[s]; ++i) {
      sym[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  for (uint32_t u = 0; u < size; ++u) ct.state[cumul[sym[u]]++] = (uint16_t)(size + u);
  int32_t total = 0;
  for (int s = 0; s < nsym; ++s) {
    const int n = norm[s];
    if (n == 0) {
      ct.dnb[s] = ((tlog + 1) << 16) - size;
      ct.dfs[s] = 0;
    } else if (n == -1 || n == 1) {
      ct.dnb[s] = (tlog << 16) - size;
      ct.dfs[s] = total - 1;
      total += 1;
    } else {
      const uint32_t max_bits = tlog - (31u - (uint32_t)__builtin_clz((uint32_t)(n - 1)));
      const uint32_t min_state_plus = (uint32_t)n << max_bits;
      ct.dnb[s] = (max_bits << 16) - min_state_plus;
      ct.dfs[s] = total - n;
      total += n;
    }
  }
  ct.log = tlog;
}
template <uint32_t S>
__host__ __device__ inline void fse_build(const int16_t *norm, int nsym, uint32_t tlog, FseCTN<S> &ct) {
  uint8_t sym[S];
  uint32_t cumul[54];
  fse_build(norm, nsym, tlog, ct, sym, cumul);
}

inline ZTables build_tables() {
  ZTables t{};
  fse_build(kLLNorm, 36, 6, t.ll);
  fse_build(kMLNorm, 53, 6, t.ml);
  fse_build(kOFNorm, 29, 5, t.of);
  return t;
}

// ---- bit writer (forward, little-endian: the decoder reads it backwards) --
struct BitW {
  uint8_t *p;      // next byte to write
  uint8_t *end;    // capacity limit (write fails past it)
  uint64_t acc;    // pending bits
  uint32_t n;      // pending bit count (< 64)
  bool over;
  bool wr = true;  // this lane stores (a wave running the writer in lockstep stores from one lane)
  __host__ __device__ void add(uint64_t v, uint32_t nb) {
    acc |= (v & ((nb >= 64) ? ~0ull : ((1ull << nb) - 1))) << n;
    n += nb;
    if (n >= 32) flush();
  }
  __host__ __device__ void flush() {
    while (n >= 8) {
      if (p >= end) over = true;
      else if (wr) *p = (uint8_t)acc;
      ++p;
      acc >>= 8;
      n -= 8;
    }
  }
  // end mark (a 1 bit) + the last partial byte; returns false on overflow
  __host__ __device__ bool close() {
    add(1, 1);
    flush();
    if (n) {
      if (p >= end) over = true;
      else if (wr) *p = (uint8_t)acc;
      ++p;
      n = 0;
    }
    return !over;
  }
};

struct FseState {
  uint32_t value;
};
template <class CT>
__host__ __device__ inline void fse_init(FseState &st, const CT &ct, uint32_t s) {
  const uint32_t nb = (ct.dnb[s] + (1u << 15)) >> 16;
  uint32_t v = (nb << 16) - ct.dnb[s];
  st.value = ct.state[(v >> nb) + ct.dfs[s]];
}
template <class CT>
__host__ __device__ inline void fse_encode(BitW &bw, FseState &st, const CT &ct, uint32_t s) {
  const uint32_t nb = (st.value + ct.dnb[s]) >> 16;
  bw.add(st.value, nb);
  st.value = ct.state[(st.value >> nb) + ct.dfs[s]];
}
template <class CT>
__host__ __device__ inline void fse_flush(BitW &bw, const FseState &st, const CT &ct) { bw.add(st.value, ct.log); }

// One sequence: literal length, match length (>= 3) and the Offset_Value
// (RFC 8878 §3.1.1.5: offset + 3 for an explicit offset, 1-3 a repeat code).
// Packed in 64 bits: ll 21 | ml 21 | offset value 22 (block <= 128 KiB,
// window 2^20).
__host__ __device__ inline uint64_t seq_pack_ov(uint32_t ll, uint32_t ml, uint32_t ov) {
  return (uint64_t)ll | (uint64_t)ml << 21 | (uint64_t)ov << 42;
}
// an explicit offset (>= 1)
__host__ __device__ inline uint64_t seq_pack(uint32_t ll, uint32_t ml, uint32_t off) {
  return seq_pack_ov(ll, ml, off + 3);
}
__host__ __device__ inline uint32_t seq_ll(uint64_t s) { return (uint32_t)(s & 0x1FFFFF); }
__host__ __device__ inline uint32_t seq_ml(uint64_t s) { return (uint32_t)((s >> 21) & 0x1FFFFF); }
__host__ __device__ inline uint32_t seq_ov(uint64_t s) { return (uint32_t)(s >> 42); }
__host__ __device__ inline uint32_t seq_off(uint64_t s) { return seq_ov(s) - 3; }  // (explicit offsets)

// Repeat offsets (RFC 8878 §3.1.1.5) over one block's sequences, in order,
// in place: an explicit offset equal to a repeat offset becomes its repeat
// code.  Only repeat offsets this block itself set are used (bit k of
// `known`: rep[k] came from this block's sequences): the history a block
// starts with depends on whether the blocks before it ended up compressed,
// which is decided after every block is encoded in parallel.  rep / known
// start as {0, 0, 0} / 0 for a block.
struct RepHist {
  uint32_t rep[3];
  uint32_t known;
};
__host__ __device__ inline uint64_t rep_code(RepHist &R, uint64_t s) {
  const uint32_t ll = seq_ll(s), off = seq_off(s);
  const uint32_t r0 = R.rep[0], r1 = R.rep[1], r2 = R.rep[2], k = R.known;
  uint32_t code = 0;
  if (ll) {
    if ((k & 1) && off == r0) code = 1;
    else if ((k & 2) && off == r1) code = 2;
    else if ((k & 4) && off == r2) code = 3;
  } else {  // ll == 0: 1 = rep[1], 2 = rep[2], 3 = rep[0] - 1
    if ((k & 2) && off == r1) code = 2;       // (as the value 1)
    else if ((k & 4) && off == r2) code = 3;  // (as the value 2)
    else if ((k & 1) && r0 > 1 && off == r0 - 1) code = 4;  // (as the value 3)
  }
  auto kb = [&](uint32_t i) { return (k >> i) & 1u; };
  switch (code) {
    case 0:  // a new offset: [off, r0, r1]
      R.rep[0] = off; R.rep[1] = r0; R.rep[2] = r1;
      R.known = 1u | kb(0) << 1 | kb(1) << 2;
      return s;
    case 1:  // rep[0]: unchanged
      return seq_pack_ov(ll, seq_ml(s), 1);
    case 2:  // rep[1]: [r1, r0, r2]
      R.rep[0] = r1; R.rep[1] = r0;
      R.known = kb(1) | kb(0) << 1 | kb(2) << 2;
      return seq_pack_ov(ll, seq_ml(s), ll ? 2 : 1);
    case 3:  // rep[2]: [r2, r0, r1]
      R.rep[0] = r2; R.rep[1] = r0; R.rep[2] = r1;
      R.known = kb(2) | kb(0) << 1 | kb(1) << 2;
      return seq_pack_ov(ll, seq_ml(s), ll ? 3 : 2);
    default:  // rep[0] - 1 (ll == 0): a new offset [r0 - 1, r0, r1]
      R.rep[0] = r0 - 1; R.rep[1] = r0; R.rep[2] = r1;
      R.known = 1u | kb(0) << 1 | kb(1) << 2;
      return seq_pack_ov(ll, seq_ml(s), 3);
  }
}

// Sequences_Section (RFC 8878 §3.1.1.3.2) of nseq sequences (seqs[i], in
// order) coded with the tables tll / tof / tml, written at dst (capacity
// cap): the sequence count, the Symbol_Compression_Modes byte `modes`, the
// table description desc[doff[k], + dlen[k]) of each type k (LL, OF, ML)
// whose mode is FSE_Compressed, then the bitstream.  Returns the section
// size, or 0 when it does not fit.  wr false: sizes only, nothing stored (a
// wave running one writer in lockstep).
template <class CLL, class COF, class CML, class SeqAt>
__host__ __device__ inline uint32_t encode_sequences_with(const CLL &tll, const COF &tof, const CML &tml,
                                                          uint32_t modes, const uint8_t *desc, const uint32_t *doff,
                                                          const uint32_t *dlen, SeqAt seq_at, uint32_t nseq,
                                                          uint8_t *dst, uint32_t cap, bool wr = true) {
  uint32_t h = 0, ndesc = 0;
  for (uint32_t k = 0; k < 3; ++k)
    if (((modes >> (6 - 2 * k)) & 3) == 2) ndesc += dlen[k];
  if (cap < 4 + ndesc) return 0;
  auto put = [&](uint32_t v) {
    if (wr) dst[h] = (uint8_t)v;
    ++h;
  };
  if (nseq < 128) {
    put(nseq);
  } else if (nseq < 0x7F00) {
    put((nseq >> 8) + 0x80);
    put(nseq);
  } else {
    put(0xFF);
    put(nseq - 0x7F00);
    put((nseq - 0x7F00) >> 8);
  }
  if (nseq == 0) return h;
  put(modes);  // Symbol_Compression_Modes, then the descriptions of the FSE_Compressed types (LL, OF, ML)
  for (uint32_t k = 0; k < 3; ++k)
    if (((modes >> (6 - 2 * k)) & 3) == 2)
      for (uint32_t j = 0; j < dlen[k]; ++j) put(desc[doff[k] + j]);
  BitW bw{dst + h, dst + cap, 0, 0, false, wr};
  // the last sequence first (the decoder reads the stream backwards)
  uint64_t s = seq_at(nseq - 1);
  uint32_t ll = seq_ll(s), mb = seq_ml(s) - 3, ob = seq_ov(s);
  uint32_t llc = ll_code(ll), mlc = ml_code(mb), ofc = highbit(ob);
  FseState sml, sof, sll;
  fse_init(sml, tml, mlc);
  fse_init(sof, tof, ofc);
  fse_init(sll, tll, llc);
  bw.add(ll, ll_bits(llc));
  bw.add(mb, ml_bits(mlc));
  bw.add(ob, ofc);
  for (int32_t i = (int32_t)nseq - 2; i >= 0; --i) {
    s = seq_at((uint32_t)i);
    ll = seq_ll(s);
    mb = seq_ml(s) - 3;
    ob = seq_ov(s);
    llc = ll_code(ll);
    mlc = ml_code(mb);
    ofc = highbit(ob);
    fse_encode(bw, sof, tof, ofc);
    fse_encode(bw, sml, tml, mlc);
    fse_encode(bw, sll, tll, llc);
    bw.add(ll, ll_bits(llc));
    bw.add(mb, ml_bits(mlc));
    bw.add(ob, ofc);
    if (bw.over) return 0;
  }
  fse_flush(bw, sml, tml);
  fse_flush(bw, sof, tof);
  fse_flush(bw, sll, tll);
  if (!bw.close()) return 0;
  return (uint32_t)(bw.p - dst);
}

// The same with Predefined_Mode for all three symbol types.
template <class SeqAt>
__host__ __device__ inline uint32_t encode_sequences(const ZTables &T, SeqAt seq_at, uint32_t nseq, uint8_t *dst,
                                                     uint32_t cap) {
  const uint32_t none[3] = {0, 0, 0};
  return encode_sequences_with(T.ll, T.of, T.ml, 0u, (const uint8_t *)nullptr, none, none, seq_at, nseq, dst, cap);
}

// ---- a block's own FSE tables (FSE_Compressed_Mode, RFC 8878 §4.1.1) -------
// Per symbol type k (0 LL, 1 OF, 2 ML: the order of the modes byte and of the
// descriptions): symbols, the largest accuracy log the format allows, and
// the predefined distribution the choice is priced against.
constexpr uint32_t kSeqNSym[3] = {36, 32, 53};
constexpr uint32_t kSeqMaxLog[3] = {9, 8, 9};
constexpr uint32_t kSeqDescMax = 80;  // bytes of one description (<= 53 symbols of <= 10 bits + 4)

// Accuracy log for n symbols whose largest value is maxsym (zstd's
// FSE_optimalTableLog: about log2(n) - 2, at least enough for the alphabet,
// within [5, maxlog]).  n >= 2, maxsym >= 1.
__host__ __device__ inline uint32_t fse_table_log(uint32_t n, uint32_t maxsym, uint32_t maxlog) {
  const uint32_t hb = highbit(n - 1);
  uint32_t tl = maxlog;
  if (hb < 2 + tl) tl = hb >= 2 ? hb - 2 : 0;
  uint32_t minb = highbit(maxsym) + 2;
  if (hb + 1 < minb) minb = hb + 1;
  if (minb > tl) tl = minb;
  if (tl < 5) tl = 5;
  if (tl > maxlog) tl = maxlog;
  return tl;
}

// Normalized counts summing to 2^tl, every present symbol at least 1 (no
// "less than 1" entries), the largest symbol absorbing the rounding.  false
// when that leaves it below 1 (then the caller keeps the predefined table).
__host__ __device__ inline bool fse_normalize(const uint32_t *cnt, uint32_t nsym, uint32_t total, uint32_t tl,
                                              int16_t *norm) {
  const uint32_t scale = 1u << tl;
  int32_t sum = 0;
  uint32_t big = 0, bigc = 0;
  for (uint32_t s = 0; s < nsym; ++s) {
    if (!cnt[s]) {
      norm[s] = 0;
      continue;
    }
    uint32_t v = (uint32_t)(((uint64_t)cnt[s] * scale + total / 2) / total);
    if (v == 0) v = 1;
    norm[s] = (int16_t)v;
    sum += (int32_t)v;
    if (cnt[s] > bigc) {
      bigc = cnt[s];
      big = s;
    }
  }
  const int32_t fixed = norm[big] + ((int32_t)scale - sum);
  if (fixed < 1) return false;
  norm[big] = (int16_t)fixed;
  return true;
}

// Bits to code cnt[] with the distribution norm[] (-1 = one state) at
// accuracy log tl: sum of cnt * (tl - log2 states); huge when a present
// symbol has no state.
__host__ __device__ inline float fse_cost(const uint32_t *cnt, uint32_t ncnt, const int16_t *norm, uint32_t nnorm,
                                          uint32_t tl) {
  float b = 0;
  for (uint32_t s = 0; s < ncnt; ++s) {
    if (!cnt[s]) continue;
    const int32_t n = s < nnorm ? (norm[s] == -1 ? 1 : norm[s]) : 0;
    if (n <= 0) return 1e30f;
    b += (float)cnt[s] * ((float)tl - log2f((float)n));
  }
  return b;
}

// FSE table description (zstd's FSE_writeNCount, read by RFC 8878 §4.1.1):
// accuracy log - 5 in 4 bits, then per symbol its count + 1 in a variable
// number of bits (one fewer for small values), zero runs as 2-bit repeat
// flags, up to the last symbol with a nonzero count.  Returns its bytes.
__host__ __device__ inline uint32_t fse_write_ncount(const int16_t *norm, uint32_t nsym, uint32_t tl, uint8_t *dst) {
  uint32_t out = 0, nb = 4;
  uint64_t bits = tl - 5;
  auto drain = [&]() {
    while (nb >= 8) {
      dst[out++] = (uint8_t)bits;
      bits >>= 8;
      nb -= 8;
    }
  };
  int32_t remaining = (1 << tl) + 1, threshold = 1 << tl;
  uint32_t nbits = tl + 1, s = 0;
  bool prev0 = false;
  while (s < nsym && remaining > 1) {
    if (prev0) {
      uint32_t start = s;
      while (s < nsym && !norm[s]) ++s;
      while (s >= start + 24) {
        start += 24;
        bits |= 0xFFFFull << nb;
        nb += 16;
        drain();
      }
      while (s >= start + 3) {
        start += 3;
        bits |= 3ull << nb;
        nb += 2;
      }
      bits |= (uint64_t)(s - start) << nb;
      nb += 2;
      drain();
    }
    int32_t count = norm[s++];
    const int32_t mx = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    ++count;
    if (count >= threshold) count += mx;
    bits |= (uint64_t)(uint32_t)count << nb;
    nb += nbits;
    nb -= (count < mx) ? 1u : 0u;
    prev0 = count == 1;
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
    drain();
  }
  if (nb) dst[out++] = (uint8_t)bits;
  return out;
}

// The choice for one block's sequences, from the code histograms: per symbol
// type the predefined table or the block's own (when its estimated bits plus
// its description are fewer; only for 32 or more sequences with two or more
// distinct codes).  The tables themselves are built by the caller from
// norm / tl (fse_build on the host, k_zc_encode's wave on the GPU).
//
// The counts may cover several blocks (the GPU plans one table set for the 64
// blocks of a wave, each of which then carries the descriptions): nblk blocks
// pay the descriptions, and the accuracy log follows the mean block's count.
struct SeqPlan {
  int16_t norm[3][53];
  uint32_t tl[3];
  uint32_t own[3];               // 1: FSE_Compressed_Mode, 0: Predefined_Mode
  uint32_t doff[3], dlen[3];     // description of type k: desc[doff[k], + dlen[k])
  uint32_t modes, ndesc;
  uint8_t desc[3 * kSeqDescMax];
};
__host__ __device__ inline void seq_plan(const uint32_t *cll, const uint32_t *cof, const uint32_t *cml, uint32_t nseq,
                                         SeqPlan &P, uint32_t nblk = 1) {
  const uint32_t *cnt[3] = {cll, cof, cml};
  const int16_t *pre[3] = {kLLNorm, kOFNorm, kMLNorm};
  const uint32_t npre[3] = {36, 29, 53}, tpre[3] = {6, 5, 6}, shift[3] = {6, 4, 2};
  P.modes = 0;
  P.ndesc = 0;
  for (int k = 0; k < 3; ++k) {
    P.own[k] = 0;
    P.tl[k] = tpre[k];
    P.doff[k] = P.ndesc;
    P.dlen[k] = 0;
    uint32_t distinct = 0, maxsym = 0;
    for (uint32_t s = 0; s < kSeqNSym[k]; ++s)
      if (cnt[k][s]) {
        ++distinct;
        maxsym = s;
      }
    const uint32_t mean = nseq / (nblk ? nblk : 1);
    if (mean < 32 || distinct < 2) continue;
    const uint32_t tl = fse_table_log(mean, maxsym, kSeqMaxLog[k]);
    if (!fse_normalize(cnt[k], maxsym + 1, nseq, tl, P.norm[k])) continue;
    uint8_t *d = P.desc + P.ndesc;
    const uint32_t nd = fse_write_ncount(P.norm[k], maxsym + 1, tl, d);
    const float own = fse_cost(cnt[k], maxsym + 1, P.norm[k], maxsym + 1, tl) + 8.0f * (float)nd * (float)nblk;
    const float predef = fse_cost(cnt[k], maxsym + 1, pre[k], npre[k], tpre[k]);
    if (own >= predef) continue;
    for (uint32_t s = maxsym + 1; s < 53; ++s) P.norm[k][s] = 0;
    P.own[k] = 1;
    P.tl[k] = tl;
    P.dlen[k] = nd;
    P.ndesc += nd;
    P.modes |= 2u << shift[k];
  }
}

// Serial (host) form of the whole section with the planned tables: the CPU
// format test's reference for k_zc_encode.
template <class SeqAt>
inline uint32_t encode_sequences_auto(const ZTables &T, SeqAt seq_at, uint32_t nseq, uint8_t *dst, uint32_t cap,
                                      SeqPlan *plan_out = nullptr) {
  uint32_t c[3][53] = {{0}};
  for (uint32_t i = 0; i < nseq; ++i) {
    const uint64_t s = seq_at(i);
    ++c[0][ll_code(seq_ll(s))];
    ++c[1][highbit(seq_ov(s))];
    ++c[2][ml_code(seq_ml(s) - 3)];
  }
  SeqPlan P;
  seq_plan(c[0], c[1], c[2], nseq, P);
  if (plan_out) *plan_out = P;
  static FseCTL t[3];
  const FseCT *pre[3] = {&T.ll, &T.of, &T.ml};
  for (int k = 0; k < 3; ++k) {
    if (P.own[k]) {
      fse_build(P.norm[k], 53, P.tl[k], t[k]);
    } else {
      for (uint32_t u = 0; u < 64; ++u) t[k].state[u] = pre[k]->state[u];
      for (uint32_t u = 0; u < 53; ++u) {
        t[k].dfs[u] = pre[k]->dfs[u];
        t[k].dnb[u] = pre[k]->dnb[u];
      }
      t[k].log = pre[k]->log;
    }
  }
  return encode_sequences_with(t[0], t[1], t[2], P.modes, P.desc, P.doff, P.dlen, seq_at, nseq, dst, cap);
}

// ---- Huffman-coded literals (RFC 8878 §3.1.1.3.1, §4.2) ------------------
constexpr uint32_t kHufMaxBits = 11;

struct HufCT {
  uint16_t code[256];  // canonical code (valid where nb > 0)
  uint8_t nb[256];     // code length, 0 = absent
  uint32_t last;       // highest present symbol (its weight is implied)
  uint32_t maxb;       // longest code
};

// Scratch of huf_build (LDS on the GPU: dynamically indexed arrays in a
// lane's registers would live in scratch memory).
struct HufWork {
  uint32_t f[512];      // node weights: leaves 0..n-1 (ascending), internal nodes after
  uint16_t sym[256];    // symbols by count ascending (ties: by symbol)
  uint16_t par[512];    // parent of each node
  uint8_t dep[512];     // node depth
  uint32_t bl[64];      // leaves per depth
  uint32_t rank[kHufMaxBits + 2], val[kHufMaxBits + 2];
};

// Code lengths of a Huffman code over the symbols with cnt > 0 (cnt: 256
// counts, at least two present), limited to kHufMaxBits, then canonical codes
// as zstd's decoder rebuilds them from the weights: by rank from the longest
// length down (start 0; next rank's start = (start + count) >> 1), within a
// rank in symbol order.  Serial (one lane per block on the GPU).  sorted:
// w.sym already holds the present symbols by count ascending, ties by symbol
// (the GPU ranks them with the whole wave).
__host__ __device__ inline void huf_build(const uint32_t *cnt, HufCT &ct, HufWork &w, bool sorted = false) {
  uint16_t *sym = w.sym;
  uint32_t *f = w.f;
  uint32_t n = 0;
  for (uint32_t s = 0; s < 256; ++s) {
    ct.nb[s] = 0;
    if (cnt[s]) {
      if (!sorted) sym[n] = (uint16_t)s;
      ++n;
    }
  }
  // symbols by count ascending (insertion sort, stable: n <= 256)
  for (uint32_t i = 1; !sorted && i < n; ++i) {
    const uint16_t v = sym[i];
    uint32_t j = i;
    while (j > 0 && cnt[sym[j - 1]] > cnt[v]) {
      sym[j] = sym[j - 1];
      --j;
    }
    sym[j] = v;
  }
  // two-queue Huffman: leaves 0..n-1 (sorted), internal nodes n.. in creation order
  for (uint32_t i = 0; i < n; ++i) f[i] = cnt[sym[i]];
  uint32_t li = 0, ni = n, nn = n;
  auto take = [&]() -> uint32_t {
    if (li < n && (ni >= nn || f[li] <= f[ni])) return li++;
    return ni++;
  };
  while (nn < 2 * n - 1) {
    const uint32_t a = take(), b = take();
    f[nn] = f[a] + f[b];
    w.par[a] = w.par[b] = (uint16_t)nn;
    ++nn;
  }
  // depths: the root (2n - 2) at 0, a node one deeper than its parent
  uint32_t *bl = w.bl;
  for (uint32_t d = 0; d < 64; ++d) bl[d] = 0;
  w.dep[2 * n - 2] = 0;
  for (int32_t i = (int32_t)(2 * n) - 3; i >= 0; --i) w.dep[i] = (uint8_t)(w.dep[w.par[i]] + 1);
  uint32_t maxd = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t d = w.dep[i] < 63 ? w.dep[i] : 63;
    ++bl[d];
    if (d > maxd) maxd = d;
  }
  // limit to kHufMaxBits: leaves deeper than the limit move up to it, which
  // over-subscribes the code by an integer number of 2^-kHufMaxBits units
  // (the subtrees they came from were complete); each step below turns a
  // shorter leaf into a node over itself and one leaf taken from the longest
  // rank, -1 unit, until the Kraft sum is exactly 1 again (zlib's gen_bitlen)
  if (maxd > kHufMaxBits) {
    for (uint32_t d = kHufMaxBits + 1; d <= maxd; ++d) {
      bl[kHufMaxBits] += bl[d];
      bl[d] = 0;
    }
    uint64_t kraft = 0;  // in units of 2^-kHufMaxBits
    for (uint32_t d = 1; d <= kHufMaxBits; ++d) kraft += (uint64_t)bl[d] << (kHufMaxBits - d);
    while (kraft > (1ull << kHufMaxBits)) {  // (n <= 256 < 2^11 leaves: a shorter leaf always exists)
      uint32_t d = kHufMaxBits - 1;
      while (bl[d] == 0) --d;
      --bl[d];
      bl[d + 1] += 2;
      --bl[kHufMaxBits];
      --kraft;
    }
    maxd = kHufMaxBits;
  }
  // lengths: the most frequent symbols (sym[] ascending by count) get the shortest
  uint32_t k = n;
  for (uint32_t d = 1; d <= maxd; ++d)
    for (uint32_t c = 0; c < bl[d]; ++c) ct.nb[sym[--k]] = (uint8_t)d;
  ct.maxb = maxd;
  ct.last = sym[0];
  for (uint32_t i = 0; i < n; ++i)
    if (sym[i] > ct.last) ct.last = sym[i];
  // canonical codes
  for (uint32_t d = 0; d < kHufMaxBits + 2; ++d) w.rank[d] = 0;
  for (uint32_t d = 1; d <= maxd; ++d) w.rank[d] = bl[d];
  uint32_t mn = 0;
  for (uint32_t d = maxd; d > 0; --d) {
    w.val[d] = mn;
    mn = (mn + w.rank[d]) >> 1;
  }
  for (uint32_t s = 0; s <= ct.last; ++s)
    if (ct.nb[s]) ct.code[s] = (uint16_t)w.val[ct.nb[s]]++;
}

// Weight of symbol s: maxb + 1 - length, 0 for an absent symbol.
__host__ __device__ inline uint32_t huf_weight(const HufCT &ct, uint32_t s) {
  return ct.nb[s] ? ct.maxb + 1 - ct.nb[s] : 0u;
}

// Huffman_Tree_Description in the direct representation: headerByte = 127 +
// Number_of_Weights (the weights of symbols 0 .. last - 1, 4 bits each, first
// in the high nibble; the last symbol's weight is implied).  Only for last <=
// 128.  Returns its size.
__host__ __device__ inline uint32_t huf_tree_direct(const HufCT &ct, uint8_t *dst) {
  const uint32_t nw = ct.last;  // 1 .. 128
  dst[0] = (uint8_t)(127 + nw);
  for (uint32_t i = 0; i < nw; i += 2) {
    const uint32_t w0 = huf_weight(ct, i), w1 = i + 1 < nw ? huf_weight(ct, i + 1) : 0u;
    dst[1 + i / 2] = (uint8_t)(w0 << 4 | w1);
  }
  return 1 + (nw + 1) / 2;
}

// Workspace of the tree descriptions (LDS on the GPU, see fse_build).
struct HufDescWork {
  uint32_t cnt[13];
  uint32_t cumul[54];
  int16_t norm[53];
  uint8_t sym[64];
  uint8_t tmp[130];
  FseCTN<64> t;
};

// The weights FSE-compressed (RFC 8878 §4.2.1.2, as zstd's HUF_compressWeights
// writes them): an FSE table description of the weight histogram (accuracy
// log <= 6), then one bitstream with two interleaved states -- weights at even
// indices decoded from state 1, odd from state 2 -- written from the last
// weight back (FSE_compress_usingCTable's order), the first two encoded
// weights as the initial states.  headerByte = the compressed size (< 128).
// Returns the description's size (1 + compressed size), or 0 when the weights
// do not FSE-compress (a single distinct weight, or 128 bytes or more).
__host__ __device__ inline uint32_t huf_tree_fse(const HufCT &ct, uint8_t *dst, HufDescWork &ws) {
  const uint32_t nw = ct.last;  // 1 .. 255
  if (nw < 2) return 0;
  uint32_t *cnt = ws.cnt;
  for (uint32_t w = 0; w < 13; ++w) cnt[w] = 0;
  uint32_t maxw = 0;
  for (uint32_t i = 0; i < nw; ++i) {
    const uint32_t w = huf_weight(ct, i);
    ++cnt[w];
    if (w > maxw) maxw = w;
  }
  for (uint32_t w = 0; w <= maxw; ++w)
    if (cnt[w] == nw) return 0;  // (one distinct weight: zstd's "rle", not FSE-coded)
  const uint32_t tl = fse_table_log(nw, maxw, 6);
  int16_t *norm = ws.norm;
  if (!fse_normalize(cnt, maxw + 1, nw, tl, norm)) return 0;
  for (uint32_t w = maxw + 1; w < 53; ++w) norm[w] = 0;
  uint8_t *o = dst + 1;
  const uint32_t nd = fse_write_ncount(norm, maxw + 1, tl, o);
  FseCTN<64> &t = ws.t;
  fse_build(norm, (int)(maxw + 1), tl, t, ws.sym, ws.cumul);
  BitW bw{o + nd, dst + 128, 0, 0, false};
  FseState s1, s2;
  uint32_t i = nw;
  if (nw & 1) {
    fse_init(s1, t, huf_weight(ct, --i));
    fse_init(s2, t, huf_weight(ct, --i));
    fse_encode(bw, s1, t, huf_weight(ct, --i));
  } else {
    fse_init(s2, t, huf_weight(ct, --i));
    fse_init(s1, t, huf_weight(ct, --i));
  }
  while (i > 0) {
    fse_encode(bw, s2, t, huf_weight(ct, --i));
    fse_encode(bw, s1, t, huf_weight(ct, --i));
  }
  fse_flush(bw, s2, t);
  fse_flush(bw, s1, t);
  if (!bw.close()) return 0;
  const uint32_t csize = (uint32_t)(bw.p - o);
  if (csize >= 128) return 0;
  dst[0] = (uint8_t)csize;
  return 1 + csize;
}

// The shorter of the two descriptions (direct only for last <= 128); 0 when
// neither applies (the literals then stay raw).  dst holds 130 bytes.
__host__ __device__ inline uint32_t huf_tree_desc(const HufCT &ct, uint8_t *dst, HufDescWork &ws) {
  uint8_t *tmp = ws.tmp;
  const uint32_t f = huf_tree_fse(ct, tmp, ws);
  const uint32_t d = ct.last <= 128 ? 1 + (ct.last + 1) / 2 : 0xFFFFFFFFu;
  if (f && f < d) {
    for (uint32_t i = 0; i < f; ++i) dst[i] = tmp[i];
    return f;
  }
  return d != 0xFFFFFFFFu ? huf_tree_direct(ct, dst) : 0u;
}
inline uint32_t huf_tree_desc(const HufCT &ct, uint8_t *dst) {
  HufDescWork ws;
  return huf_tree_desc(ct, dst, ws);
}

// Bits of one Huffman stream of n literals (without the end mark).
template <class LitAt>
__host__ __device__ inline uint32_t huf_stream_bits(const HufCT &ct, LitAt lit_at, uint32_t a, uint32_t n) {
  uint32_t b = 0;
  for (uint32_t i = 0; i < n; ++i) b += ct.nb[lit_at(a + i)];
  return b;
}
// One stream: literals [a, a + n) from the last to the first (the decoder
// reads backwards and decodes them in order), closed by the end mark.
template <class LitAt>
__host__ __device__ inline uint32_t huf_stream(const HufCT &ct, LitAt lit_at, uint32_t a, uint32_t n, uint8_t *dst,
                                               uint32_t cap) {
  BitW bw{dst, dst + cap, 0, 0, false};
  for (uint32_t i = n; i-- > 0;) {
    const uint32_t x = lit_at(a + i);
    bw.add(ct.code[x], ct.nb[x]);
  }
  if (!bw.close()) return 0;
  return (uint32_t)(bw.p - dst);
}

// Literals_Section_Header of a Compressed_Literals_Block; returns its size.
// Size_Format 00 (one stream, 10-bit sizes), 10 (four streams, 14-bit), 11
// (four streams, 18-bit).
__host__ __device__ inline uint32_t lit_hdr_size(uint32_t nlit, uint32_t csize, bool one) {
  if (one) return 3;
  return (nlit < (1u << 14) && csize < (1u << 14)) ? 4 : 5;
}
__host__ __device__ inline void put_huf_lit_header(uint8_t *d, uint32_t nlit, uint32_t csize, bool one) {
  if (one) {  // 2 + 2 + 10 + 10 bits
    const uint32_t v = 2u | 0u << 2 | nlit << 4 | csize << 14;
    d[0] = (uint8_t)v; d[1] = (uint8_t)(v >> 8); d[2] = (uint8_t)(v >> 16);
  } else if (lit_hdr_size(nlit, csize, false) == 4) {  // 2 + 2 + 14 + 14
    const uint32_t v = 2u | 2u << 2 | nlit << 4 | csize << 18;
    d[0] = (uint8_t)v; d[1] = (uint8_t)(v >> 8); d[2] = (uint8_t)(v >> 16); d[3] = (uint8_t)(v >> 24);
  } else {  // 2 + 2 + 18 + 18
    const uint64_t v = 2ull | 3ull << 2 | (uint64_t)nlit << 4 | (uint64_t)csize << 22;
    for (int k = 0; k < 5; ++k) d[k] = (uint8_t)(v >> (8 * k));
  }
}
// RLE_Literals_Block header, Size_Format 11 (3 bytes, 20-bit size), then the byte
__host__ __device__ inline void put_rle_lit_header(uint8_t *d, uint32_t nlit) {
  d[0] = (uint8_t)(0x0D | (nlit & 0xF) << 4);
  d[1] = (uint8_t)(nlit >> 4);
  d[2] = (uint8_t)(nlit >> 12);
}

// Sizes of a Huffman literals section for the literals whose Huffman table
// is ct, with a tree description of `tree` bytes (stream bits sb[0..3], or
// sb[0] alone for one stream): section size = header + tree + (jump table) +
// streams.
__host__ __device__ inline uint32_t huf_section_size(uint32_t tree, uint32_t nlit, const uint32_t *sb, bool one,
                                                     uint32_t *ssz) {
  uint32_t streams = 0;
  for (int k = 0; k < (one ? 1 : 4); ++k) {
    ssz[k] = (sb[k] + 1 + 7) / 8;
    streams += ssz[k];
  }
  const uint32_t csize = tree + (one ? 0 : 6) + streams;
  return lit_hdr_size(nlit, csize, one) + csize;
}

// Headers.
__host__ __device__ inline void put_block_header(uint8_t *d, bool last, uint32_t type, uint32_t size) {
  const uint32_t h = (last ? 1u : 0u) | type << 1 | size << 3;
  d[0] = (uint8_t)h;
  d[1] = (uint8_t)(h >> 8);
  d[2] = (uint8_t)(h >> 16);
}
// Raw_Literals_Block header, Size_Format 11 (3 bytes, 20-bit size)
__host__ __device__ inline void put_raw_lit_header(uint8_t *d, uint32_t nlit) {
  d[0] = (uint8_t)(0x0C | (nlit & 0xF) << 4);
  d[1] = (uint8_t)(nlit >> 4);
  d[2] = (uint8_t)(nlit >> 12);
}
__host__ __device__ inline void put_frame_header(uint8_t *d) {
  d[0] = 0x28;
  d[1] = 0xB5;
  d[2] = 0x2F;
  d[3] = 0xFD;
  d[4] = kFhd;
  d[5] = kWd;
}

// The literals section of a compressed block, serial (the CPU format test's
// reference; the GPU makes the same choice with the same pieces, in
// parallel): RLE for one distinct byte, Huffman when that section is smaller
// than raw, else raw.  dst holds at least kLitHdr + n bytes.  Returns the
// section size.
template <class LitAt>
__host__ __device__ inline uint32_t encode_literals(LitAt lit_at, uint32_t n, uint8_t *dst) {
  uint32_t hist[256] = {0};
  for (uint32_t i = 0; i < n; ++i) ++hist[lit_at(i)];
  uint32_t distinct = 0, high = 0;
  for (uint32_t k = 0; k < 256; ++k)
    if (hist[k]) {
      ++distinct;
      high = k;
    }
  auto raw = [&]() {
    put_raw_lit_header(dst, n);
    for (uint32_t i = 0; i < n; ++i) dst[kLitHdr + i] = (uint8_t)lit_at(i);
    return kLitHdr + n;
  };
  if (n >= 32 && distinct == 1) {
    put_rle_lit_header(dst, n);
    dst[3] = (uint8_t)high;
    return 4;
  }
  if (n < 32) return raw();
  HufCT ct;
  HufWork hw;
  huf_build(hist, ct, hw);
  uint8_t tdesc[130];
  const uint32_t tree = huf_tree_desc(ct, tdesc);
  if (!tree) return raw();
  const bool one = n < 1024;
  const uint32_t seg = one ? n : (n + 3) / 4;
  uint32_t sb[4] = {0, 0, 0, 0}, ssz[4];
  for (int k = 0; k < (one ? 1 : 4); ++k) {
    const uint32_t a = k * seg, e = a + seg < n ? a + seg : n;
    sb[k] = huf_stream_bits(ct, lit_at, a, e - a);
  }
  const uint32_t total = huf_section_size(tree, n, sb, one, ssz);
  const uint32_t csize = tree + (one ? 0 : 6) + ssz[0] + (one ? 0 : ssz[1] + ssz[2] + ssz[3]);
  if (total >= kLitHdr + n || (one && csize >= 1024)) return raw();
  const uint32_t hdr = lit_hdr_size(n, csize, one);
  put_huf_lit_header(dst, n, csize, one);
  for (uint32_t i = 0; i < tree; ++i) dst[hdr + i] = tdesc[i];
  uint32_t o = hdr + tree;
  if (!one) {
    for (int k = 0; k < 3; ++k) {
      dst[o + 2 * k] = (uint8_t)ssz[k];
      dst[o + 2 * k + 1] = (uint8_t)(ssz[k] >> 8);
    }
    o += 6;
  }
  for (int k = 0; k < (one ? 1 : 4); ++k) {
    const uint32_t a = k * seg, e = a + seg < n ? a + seg : n;
    huf_stream(ct, lit_at, a, e - a, dst + o, ssz[k]);
    o += ssz[k];
  }
  return o;
}

}  // namespace zs
}  // namespace mcdc
