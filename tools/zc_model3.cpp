// zc_model3 — CPU model of the GPU match finder as it runs (tools only: prices
// finder choices before kernels are written, with the exact sizes of the
// format pieces in mcdc_zstd.h).  Models k_zc_find segment by segment: 8
// blocks of 32 KiB, the kPrime bytes before a segment re-inserted, tiles of
// 1024 positions (a tile reads the tables as the earlier tiles left them),
// the GPU's 24-bit-multiply keys, 13-bit tags, one verified candidate of 16
// bytes; then the greedy parse (a 16-byte match extended to its end within
// the block).  Optionally the far table: content-defined anchors (1 position
// in 2^A by a hash of the 8-byte key) whose latest position per slot over the
// 1 MiB window before the segment is preloaded, and the segment's own anchors
// inserted tile by tile; an anchor's far candidate, and (prop) a position
// without a local candidate takes the offset of the nearest far-matched
// anchor of its 64-position wave.  libzstd level 3 (streaming, window log 20:
// the crate's encoder, storage.rs:74-84) on the same chunks beside it.
//
// Usage: zc_model3 file P(16|512) [maxMiB]
// env: ZC_FAR (0/1) ZC_A (log2 anchor spacing, 8) ZC_F (far slots log2, 12)
//      ZC_HS (15) ZC_HL (13) ZC_PRIME (131072) ZC_PROP (0/1/2) ZC_PRI (0: far
//      first, 1: local long first) ZC_SEG (blocks per segment, 8; 0 = whole
//      chunk in one segment: the dense tables carried across the chunk)
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mapache_amd/csrc/mcdc_zstd.h"
extern "C" {
#include "../oracle/fastcdc_oracle.h"
}

using namespace mcdc::zs;

static uint32_t u24(uint32_t x, uint32_t k) { return (uint32_t)((uint64_t)(x & 0xFFFFFF) * k); }
static uint32_t mix5(uint32_t lo, uint32_t hi) { return u24(lo & 0xFFFFFF, 0x9E3779u) + u24(lo >> 24 | (hi & 0xFF) << 8, 0xC2B2AFu); }
static uint32_t mix8(uint32_t lo, uint32_t hi) {
  return u24(lo & 0xFFFFFF, 0x85EBCBu) ^ u24(lo >> 24 | (hi & 0xFFFF) << 8, 0x27D4EBu) ^ u24(hi >> 16, 0x165667u);
}
static int env(const char *k, int d) { return getenv(k) ? atoi(getenv(k)) : d; }

struct ZIn { const void *src; size_t size, pos; };
struct ZOut { void *dst; size_t size, pos; };

int main(int argc, char **argv) {
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  std::vector<uint8_t> d;
  std::fseek(f, 0, SEEK_END);
  d.resize(std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (std::fread(d.data(), 1, d.size(), f) != d.size()) return 1;
  std::fclose(f);
  const int P = argc > 2 ? atoi(argv[2]) : 16;
  const size_t maxb = (size_t)(argc > 3 ? atoi(argv[3]) : 64) << 20;
  if (d.size() > maxb) d.resize(maxb);
  const size_t n = d.size();
  d.resize(n + 64, 0);
  const int FAR = env("ZC_FAR", 0), A = env("ZC_A", 8), F = env("ZC_F", 12), HS = env("ZC_HS", 15),
            HL = env("ZC_HL", 13), PRIME = env("ZC_PRIME", 131072), PROP = env("ZC_PROP", 0), PRI = env("ZC_PRI", 0),
            SEG = env("ZC_SEG", 8);
  const uint32_t BS = 32768, TILE = env("ZC_TILE", 1024), CAP = 16;
  oc_params op;
  if (P == 512) oc_params_init(&op, 524288, 1048576, 8388608, 1);
  else oc_params_init(&op, 16384, 65536, 262144, 1);
  std::vector<oc_chunk> ch(n / 16383 + 2);
  const size_t nch = oc_chunk_slice(&op, d.data(), n, ch.data(), ch.size());
  void *zh = dlopen("libzstd.so.1", RTLD_NOW);
  auto zcreate = (void *(*)())dlsym(zh, "ZSTD_createCCtx");
  auto zset = (size_t(*)(void *, int, int))dlsym(zh, "ZSTD_CCtx_setParameter");
  auto zstream = (size_t(*)(void *, ZOut *, ZIn *, int))dlsym(zh, "ZSTD_compressStream2");
  auto zfree = (size_t(*)(void *))dlsym(zh, "ZSTD_freeCCtx");
  std::vector<uint8_t> zbuf(20 << 20), buf(1 << 21);
  const ZTables T = build_tables();
  std::vector<uint32_t> hs(1u << HS), hl(1u << HL), ft(1u << F), word;
  double tot = 0, tot_z = 0;
  uint64_t far_words = 0, prop_words = 0;
  for (size_t c = 0; c < nch; ++c) {
    const uint8_t *p = d.data() + ch[c].offset;
    const uint32_t clen = (uint32_t)ch[c].length;
    {
      void *cc = zcreate();
      zset(cc, 100, 3);
      zset(cc, 101, 20);
      zset(cc, 201, 0);
      zset(cc, 200, 0);
      ZIn in{p, clen, 0};
      ZOut out{zbuf.data(), zbuf.size(), 0};
      zstream(cc, &out, &in, 0);
      while (zstream(cc, &out, &in, 2) != 0) {
      }
      tot_z += out.pos;
      zfree(cc);
    }
    word.assign(clen + 1, 0);  // match length << 24 | offset
    auto key = [&](uint32_t q, uint32_t &m5, uint32_t &m8) {
      uint32_t lo, hi;
      std::memcpy(&lo, p + q, 4);
      std::memcpy(&hi, p + q + 4, 4);
      m5 = mix5(lo, hi);
      m8 = mix8(lo, hi);
    };
    // anchors: hf = m8 * K; anchor iff the top A bits are 0; slot the next F bits, tag the low 9
    auto far_hash = [&](uint32_t m8) { return m8 * 0x2545F491u; };
    auto is_anchor = [&](uint32_t q, uint32_t hf) { return q + 8 <= clen && (hf >> (32 - A)) == 0; };
    auto fslot = [&](uint32_t hf) { return (hf >> (32 - A - F)) & ((1u << F) - 1); };
    const uint32_t segb = SEG ? SEG * BS : 0xFFFFFFFFu;
    for (uint32_t seg0 = 0; seg0 < clen; seg0 += segb) {
      const uint32_t seg1 = std::min<uint64_t>(clen, (uint64_t)seg0 + segb);
      const uint32_t prime0 = seg0 > (uint32_t)PRIME ? seg0 - PRIME : 0;
      std::fill(hs.begin(), hs.end(), 0);
      std::fill(hl.begin(), hl.end(), 0);
      if (FAR) {  // preload: every anchor of [seg0 - 5 segments, seg0), latest per slot
        std::fill(ft.begin(), ft.end(), 0);
        const uint32_t f0 = seg0 > 5 * 262144 ? seg0 - 5 * 262144 : 0;
        for (uint32_t q = f0; q < seg0; ++q) {
          uint32_t m5, m8;
          key(q, m5, m8);
          const uint32_t hf = far_hash(m8);
          if (is_anchor(q, hf)) ft[fslot(hf)] = (q + 1) << 9 | (hf & 511);
        }
      }
      for (uint32_t t0 = prime0; t0 < seg1; t0 += TILE) {
        const uint32_t t1 = std::min(seg1, t0 + TILE);
        const bool find = t0 >= seg0;
        std::vector<uint32_t> cand(TILE, 0), farc(TILE, 0);
        std::vector<uint8_t> loc(TILE, 0);
        for (uint32_t q = t0; q < t1 && find; ++q) {
          uint32_t m5, m8;
          key(q, m5, m8);
          const bool vs = q + 5 <= clen, vl = q + 8 <= clen;
          const uint32_t es = vs ? hs[m5 >> (32 - HS)] : 0, el = vl ? hl[m8 >> (32 - HL)] : 0;
          const uint32_t gs = (m5 >> (32 - HS - 13)) & 0x1FFF, gl = (m8 >> (32 - HL - 13)) & 0x1FFF;
          const uint32_t cl = prime0 + (el >> 13) - 1, cs = prime0 + (es >> 13) - 1;
          const bool okl = el && (el & 0x1FFF) == gl && q - cl <= kWindow;
          const bool oks = es && (es & 0x1FFF) == gs && q - cs <= kWindow;
          uint32_t qc = okl ? cl : oks ? cs : q;
          static const int both = env("ZC_BOTH", 0);
          if (both && okl && oks) {  // (model only: the longer of the two)
            auto ml = [&](uint32_t c) { uint32_t m = 0; while (m < 16 && q + m < clen && p[c + m] == p[q + m]) ++m; return m; };
            if (ml(cs) > ml(cl)) qc = cs;
          }
          loc[q - t0] = okl || oks;
          if (FAR) {
            const uint32_t hf = far_hash(m8);
            if (is_anchor(q, hf)) {
              const uint32_t e = ft[fslot(hf)];
              const uint32_t cf = (e >> 9) - 1;
              if (e && (e & 511) == (hf & 511) && cf < q && q - cf <= kWindow) {
                farc[q - t0] = cf + 1;
                if (PRI == 0 || !loc[q - t0]) qc = cf, loc[q - t0] = 2;
              }
            }
          }
          cand[q - t0] = qc;
        }
        if (FAR && PROP && find) {  // positions without a candidate: the offset of a far-matched anchor of the wave
          for (uint32_t w0 = t0; w0 < t1; w0 += 64) {
            for (uint32_t q = w0; q < std::min(t1, w0 + 64); ++q) {
              if (loc[q - t0]) continue;
              int best = -1;
              for (uint32_t a = w0; a < std::min(t1, w0 + 64); ++a)
                if (farc[a - t0] && (PROP == 2 || a >= q)) {
                  if (best < 0 || (PROP == 2 ? std::abs((int)a - (int)q) < std::abs(best - (int)q)
                                             : (int)a < best))
                    best = (int)a;
                }
              if (best >= 0) {
                const uint32_t off = best - (farc[best - t0] - 1);
                if (off <= q) cand[q - t0] = q - off, loc[q - t0] = 3;
              }
            }
          }
        }
        for (uint32_t q = t0; q < t1 && find; ++q) {  // verify 16 bytes within the block
          const uint32_t qc = cand[q - t0];
          if (qc == q) continue;
          const uint32_t bend = std::min(clen, (q / BS + 1) * BS), lim = std::min(CAP, bend - q);
          uint32_t m = 0;
          while (m < lim && p[qc + m] == p[q + m]) ++m;
          if (m >= kMinMatch) {
            word[q] = m << 24 | (q - qc);
            far_words += loc[q - t0] == 2;
            prop_words += loc[q - t0] == 3;
          }
        }
        for (uint32_t q = t0; q < t1; ++q) {  // inserts
          uint32_t m5, m8;
          key(q, m5, m8);
          const uint32_t r = (q - prime0 + 1) << 13;
          static const uint32_t SS = env("ZC_SS", 1), LS = env("ZC_LS", 1);
          if (q % SS == 0 && q + 5 <= clen) hs[m5 >> (32 - HS)] = std::max(hs[m5 >> (32 - HS)], r | ((m5 >> (32 - HS - 13)) & 0x1FFF));
          if (q % LS == 0 && q + 8 <= clen) hl[m8 >> (32 - HL)] = std::max(hl[m8 >> (32 - HL)], r | ((m8 >> (32 - HL - 13)) & 0x1FFF));
          if (FAR) {
            const uint32_t hf = far_hash(m8);
            if (is_anchor(q, hf)) ft[fslot(hf)] = std::max(ft[fslot(hf)], (q + 1) << 9 | (hf & 511));
          }
        }
      }
    }
    // ZC_POST=B: the far pass after the finder (FAR=0): anchors of each
    // segment look up the latest anchor per slot of the 5 segments before it
    // (their own segment's are not seen), verify 16 bytes, extend backwards
    // up to B bytes, and overwrite the words of [start, anchor] with the far
    // offset (the parse extends it)
    static const int POST = env("ZC_POST", 0);
    if (POST) {
      const uint32_t S = 262144, nseg = (clen + S - 1) / S;
      std::vector<std::vector<uint32_t>> tabs(nseg, std::vector<uint32_t>(1u << F, 0));
      std::vector<std::vector<uint32_t>> anc(nseg);
      for (uint32_t q = 0; q + 8 <= clen; ++q) {
        uint32_t m5, m8;
        key(q, m5, m8);
        const uint32_t hf = far_hash(m8);
        if (!is_anchor(q, hf)) continue;
        tabs[q / S][fslot(hf)] = (q + 1) << 9 | (hf & 511);
        anc[q / S].push_back(q);
      }
      for (uint32_t s = 1; s < nseg; ++s)
        for (uint32_t q : anc[s]) {
          uint32_t m5, m8;
          key(q, m5, m8);
          const uint32_t hf = far_hash(m8);
          uint32_t cf = 0xFFFFFFFFu;
          for (uint32_t k = 1; k <= 5 && k <= s; ++k) {
            const uint32_t e = tabs[s - k][fslot(hf)];
            if (e && (e & 511) == (hf & 511) && q - ((e >> 9) - 1) <= kWindow) {
              cf = (e >> 9) - 1;
              break;
            }
          }
          if (cf == 0xFFFFFFFFu) continue;
          const uint32_t bend = std::min(clen, (q / BS + 1) * BS);
          uint32_t m = 0;
          while (m < CAP && q + m < bend && p[cf + m] == p[q + m]) ++m;
          if (m < CAP) continue;
          const uint32_t off = q - cf;
          uint32_t b = 0;
          while (b < (uint32_t)POST && b < cf && p[q - 1 - b] == p[cf - 1 - b]) ++b;
          for (uint32_t x = q - b; x <= q; ++x) {
            const uint32_t xe = std::min(clen, (x / BS + 1) * BS);
            const uint32_t lim = std::min(CAP, xe - x);
            word[x] = (lim >= kMinMatch ? lim : 0) << 24 | off;
            if (lim < kMinMatch) word[x] = 0;
            ++far_words;
          }
        }
    }
    // greedy parse per block; a capped match extended to its end in the block
    std::vector<uint64_t> seqs;
    std::vector<uint8_t> lits;
    for (uint32_t b0 = 0; b0 < clen; b0 += BS) {
      const uint32_t end = std::min(clen, b0 + BS), blen = end - b0;
      seqs.clear();
      lits.clear();
      uint32_t i = b0, lit0 = b0;
      while (i < end) {
        uint32_t m = word[i] >> 24;
        if (m) {
          const uint32_t off = word[i] & 0xFFFFFF;
          if (m == CAP)
            while (i + m < end && p[i + m] == p[i + m - off]) ++m;
          for (uint32_t k = lit0; k < i; ++k) lits.push_back(p[k]);
          seqs.push_back(seq_pack(i - lit0, m, off));
          i += m;
          lit0 = i;
        } else {
          ++i;
        }
      }
      for (uint32_t k = lit0; k < end; ++k) lits.push_back(p[k]);
      RepHist R{{0, 0, 0}, 0};
      for (auto &s : seqs) s = rep_code(R, s);
      const uint32_t ls = encode_literals([&](uint32_t k) { return (uint32_t)lits[k]; }, (uint32_t)lits.size(),
                                          buf.data());
      const uint32_t ss = encode_sequences_auto(T, [&](uint32_t k) { return seqs[k]; }, (uint32_t)seqs.size(),
                                                buf.data() + ls, (uint32_t)(buf.size() - ls));
      const double blk = (ss ? ls + ss : 1e9);
      tot += 3 + std::min<double>(blk, blen) + (b0 == 0 ? 6 : 0);
    }
  }
  std::printf("P%d far %d A %d F %d HS %d HL %d prime %d prop %d pri %d seg %d | far %.4f prop %.4f /B | "
              "ratio %.4f  zstd-3 %.4f  (%.1f%%)\n",
              P, FAR, A, F, HS, HL, PRIME, PROP, PRI, SEG, (double)far_words / n, (double)prop_words / n, n / tot,
              n / tot_z, 100.0 * (n / tot) / (n / tot_z));
  return 0;
}
