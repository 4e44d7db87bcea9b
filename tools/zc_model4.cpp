// zc_model4 — CPU model of the GPU compressor on many small files (the
// configs[3] kernel-tree mix; tools only).  Splits the ratio gap to libzstd
// level 3 into its two halves:
//   zstd      the crate's encoder (streaming, level 3, window log 20:
//             storage.rs:74-84), file by file
//   zseq      libzstd's own sequences (ZSTD_generateSequences, level 3) coded
//             by the GPU's entropy stage (mcdc_zstd.h): the entropy stage's
//             share of the gap
//   gpu       the finder as modelled (tiles of ZC_TILE positions that read the
//             tables as earlier tiles left them, ZC_HS / ZC_HL slot logs,
//             13-bit tags, one verified candidate or ZC_BOTH the longer of the
//             two, ZC_REP: the previous match's offset tried first at each
//             position) and the greedy parse, coded by the same entropy stage
// Files above 32 KiB (one GPU block) are split in 32 KiB blocks for gpu and
// zseq alike (zseq: sequences cut at the block edges).
//
// Usage: zc_model4 arena sizes(u64 LE) [maxfiles]
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mapache_amd/csrc/mcdc_zstd.h"

using namespace mcdc::zs;

static uint32_t u24(uint32_t x, uint32_t k) { return (uint32_t)((uint64_t)(x & 0xFFFFFF) * k); }
static uint32_t mix5(uint32_t lo, uint32_t hi) { return u24(lo & 0xFFFFFF, 0x9E3779u) + u24(lo >> 24 | (hi & 0xFF) << 8, 0xC2B2AFu); }
static uint32_t mix8(uint32_t lo, uint32_t hi) {
  return u24(lo & 0xFFFFFF, 0x85EBCBu) ^ u24(lo >> 24 | (hi & 0xFFFF) << 8, 0x27D4EBu) ^ u24(hi >> 16, 0x165667u);
}
static int env(const char *k, int d) { return getenv(k) ? atoi(getenv(k)) : d; }
static int HSg, HLg, TILEg;

struct ZIn { const void *src; size_t size, pos; };
struct ZOut { void *dst; size_t size, pos; };
struct ZSeq { unsigned offset, litLength, matchLength, rep; };

static std::vector<uint8_t> slurp(const char *path) {
  std::vector<uint8_t> d;
  FILE *f = std::fopen(path, "rb");
  if (!f) return d;
  std::fseek(f, 0, SEEK_END);
  d.resize(std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (std::fread(d.data(), 1, d.size(), f) != d.size()) d.clear();
  std::fclose(f);
  return d;
}

int main(int argc, char **argv) {
  std::vector<uint8_t> d = slurp(argv[1]), sz = slurp(argv[2]);
  const size_t nfiles_all = sz.size() / 8, maxf = argc > 3 ? (size_t)atol(argv[3]) : nfiles_all;
  const size_t nfiles = std::min(nfiles_all, maxf);
  const uint64_t *len = reinterpret_cast<const uint64_t *>(sz.data());
  d.resize(d.size() + 64, 0);
  HSg = env("ZC_HS", 15), HLg = env("ZC_HL", 13), TILEg = env("ZC_TILE", 1024);
  const int BOTH = env("ZC_BOTH", 0),
            REP = env("ZC_REP", 0), LAZY = env("ZC_LAZY", 0);
  const uint32_t BS = 32768, CAP = 16;
  // ZC_SMALL: files up to this many bytes take the small finder (tiles of
  // ZC_STILE positions, tables sized to the file: short log = ceil(log2 L) +
  // ZC_SADJ clamped to [10, ZC_SMAX], long log one less)
  const int SMALL = env("ZC_SMALL", 0), STILE = env("ZC_STILE", 64), SADJ = env("ZC_SADJ", 0), SMAX = env("ZC_SMAX", 13);
  double small_lds = 0;
  void *zh = dlopen("libzstd.so.1", RTLD_NOW);
  auto zcreate = (void *(*)())dlsym(zh, "ZSTD_createCCtx");
  auto zset = (size_t(*)(void *, int, int))dlsym(zh, "ZSTD_CCtx_setParameter");
  auto zstream = (size_t(*)(void *, ZOut *, ZIn *, int))dlsym(zh, "ZSTD_compressStream2");
  auto zgen = (size_t(*)(void *, ZSeq *, size_t, const void *, size_t))dlsym(zh, "ZSTD_generateSequences");
  auto zfree = (size_t(*)(void *))dlsym(zh, "ZSTD_freeCCtx");
  std::vector<uint8_t> zbuf(4 << 20), buf(1 << 21);
  std::vector<ZSeq> zs_(1 << 20);
  const ZTables T = build_tables();
  std::vector<uint32_t> hs(1u << 16), hl(1u << 16), word;
  double tot_in = 0, tot_z = 0, tot_zseq = 0, tot_g = 0, small_in = 0, small_z = 0, small_zseq = 0, small_g = 0;
  uint64_t nlit_z = 0, nlit_g = 0, nseq_z = 0, nseq_g = 0;
  // the entropy stage over one block's literals and sequences (sizes as the GPU frames them)
  auto code_block = [&](const std::vector<uint8_t> &lits, std::vector<uint64_t> &seqs, uint32_t blen, bool first) {
    RepHist R{{0, 0, 0}, 0};
    for (auto &s : seqs) s = rep_code(R, s);
    const uint32_t ls = encode_literals([&](uint32_t k) { return (uint32_t)lits[k]; }, (uint32_t)lits.size(), buf.data());
    const uint32_t ss = encode_sequences_auto(T, [&](uint32_t k) { return seqs[k]; }, (uint32_t)seqs.size(),
                                              buf.data() + ls, (uint32_t)(buf.size() - ls));
    const double blk = ss ? ls + ss : 1e9;
    return 3 + std::min<double>(blk, blen) + (first ? 6 : 0);
  };
  size_t at = 0;
  for (size_t f = 0; f < nfiles; at += len[f], ++f) {
    const uint8_t *p = d.data() + at;
    const uint32_t clen = (uint32_t)len[f];
    double z = 0, zq = 0, g = 0;
    {  // the crate's encoder
      void *cc = zcreate();
      zset(cc, 100, 3);
      zset(cc, 101, 20);
      zset(cc, 201, 0);
      ZIn in{p, clen, 0};
      ZOut out{zbuf.data(), zbuf.size(), 0};
      zstream(cc, &out, &in, 0);
      while (zstream(cc, &out, &in, 2) != 0) {
      }
      z = (double)out.pos;
      zfree(cc);
    }
    {  // libzstd's sequences, the GPU's entropy stage, cut at 32 KiB blocks
      void *cc = zcreate();
      zset(cc, 100, 3);
      zset(cc, 101, 20);
      const size_t ns = zgen(cc, zs_.data(), zs_.size(), p, clen);
      zfree(cc);
      std::vector<uint8_t> lits;
      std::vector<uint64_t> seqs;
      uint32_t pos = 0, b0 = 0, run = 0;  // run: literals since the block's previous sequence
      auto flush = [&](uint32_t bend) {
        run = 0;
        zq += code_block(lits, seqs, bend - b0, b0 == 0);
        nlit_z += lits.size();
        nseq_z += seqs.size();
        lits.clear();
        seqs.clear();
        b0 = bend;
      };
      for (size_t k = 0; k < ns; ++k) {
        uint32_t ll = zs_[k].litLength, ml = zs_[k].matchLength;
        const uint32_t off = zs_[k].offset;
        while (ll) {  // literals, cut at block edges
          const uint32_t take = std::min(ll, b0 + BS - pos);
          for (uint32_t i = 0; i < take; ++i) lits.push_back(p[pos + i]);
          run += take;
          pos += take, ll -= take;
          if (pos == b0 + BS) flush(pos);
        }
        if (!ml) continue;
        // a match cut at the block edge: the part past it becomes literals
        // of the next block when shorter than 3 (rare)
        while (ml) {
          const uint32_t take = std::min(ml, b0 + BS - pos);
          if (take >= 3 && off <= pos) {
            seqs.push_back(seq_pack(run, take, off));
            run = 0;
          } else {
            for (uint32_t i = 0; i < take; ++i) lits.push_back(p[pos + i]);
            run += take;
          }
          pos += take, ml -= take;
          if (pos == b0 + BS) flush(pos);
        }
      }
      if (pos > b0 || clen == 0) flush(clen);
    }
    {  // the GPU finder as modelled
      int HS = ::HSg, HL = ::HLg;
      uint32_t TILE = (uint32_t)::TILEg;
      static const int CLS = env("ZC_CLASSES", 0);
      if (CLS && clen <= 32768) {  // the small finder's classes: (len <=, HS, HL, tile)
        static const uint32_t tab[4][4] = {{4096, 11, 10, 64}, {8192, 12, 11, 64}, {16384, 12, 11, 128},
                                           {32768, 13, 12, 256}};
        static const int C1HS = env("ZC_C1HS", 12), C2T = env("ZC_C2T", 256), C1T = env("ZC_C1T", 128);
        for (auto &t : tab)
          if (clen <= t[0]) {
            HS = (int)t[1], HL = (int)t[2], TILE = t[3];
            if (t[0] == 16384) HS = C1HS, HL = C1HS - 1, TILE = C1T;
            if (t[0] == 32768) TILE = C2T, HL = env("ZC_C2HL", 12);
            if (t[0] == 8192) TILE = env("ZC_BT", 64);
            break;
          }
        small_lds += 4.0 * ((1 << HS) + (1 << HL));
      } else if (clen <= (uint32_t)SMALL) {
        int lg = 10;
        while ((1u << lg) < clen) ++lg;
        HS = std::min(SMAX, std::max(10, lg + SADJ));
        HL = HS - 1;
        TILE = STILE;
        small_lds += 4.0 * ((1 << HS) + (1 << HL));
      }
      word.assign(clen + 1, 0);
      std::fill(hs.begin(), hs.begin() + (1u << HS), 0);
      std::fill(hl.begin(), hl.begin() + (1u << HL), 0);
      auto key = [&](uint32_t q, uint32_t &m5, uint32_t &m8) {
        uint32_t lo, hi;
        std::memcpy(&lo, p + q, 4);
        std::memcpy(&hi, p + q + 4, 4);
        m5 = mix5(lo, hi);
        m8 = mix8(lo, hi);
      };
      auto mlen = [&](uint32_t q, uint32_t c) {
        const uint32_t bend = std::min(clen, (q / BS + 1) * BS), lim = std::min(CAP, bend - q);
        uint32_t m = 0;
        while (m < lim && p[c + m] == p[q + m]) ++m;
        return m;
      };
      std::vector<uint32_t> cand(TILE + 1), cand2(TILE + 1);
      for (uint32_t t0 = 0; t0 < clen; t0 += TILE) {
        const uint32_t t1 = std::min(clen, t0 + TILE);
        for (uint32_t q = t0; q < t1; ++q) {
          uint32_t m5, m8;
          key(q, m5, m8);
          const bool vs = q + 5 <= clen, vl = q + 8 <= clen;
          const uint32_t es = vs ? hs[m5 >> (32 - HS)] : 0, el = vl ? hl[m8 >> (32 - HL)] : 0;
          const uint32_t gs = (m5 >> (32 - HS - 13)) & 0x1FFF, gl = (m8 >> (32 - HL - 13)) & 0x1FFF;
          const uint32_t cl = (el >> 13) - 1, cs = (es >> 13) - 1;
          const bool okl = el && (el & 0x1FFF) == gl, oks = es && (es & 0x1FFF) == gs;
          cand[q - t0] = okl ? cl : oks ? cs : q;
          cand2[q - t0] = BOTH && okl && oks ? cs : q;
        }
        for (uint32_t q = t0; q < t1; ++q) {
          uint32_t best = 0, boff = 0;
          for (uint32_t c : {cand[q - t0], cand2[q - t0]}) {
            if (c == q) continue;
            const uint32_t m = mlen(q, c);
            if (m > best) best = m, boff = q - c;
          }
          if (best >= kMinMatch) word[q] = best << 24 | boff;
        }
        for (uint32_t q = t0; q < t1; ++q) {
          uint32_t m5, m8;
          key(q, m5, m8);
          const uint32_t r = (q + 1) << 13;
          if (q + 5 <= clen) hs[m5 >> (32 - HS)] = std::max(hs[m5 >> (32 - HS)], r | ((m5 >> (32 - HS - 13)) & 0x1FFF));
          if (q + 8 <= clen) hl[m8 >> (32 - HL)] = std::max(hl[m8 >> (32 - HL)], r | ((m8 >> (32 - HL - 13)) & 0x1FFF));
        }
      }
      std::vector<uint64_t> seqs;
      std::vector<uint8_t> lits;
      for (uint32_t b0 = 0; b0 < clen || (clen == 0 && b0 == 0); b0 += BS) {
        const uint32_t end = std::min(clen, b0 + BS), blen = end - b0;
        seqs.clear();
        lits.clear();
        uint32_t i = b0, lit0 = b0, prev = 0;
        while (i < end) {
          uint32_t m = word[i] >> 24, off = word[i] & 0xFFFFFF;
          if (REP && prev && i >= prev && i + 4 <= end) {  // the previous offset at this position
            uint32_t mr = 0;
            while (i + mr < end && mr < 64 && p[i + mr] == p[i + mr - prev]) ++mr;
            if (mr >= 4 && mr >= m) m = mr, off = prev;
          }
          if (m && LAZY && i + 1 < end && (word[i + 1] >> 24) > m + 1) {  // (model: one step of lazy)
            ++i;
            continue;
          }
          if (m) {
            if (m == CAP)
              while (i + m < end && p[i + m] == p[i + m - off]) ++m;
            else if (m > CAP || (REP && off == prev))
              while (i + m < end && p[i + m] == p[i + m - off]) ++m;
            for (uint32_t k = lit0; k < i; ++k) lits.push_back(p[k]);
            seqs.push_back(seq_pack(i - lit0, m, off));
            prev = off;
            i += m;
            lit0 = i;
          } else {
            ++i;
          }
        }
        for (uint32_t k = lit0; k < end; ++k) lits.push_back(p[k]);
        nlit_g += lits.size();
        nseq_g += seqs.size();
        g += code_block(lits, seqs, blen, b0 == 0);
        if (clen == 0) break;
      }
    }
    tot_in += clen, tot_z += z, tot_zseq += zq, tot_g += g;
    if (clen <= 8192) small_in += clen, small_z += z, small_zseq += zq, small_g += g;
  }
  std::printf("small %d stile %d sadj %d smax %d (avg small LDS %.0f) ", SMALL, STILE, SADJ, SMAX, small_lds / nfiles);
  std::printf("files %zu  TILE %d HS %d HL %d BOTH %d REP %d LAZY %d | ratio zstd-3 %.4f  zseq %.4f (%.1f%%)  gpu %.4f "
              "(%.1f%%) | <=8KiB: zstd %.4f zseq %.4f gpu %.4f | lit/B z %.3f g %.3f seq/KiB z %.2f g %.2f\n",
              nfiles, TILEg, HSg, HLg, BOTH, REP, LAZY, tot_in / tot_z, tot_in / tot_zseq, 100.0 * tot_z / tot_zseq,
              tot_in / tot_g, 100.0 * tot_z / tot_g, small_in / small_z, small_in / small_zseq, small_in / small_g,
              nlit_z / tot_in, nlit_g / tot_in, nseq_z * 1024.0 / tot_in, nseq_g * 1024.0 / tot_in);
  return 0;
}
