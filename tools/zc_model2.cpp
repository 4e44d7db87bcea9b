// zc_model2 — CPU model of the round-4 GPU zstd parse (tools only: prices
// parse choices before kernels are written; exact sizes from the real format
// pieces of mcdc_zstd.h).  The input is cut by the FastCDC oracle at
// 16/64/256 KiB (the bench's chunks); each chunk is one frame of blocks.
//
// Per position p of a chunk, candidates come from hash tables of the latest
// positions with the same key, filled TILE positions at a time (the GPU reads
// a tile's candidates before it inserts the tile's positions; intra=1 models
// exact most-recent semantics instead): a short table (hb-byte key, 2^hlog
// entries) and optionally a long one (8-byte key, 2^llog).  Match length = the
// longer verified candidate, within the block, >= minm.  The parse per block
// is greedy or lazy (lazy=1: a match is deferred when the next position's is
// longer by `lazyd` or more).  Offsets use repeat codes the block set
// (rep_code).  Literals: encode_literals (Huffman over 256 symbols, FSE
// weights); sequences: encode_sequences_auto (per-block FSE tables).
// libzstd level 3 (window log 20) on the same chunks for comparison.
//
// Usage: zc_model2 file [bs hlog tile lazy minm hb llog intra lazyd maxbytes reach]
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mapache_amd/csrc/mcdc_zstd.h"
extern "C" {
#include "../oracle/fastcdc_oracle.h"
}

using namespace mcdc::zs;

static uint64_t rd64(const uint8_t *q) {
  uint64_t v;
  std::memcpy(&v, q, 8);
  return v;
}

int main(int argc, char **argv) {
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  std::vector<uint8_t> d;
  std::fseek(f, 0, SEEK_END);
  d.resize(std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (std::fread(d.data(), 1, d.size(), f) != d.size()) return 1;
  std::fclose(f);
  auto arg = [&](int i, long dflt) { return argc > i ? std::atol(argv[i]) : dflt; };
  const uint32_t bs = arg(2, 16384), hlog = arg(3, 14), tile = arg(4, 256), lazy = arg(5, 0), minm = arg(6, 4),
                 hb = arg(7, 5), llog = arg(8, 0), intra = arg(9, 0), lazyd = arg(10, 1);
  const size_t maxbytes = arg(11, 16 << 20);
  const uint32_t reach = arg(12, kWindow);  // largest offset (16-bit table entries: 65535)
  if (d.size() > maxbytes) d.resize(maxbytes);
  d.resize(d.size() + 64, 0);  // (8-byte keys read past the end)
  const size_t n = d.size() - 64;
  oc_params P;
  oc_params_init(&P, 16384, 65536, 262144, 1);
  std::vector<oc_chunk> ch(n / 16383 + 2);
  const size_t nch = oc_chunk_slice(&P, d.data(), n, ch.data(), ch.size());
  // libzstd level 3 for comparison
  void *zh = dlopen("libzstd.so.1", RTLD_NOW);
  auto zc = (size_t(*)(void *, size_t, const void *, size_t, int))dlsym(zh, "ZSTD_compress");
  const ZTables T = build_tables();
  std::vector<uint32_t> st(1u << hlog), lt(llog ? 1u << llog : 1);
  std::vector<uint32_t> ml, off;
  std::vector<uint64_t> seqs;
  std::vector<uint8_t> lits, buf(1 << 21), zbuf(1 << 20);
  double tot = 0, tot_z = 0;
  uint64_t nseq_all = 0, nlit_all = 0, nrep = 0;
  const int hk = getenv("ZC_HASH") ? atoi(getenv("ZC_HASH")) : 0;  // 1: the GPU's 32-bit forms
  auto u24 = [](uint32_t x, uint32_t k) { return (uint32_t)((uint64_t)(x & 0xFFFFFF) * k); };
  auto hshort = [&](const uint8_t *q) {
    const uint64_t v = rd64(q);
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (hk == 1) return (u24(lo & 0xFFFFFF, 0x9E3779u) + u24(lo >> 24 | (hi & 0xFF) << 8, 0xC2B2AFu)) >> (32 - hlog);
    if (hk == 2) return (lo * 2654435761u + (hi & 0xFFu) * 0x85EBCA77u) >> (32 - hlog);
    return (uint32_t)(((rd64(q) << (64 - 8 * hb)) * 0xCF1BBCDCB7A56463ull) >> (64 - hlog));
  };
  auto hlong = [&](const uint8_t *q) {
    const uint64_t v = rd64(q);
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (hk == 1)
      return (u24(lo & 0xFFFFFF, 0x85EBCBu) ^ u24(lo >> 24 | (hi & 0xFFFF) << 8, 0x27D4EBu) ^ u24(hi >> 16, 0x165667u)) >>
             (32 - llog);
    return (uint32_t)((rd64(q) * 0x9E3779B185EBCA87ull) >> (64 - llog));
  };
  for (size_t c = 0; c < nch; ++c) {
    const uint8_t *p = d.data() + ch[c].offset;
    const uint32_t clen = (uint32_t)ch[c].length;
    tot_z += zc(zbuf.data(), zbuf.size(), p, clen, 3);
    std::fill(st.begin(), st.end(), 0);
    std::fill(lt.begin(), lt.end(), 0);
    ml.assign(clen + 1, 0);
    off.assign(clen + 1, 0);
    // candidates, tile by tile
    for (uint32_t t0 = 0; t0 < clen; t0 += tile) {
      const uint32_t t1 = std::min(clen, t0 + tile);
      for (uint32_t q = t0; q < t1; ++q) {
        const uint32_t bend = std::min(clen, (q / bs + 1) * bs);
        uint32_t best = 0, bo = 0;
        auto try_c = [&](uint32_t cand) {
          if (!cand) return;
          const uint32_t cc = cand - 1;
          if (cc >= q || q - cc > reach) return;
          uint32_t m = 0;
          while (q + m < bend && p[cc + m] == p[q + m]) ++m;
          if (m > best) best = m, bo = q - cc;
        };
        const uint32_t hs = hshort(p + q);
        static const int single = getenv("ZC_SINGLE") ? atoi(getenv("ZC_SINGLE")) : 0;
        if (single == 2 && llog) {  // tags: the long candidate if its 8-byte key matches, else the short if its 5 bytes do
          const uint32_t cl = lt[hlong(p + q)], cs = st[hs];
          auto keyeq = [&](uint32_t c, uint32_t nbk) {
            return c && c - 1 < q && q - (c - 1) <= reach && std::memcmp(p + c - 1, p + q, nbk) == 0;
          };
          if (keyeq(cl, 8)) try_c(cl);
          else if (keyeq(cs, 5)) try_c(cs);
        } else if (single && llog) {  // one candidate verified: the long table's if it has one in reach, else the short's
          const uint32_t cl = lt[hlong(p + q)];
          if (cl && cl - 1 < q && q - (cl - 1) <= reach) try_c(cl);
          else try_c(st[hs]);
        } else {
          try_c(st[hs]);
          if (llog) try_c(lt[hlong(p + q)]);
        }
        if (intra) {
          st[hs] = q + 1;
          if (llog) lt[hlong(p + q)] = q + 1;
        }
        if (best >= minm && q + 8 <= clen) ml[q] = best, off[q] = bo;
      }
      if (!intra)
        for (uint32_t q = t0; q < t1; ++q) {
          st[hshort(p + q)] = q + 1;
          if (llog) lt[hlong(p + q)] = q + 1;
        }
    }
    // parse and encode per block
    for (uint32_t b0 = 0; b0 < clen; b0 += bs) {
      const uint32_t end = std::min(clen, b0 + bs), blen = end - b0;
      seqs.clear();
      lits.clear();
      uint32_t i = b0, lit0 = b0;
      while (i < end) {
        uint32_t m = ml[i];
        if (m && lazy && i + 1 < end && ml[i + 1] >= m + lazyd) m = 0;  // defer: the next position's match is longer
        if (m) {
          for (uint32_t k = lit0; k < i; ++k) lits.push_back(p[k]);
          seqs.push_back(seq_pack(i - lit0, m, off[i]));
          i += m;
          lit0 = i;
        } else {
          ++i;
        }
      }
      for (uint32_t k = lit0; k < end; ++k) lits.push_back(p[k]);
      RepHist R{{0, 0, 0}, 0};
      for (auto &s : seqs) {
        s = rep_code(R, s);
        nrep += seq_ov(s) <= 3;
      }
      nseq_all += seqs.size();
      nlit_all += lits.size();
      const uint32_t ls = encode_literals([&](uint32_t k) { return (uint32_t)lits[k]; }, (uint32_t)lits.size(),
                                          buf.data());
      const uint32_t ss = encode_sequences_auto(T, [&](uint32_t k) { return seqs[k]; }, (uint32_t)seqs.size(),
                                                buf.data() + ls, (uint32_t)(buf.size() - ls));
      const double blk = (ss ? ls + ss : 1e9);
      tot += 3 + std::min<double>(blk, blen) + (b0 == 0 ? 6 : 0);
    }
  }
  std::printf("bs %u hlog %u tile %u lazy %u/%u minm %u hb %u llog %u intra %u | seq/B %.4f lit %.3f rep %.3f | "
              "ratio %.4f  zstd-3 %.4f  (%.1f%%)\n",
              bs, hlog, tile, lazy, lazyd, minm, hb, llog, intra, (double)nseq_all / n, (double)nlit_all / n,
              nseq_all ? (double)nrep / nseq_all : 0.0, n / tot, n / tot_z, 100.0 * (n / tot) / (n / tot_z));
  return 0;
}
