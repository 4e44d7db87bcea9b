// zc_model — CPU model of the GPU zstd parse (k_zc_match) to price format and
// parse choices before writing kernels: greedy LZ per 16 KiB block with a
// hash table of 2^hlog latest positions, matches reaching back `reach` bytes
// within a 64 KiB chunk, min match 4; prints the compressed size with
//   raw   raw literals + predefined FSE (the round-3 first cut)
//   huf   Huffman literals + predefined FSE (the current kernels)
//   fse   Huffman literals + per-block FSE tables (entropy + ~table cost)
//   rep   as fse with zstd repeat offset 1 used where it matches
// Usage: zc_model file [hlog reach chunk minmatch hashbytes]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mapache_amd/csrc/mcdc_zstd.h"

using namespace mcdc::zs;

static double entropy_bytes(const std::vector<uint32_t> &cnt, uint64_t n) {
  double b = 0;
  for (uint32_t c : cnt)
    if (c) b -= c * std::log2((double)c / n);
  return b / 8;
}

int main(int argc, char **argv) {
  FILE *f = std::fopen(argv[1], "rb");
  std::vector<uint8_t> d;
  {
    std::fseek(f, 0, SEEK_END);
    d.resize(std::ftell(f));
    std::fseek(f, 0, SEEK_SET);
    if (std::fread(d.data(), 1, d.size(), f) != d.size()) return 1;
  }
  const uint32_t hlog = argc > 2 ? std::atoi(argv[2]) : 11;
  const uint32_t reach = argc > 3 ? std::atoi(argv[3]) : 32768;
  const uint32_t chunk = argc > 4 ? std::atoi(argv[4]) : 65536;
  const uint32_t minm = argc > 5 ? std::atoi(argv[5]) : 4;
  const uint32_t hb = argc > 6 ? std::atoi(argv[6]) : 4;  // bytes hashed
  auto H = [&](const uint8_t *q) -> uint32_t {
    uint64_t v;
    std::memcpy(&v, q, 8);
    return (uint32_t)(((v << (64 - 8 * hb)) * 0xCF1BBCDCB7A56463ull) >> (64 - hlog));
  };
  const ZTables T = build_tables();
  double tot_raw = 0, tot_huf = 0, tot_fse = 0, tot_rep = 0;
  uint64_t nseq_all = 0, nlit_all = 0;
  std::vector<uint32_t> ht(1u << hlog);
  std::vector<uint64_t> seqs;
  std::vector<uint8_t> lits, buf(1 << 20);
  for (size_t c0 = 0; c0 < d.size(); c0 += chunk) {
    const uint8_t *p = d.data() + c0;
    const uint32_t clen = (uint32_t)std::min<size_t>(chunk, d.size() - c0);
    std::fill(ht.begin(), ht.end(), 0);
    for (uint32_t b0 = 0; b0 < clen; b0 += 16384) {
      const uint32_t end = std::min(clen, b0 + 16384);
      // prime: positions [max(0, b0 - (reach - 16384)), b0) already in the table (sequential model)
      if (b0) {
        std::fill(ht.begin(), ht.end(), 0);
        const uint32_t s = b0 > reach - 16384 ? b0 - (reach - 16384) : 0;
        for (uint32_t q = s; q + 4 <= b0; ++q) ht[H(p + q)] = q + 1;
      }
      seqs.clear();
      lits.clear();
      uint32_t i = b0, lit0 = b0;
      while (i + 8 <= end) {
        const uint32_t v = *(const uint32_t *)(p + i);
        const uint32_t h = H(p + i);
        const uint32_t cand = ht[h];
        ht[h] = i + 1;
        uint32_t ml = 0;
        if (cand) {
          const uint32_t c = cand - 1;
          if (i - c <= reach && *(const uint32_t *)(p + c) == v) {
            while (i + ml < end && p[c + ml] == p[i + ml]) ++ml;
          }
          if (ml >= minm) {
            for (uint32_t k = lit0; k < i; ++k) lits.push_back(p[k]);
            seqs.push_back(seq_pack(i - lit0, ml, i - c));
            i += ml;
            lit0 = i;
            continue;
          }
        }
        ++i;
      }
      for (uint32_t k = lit0; k < end; ++k) lits.push_back(p[k]);
      const uint32_t blen = end - b0;
      nseq_all += seqs.size();
      nlit_all += lits.size();
      const uint32_t ss = encode_sequences(T, [&](uint32_t k) { return seqs[k]; }, (uint32_t)seqs.size(), buf.data(),
                                           (uint32_t)buf.size());
      // literals: Huffman estimate (entropy + 40-byte tree/jump overhead)
      std::vector<uint32_t> lc(256);
      for (uint8_t x : lits) lc[x]++;
      const double huf = lits.size() >= 32 ? std::min<double>(3 + lits.size(), 5 + entropy_bytes(lc, lits.size()) * 1.02 + 40)
                                           : 3 + lits.size();
      // per-block FSE: code entropies + extra bits + ~25 bytes of tables
      std::vector<uint32_t> cl(64), cm(64), co(64), co2(64);
      double extra = 0, extra_rep = 0;
      uint32_t rep = 0;
      for (uint64_t s : seqs) {
        const uint32_t ll = seq_ll(s), mb = seq_ml(s) - 3, ob = seq_off(s) + 3;
        cl[ll_code(ll)]++;
        cm[ml_code(mb)]++;
        co[highbit(ob)]++;
        extra += ll_bits(ll_code(ll)) + ml_bits(ml_code(mb)) + highbit(ob);
        if (seq_off(s) == rep && ll) {
          co2[0]++;
          extra_rep += ll_bits(ll_code(ll)) + ml_bits(ml_code(mb));
        } else {
          co2[highbit(ob)]++;
          extra_rep += ll_bits(ll_code(ll)) + ml_bits(ml_code(mb)) + highbit(ob);
        }
        rep = seq_off(s);
      }
      const uint64_t n = seqs.size();
      const double fse = n ? 4 + entropy_bytes(cl, n) + entropy_bytes(cm, n) + entropy_bytes(co, n) + extra / 8 + 25 : 1;
      const double fse_rep = n ? 4 + entropy_bytes(cl, n) + entropy_bytes(cm, n) + entropy_bytes(co2, n) + extra_rep / 8 + 25 : 1;
      auto pick = [&](double x) { return 3 + std::min<double>(x, blen); };
      tot_raw += pick(ss ? 3 + lits.size() + ss : 1e9);
      tot_huf += pick(huf + ss);
      tot_fse += pick(huf + std::min<double>(fse, ss));
      tot_rep += pick(huf + std::min<double>(fse_rep, ss));
    }
  }
  std::printf("hlog %u reach %u chunk %u minm %u: seq/blk-byte %.4f lit frac %.3f | ratio raw %.3f huf %.3f fse %.3f rep %.3f\n",
              hlog, reach, chunk, minm, (double)nseq_all / d.size(), (double)nlit_all / d.size(), d.size() / tot_raw,
              d.size() / tot_huf, d.size() / tot_fse, d.size() / tot_rep);
  return 0;
}
