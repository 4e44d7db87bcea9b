// CPU test of mapache_amd/host/zstd_stage.hpp (the zstd half of
// SecureStorage::encode / decode, storage.rs:74-94) under plain, ASan+UBSan
// and TSan builds: many blobs compressed and decompressed on a thread pool,
// round trips, empty blobs, a corrupt frame and a skipped (failed-tag) blob;
// zstd_compress_into's frames equal zstd_compress_all's.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "zstd_stage.hpp"

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                 \
    }                                                             \
  } while (0)

int main(int argc, char **argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  std::mt19937_64 rng(7);
  const char *words[] = {"mapache ", "chunk ", "blob ", "pack ", "index ", "tree ", "snapshot "};
  std::vector<uint8_t> data;
  std::vector<uint64_t> off, len;
  for (int i = 0; i < 300; ++i) {
    off.push_back(data.size());
    const size_t n = i % 17 == 0 ? 0 : rng() % (i % 3 ? 40000 : 300000);
    for (size_t k = 0; k < n;) {
      if (i % 2) {
        data.push_back((uint8_t)rng());
        ++k;
      } else {
        const char *w = words[rng() % 7];
        for (size_t j = 0; w[j] && k < n; ++j, ++k) data.push_back((uint8_t)w[j]);
      }
    }
    len.push_back(n);
  }
  std::vector<std::vector<uint8_t>> comp;
  std::string err = mcdc::host::zstd_compress_all(data.data(), off.data(), len.data(), off.size(), threads, comp);
  CHECK(err.empty());
  if (!err.empty()) std::printf("%s\n", err.c_str());
  // zstd_compress_into (one buffer of bound-sized regions, what
  // mcdc_encode_blobs uses): the same frames, byte for byte
  {
    const mcdc::host::ZstdApi &z = mcdc::host::zstd_api();
    std::vector<uint64_t> bo(off.size() + 1, 0), cl(off.size(), 0);
    for (size_t i = 0; i < off.size(); ++i) bo[i + 1] = bo[i] + z.compressBound(len[i]) + 64;
    std::vector<uint8_t> buf(bo.back());
    err = mcdc::host::zstd_compress_into(data.data(), off.data(), len.data(), off.size(), threads, buf.data(),
                                         bo.data(), cl.data());
    CHECK(err.empty());
    for (size_t i = 0; i < off.size(); ++i) {
      CHECK(cl[i] == comp[i].size());
      if (cl[i] == comp[i].size()) CHECK(std::memcmp(buf.data() + bo[i], comp[i].data(), cl[i]) == 0);
    }
  }
  // frames back to back, one of them corrupted, one skipped
  std::vector<uint8_t> packed;
  std::vector<uint64_t> po, pl;
  for (auto &c : comp) {
    po.push_back(packed.size());
    pl.push_back(c.size());
    packed.insert(packed.end(), c.begin(), c.end());
  }
  const size_t bad = 5, skipped = 6;
  packed[po[bad] + pl[bad] / 2] ^= 0x55;
  std::vector<int32_t> skip(off.size(), 0);
  skip[skipped] = -1;
  std::vector<std::vector<uint8_t>> dec;
  std::vector<int32_t> ok;
  err = mcdc::host::zstd_decompress_all(packed.data(), po.data(), pl.data(), skip.data(), off.size(), threads, dec,
                                        ok);
  CHECK(err.empty());
  for (size_t i = 0; i < off.size(); ++i) {
    if (i == skipped) {
      CHECK(dec[i].empty());
      continue;
    }
    if (i == bad) {  // a flipped byte in the middle of a frame: an error or (for raw blocks) other bytes
      CHECK(ok[i] == -2 || dec[i].size() != len[i] || std::memcmp(dec[i].data(), data.data() + off[i], len[i]));
      continue;
    }
    CHECK(ok[i] == 0);
    CHECK(dec[i].size() == len[i]);
    if (dec[i].size() == len[i] && len[i]) CHECK(std::memcmp(dec[i].data(), data.data() + off[i], len[i]) == 0);
  }
  // a truncated frame is an error, not a short success
  std::vector<uint64_t> to = {po[1]}, tl = {pl[1] - 3};
  err = mcdc::host::zstd_decompress_all(packed.data(), to.data(), tl.data(), nullptr, 1, 1, dec, ok);
  CHECK(err.empty() && ok[0] == -2 && dec[0].empty());
  std::printf(failures ? "FAILED (%d failures)\n" : "ALL PASSED\n", failures);
  return failures ? 1 : 0;
}
