// test_batcher.cpp — the cross-worker batching front-end (mapache_amd/host/
// batcher.hpp) driven by many submitter threads, with the oracle restatement
// as its batch function, so the group-commit logic, the per-file slicing of
// one batch result and the per-caller statuses are checked on the CPU (and,
// built with -fsanitize=thread / address,undefined, race- and memory-checked).
//
// Mirrors the deployment shape: read_concurrency rayon workers each chunking
// their own files (/root/reference/src/archiver/mod.rs:162-215,
// src/global/defaults.rs:22), here 4, 8 and 16 threads.
//
// Usage: test_batcher [threads...]   (exit 0 = pass)
#include "batcher.hpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" {
#include "../../oracle/fastcdc_oracle.h"
}

static int failures = 0;

static void expect(bool ok, const char *name) {
  std::printf("%s %s\n", ok ? "PASS" : "FAIL", name);
  if (!ok) ++failures;
}

static uint64_t rnd(uint64_t &s) {  // splitmix64
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static bool run(int threads, int files_per_thread, const oc_params &op, uint32_t gather_us, size_t max_files) {
  using mcdc::host::Batcher;
  std::atomic<int> calls{0};
  Batcher b(
      [&](const uint8_t *const *bufs, const size_t *lens, size_t k, mcdc_chunk *out, size_t cap, size_t *counts,
          size_t *n_out, std::string *msg) {
        calls.fetch_add(1);
        std::vector<oc_chunk> tmp(cap);
        const size_t t = oc_chunk_files(&op, bufs, lens, k, 1, tmp.data(), cap, counts);
        if (t == (size_t)-1) {
          *msg = "capacity";
          return MCDC_E_CAPACITY;
        }
        for (size_t i = 0; i < t; ++i) out[i] = mcdc_chunk{tmp[i].offset, tmp[i].length, tmp[i].hash};
        *n_out = t;
        return MCDC_OK;
      },
      [&](size_t len) { return len / (op.min_size - 1) + 2; }, 64u << 20, max_files, gather_us);
  std::atomic<int> bad{0}, cap_ok{0}, big_ok{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      uint64_t s = 1000 + t;
      for (int f = 0; f < files_per_thread; ++f) {
        size_t n = (size_t)(rnd(s) % (3u << 20));
        if (f % 17 == 0) n = 0;
        if (f % 23 == 0) n = op.min_size - 1;
        std::vector<uint8_t> d(n);
        oc_fill_random(d.data(), 0, n, rnd(s));
        std::vector<oc_chunk> ref(n / (op.min_size - 1) + 2);
        const size_t rn = oc_chunk_slice(&op, d.data(), n, ref.data(), ref.size());
        const bool small = f % 29 == 5 && rn > 1;  // a too-small output array
        std::vector<mcdc_chunk> got(small ? rn - 1 : ref.size());
        size_t gn = 0;
        std::string err;
        const int rc = b.chunk(d.data(), n, got.data(), got.size(), &gn, &err);
        if (small) {
          if (rc == MCDC_E_CAPACITY && gn == rn) cap_ok.fetch_add(1);
          else bad.fetch_add(1);
          continue;
        }
        bool ok = rc == MCDC_OK && gn == rn;
        for (size_t i = 0; ok && i < rn; ++i)
          ok = got[i].offset == ref[i].offset && got[i].length == ref[i].length && got[i].hash == ref[i].hash;
        if (!ok) bad.fetch_add(1);
      }
      std::vector<uint8_t> huge((64u << 20) + 1);  // over max_batch_bytes
      size_t gn = 0;
      std::string err;
      if (b.chunk(huge.data(), huge.size(), nullptr, 0, &gn, &err) == MCDC_E_TOOBIG) big_ok.fetch_add(1);
    });
  for (auto &t : ts) t.join();
  const auto st = b.stats();
  const uint64_t files = (uint64_t)threads * files_per_thread;
  std::printf("  threads %d files %llu batches %llu (calls %d) max files/batch %llu\n", threads,
              (unsigned long long)st.files, (unsigned long long)st.batches, calls.load(),
              (unsigned long long)st.max_batch_files);
  return bad.load() == 0 && big_ok.load() == threads && cap_ok.load() > 0 && st.files == files &&
         st.batches == (uint64_t)calls.load() && st.max_batch_files <= max_files &&
         (threads == 1 || st.batches < files);
}

int main(int argc, char **argv) {
  oc_params p16;
  oc_params_init(&p16, 16384, 65536, 262144, 1);
  oc_params tiny;
  oc_params_init(&tiny, 64, 256, 1024, 1);
  std::vector<int> tcounts;
  for (int i = 1; i < argc; ++i) tcounts.push_back(std::atoi(argv[i]));
  if (tcounts.empty()) tcounts = {1, 4, 8, 16};
  for (int t : tcounts) {
    char name[96];
    std::snprintf(name, sizeof name, "batcher_%d_threads_p16", t);
    expect(run(t, 40, p16, 300, 4096), name);
    std::snprintf(name, sizeof name, "batcher_%d_threads_tiny_maxfiles3", t);
    expect(run(t, 20, tiny, 50, 3), name);
  }
  std::printf("%s\n", failures ? "FAILED" : "ALL PASSED");
  return failures ? 1 : 0;
}
