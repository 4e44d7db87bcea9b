// test_host_api.cpp — tests of the C++ host mirror (mapache_amd/host) written
// after the fastcdc crate's own v2020 unit tests (the crate's test file is not
// in the container; names and expectations are the crate's, recalled):
//   test_minimum_too_low/high, test_average_too_low/high,
//   test_maximum_too_low/high   -> constructor asserts
//   test_masks                  -> normalised masks for three param sets
//   test_all_zeros              -> 10 x 1024 chunks, hash 14169102344523991076
// plus MI355X-specific checks: GPU vs the oracle restatement on random data,
// StreamCDC (windowed) == FastCDC (slice), and mapache's own parameters.
//
// Usage: test_host_api cpu | gpu      (exit 0 = pass; prints one line per test)
#include "fastcdc_v2020.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

extern "C" {
#include "../../oracle/fastcdc_oracle.h"
}

using namespace mapache_amd::fastcdc::v2020;

static int failures = 0;

static void expect(bool ok, const std::string &name) {
  std::printf("%s %s\n", ok ? "PASS" : "FAIL", name.c_str());
  if (!ok) ++failures;
}

static bool throws_invalid(const std::function<void()> &f) {
  try {
    f();
  } catch (const std::invalid_argument &) {
    return true;
  }
  return false;
}

static void cpu_tests() {
  const uint8_t zeros[16] = {0};
  expect(throws_invalid([&] { FastCDC(zeros, 16, 63, 256, 1024); }), "test_minimum_too_low");
  expect(throws_invalid([&] { FastCDC(zeros, 16, 1048577, 2097152, 4194304); }), "test_minimum_too_high");
  expect(throws_invalid([&] { FastCDC(zeros, 16, 64, 255, 1024); }), "test_average_too_low");
  expect(throws_invalid([&] { FastCDC(zeros, 16, 64, 4194305, 16777216); }), "test_average_too_high");
  expect(throws_invalid([&] { FastCDC(zeros, 16, 64, 256, 1023); }), "test_maximum_too_low");
  expect(throws_invalid([&] { FastCDC(zeros, 16, 64, 256, 16777217); }), "test_maximum_too_high");
  // test_masks: mask_l = MASKS[bits-1], mask_s = MASKS[bits+1] at Level1
  struct {
    uint32_t mn, av, mx;
    uint64_t ml, ms;
  } cases[] = {{64, 256, 1024, 0x0000000018035100ull, 0x0000019000353000ull},              // MASKS[7], [9]
               {8192, 16384, 32768, 0x0000d90303530000ull, 0x0000d90f03530000ull},         // [13], [15]
               {1048576, 4194304, 16777216, 0x0000d91767537000ull, 0x0000d93777537000ull}};  // [21], [23]
  bool ok = true;
  for (auto &c : cases) {
    mcdc_params p{c.mn, c.av, c.mx, 1};
    uint64_t ms = 0, ml = 0;
    ok &= mcdc_params_check(&p, &ms, &ml) == MCDC_OK && ms == c.ms && ml == c.ml;
  }
  expect(ok, "test_masks");
  mcdc_params bad{64, 256, 1024, 4};
  expect(mcdc_params_check(&bad, nullptr, nullptr) == MCDC_E_PARAMS, "invalid_level_rejected");
  expect(mcdc_abi_version() == MCDC_ABI_VERSION, "abi_version");
}

static std::vector<uint8_t> rand_bytes(size_t n, uint64_t seed) {
  std::vector<uint8_t> v(n);
  oc_fill_random(v.data(), 0, n, seed);
  return v;
}

struct VecReader {  // Reader with short reads, like a BufReader over a file
  const std::vector<uint8_t> *v;
  size_t pos = 0, quantum;
  long read(uint8_t *dst, size_t n) {
    const size_t k = std::min({n, quantum, v->size() - pos});
    std::memcpy(dst, v->data() + pos, k);
    pos += k;
    return static_cast<long>(k);
  }
};

static void gpu_tests() {
  Context ctx(0, size_t(64) << 20);
  {  // test_all_zeros
    std::vector<uint8_t> z(10240, 0);
    auto v = FastCDC(z.data(), z.size(), 64, 256, 1024, Normalization::Level1, &ctx).collect();
    bool ok = v.size() == 10;
    for (auto &c : v) ok &= c.length == 1024 && c.hash == 14169102344523991076ull;
    expect(ok, "test_all_zeros");
  }
  struct P {
    uint32_t mn, av, mx, lv;
  } ps[] = {{16384, 65536, 262144, 1}, {524288, 1048576, 8388608, 1}, {64, 256, 1024, 1},
            {4096, 16384, 65536, 2}, {65, 300, 1111, 3}, {1024, 4096, 16384, 0}};
  const size_t sizes[] = {0, 1, 63, 1000, 70000, (size_t(3) << 20) + 7, size_t(12) << 20};
  bool ok = true;
  for (auto &p : ps) {
    for (size_t n : sizes) {
      auto d = rand_bytes(n, 77 + n);
      auto g = FastCDC(d.data(), n, p.mn, p.av, p.mx, Normalization(p.lv), &ctx).collect();
      oc_params op;
      oc_params_init(&op, p.mn, p.av, p.mx, p.lv);
      std::vector<oc_chunk> r(n / (p.mn - 1) + 2);
      size_t k = oc_chunk_slice(&op, d.data(), n, r.data(), r.size());
      bool same = k == g.size();
      for (size_t i = 0; same && i < k; ++i)
        same = g[i].offset == r[i].offset && g[i].length == r[i].length && g[i].hash == r[i].hash;
      if (!same) std::printf("  mismatch params %u/%u/%u L%u n=%zu gpu=%zu ref=%zu\n", p.mn, p.av, p.mx, p.lv, n, g.size(), k);
      ok &= same;
    }
  }
  expect(ok, "gpu_fastcdc_equals_oracle_random");
  {  // StreamCDC windows == FastCDC slice (mapache's parameters, tiny window)
    auto d = rand_bytes(size_t(40) << 20, 99);
    auto s = FastCDC(d.data(), d.size(), 524288, 1048576, 8388608, Normalization::Level1, &ctx).collect();
    StreamCDC<VecReader> st(VecReader{&d, 0, 65536 + 3}, 524288, 1048576, 8388608, Normalization::Level1,
                            size_t(17) << 20, &ctx);
    size_t i = 0;
    bool same = true;
    uint64_t total = 0;
    while (auto r = st.next()) {
      if (std::holds_alternative<Error>(*r)) { same = false; break; }
      const ChunkData &c = std::get<ChunkData>(*r);
      same &= i < s.size() && c.offset == s[i].offset && c.length == s[i].length && c.hash == s[i].hash &&
              std::memcmp(c.data.data(), d.data() + c.offset, c.length) == 0;
      total += c.length;
      ++i;
    }
    expect(same && i == s.size() && total == d.size(), "streamcdc_equals_fastcdc_mapache_params");
  }
}

// End-to-end from pageable memory, the Archiver adapter's real input (a file's
// bytes in a Vec<u8> read through BufReader, /root/reference/src/archiver/
// processor.rs:165-167): (a) one mcdc_chunk_host call over the whole pageable
// buffer; (b) the windowed StreamCDC mirror over an in-memory reader (256 MiB
// windows, every chunk's bytes copied into its ChunkData as the crate does).
// Prints one JSON line; both outputs are compared with each other.
static int bench_stream(double gib) {
  using clk = std::chrono::steady_clock;
  const size_t n = static_cast<size_t>(gib * double(1ull << 30));
  std::vector<uint8_t> data(n);
  oc_fill_random(data.data(), 0, n, 0x6d61706163686521ull ^ 0x77);
  const uint32_t mn = 16384, av = 65536, mx = 262144;
  Context ctx(0, (size_t(512) << 20) > n ? (size_t(512) << 20) : n);
  const mcdc_params p = detail::make_params(mn, av, mx, Normalization::Level1);
  double best_host = 1e30;
  std::vector<mcdc_chunk> ref;
  mcdc_timing t{};
  for (int r = 0; r < 3; ++r) {
    const auto t0 = clk::now();
    ref = ctx.chunk_host(p, data.data(), n);
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    if (s < best_host) {
      best_host = s;
      t = ctx.timing();
    }
  }
  struct MemReader {
    const uint8_t *p;
    size_t n, at = 0;
    long read(uint8_t *dst, size_t want) {
      const size_t k = std::min(want, n - at);
      std::memcpy(dst, p + at, k);
      at += k;
      return static_cast<long>(k);
    }
  };
  Context wctx(0, size_t(256) << 20);
  double best_stream = 1e30;
  bool same = true;
  for (int r = 0; r < 3; ++r) {
    StreamCDC<MemReader> sc(MemReader{data.data(), n}, mn, av, mx, Normalization::Level1, size_t(256) << 20, &wctx);
    size_t i = 0;
    bool ok = true;
    const auto t0 = clk::now();
    while (auto c = sc.next()) {
      const ChunkData &d = std::get<ChunkData>(*c);
      ok = ok && i < ref.size() && d.offset == ref[i].offset && d.length == ref[i].length && d.hash == ref[i].hash;
      ++i;
    }
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    same = same && ok && i == ref.size();
    best_stream = std::min(best_stream, s);
  }
  const double g = double(n) / double(1ull << 30);
  std::printf("{\"bytes\": %zu, \"chunks\": %zu, \"chunk_host_pageable_gib_s\": %.2f, \"chunk_host_ms\": %.3f, "
              "\"h2d_ms\": %.3f, \"device_ms\": %.3f, \"stream_cdc_gib_s\": %.2f, \"stream_cdc_ms\": %.3f, "
              "\"identical\": %s}\n",
              n, ref.size(), g / best_host, best_host * 1e3, t.h2d_ms, t.device_ms, g / best_stream,
              best_stream * 1e3, same ? "true" : "false");
  return same ? 0 : 1;
}

int main(int argc, char **argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  if (mode == "bench_stream") return bench_stream(argc > 2 ? std::atof(argv[2]) : 8.0);
  cpu_tests();
  if (mode == "gpu") gpu_tests();
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}
