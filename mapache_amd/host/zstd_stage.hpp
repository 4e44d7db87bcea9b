// zstd_stage.hpp — the compression half of SecureStorage::encode / decode on
// host threads ("AES-GCM-SIV is GPU-friendly; zstd is
// hard"): mapache compresses every blob with zstd before it encrypts it
// (/root/reference/src/repository/storage.rs:61-65, compress :74-84:
// ZstdEncoder at level DEFAULT_COMPRESSION_LEVEL = 3, WindowLog =
// log2(AVG_CHUNK_SIZE) = 20 (:31), ChecksumFlag false; decompress :87-94 with
// window_log_max 20).  libmcdc seals on the GPU; this stage runs the system
// libzstd (libzstd.so.1, loaded at run time: the image ships no zstd headers)
// on a pool of host threads, one compression context per thread.
//
// The compressed bytes depend on the libzstd version (the crate links zstd
// 1.5.7, Cargo.lock zstd-sys 2.0.15+zstd.1.5.7), so only the decoded bytes are
// comparable with the reference; frames are standard zstd frames any decoder
// reads, with the reference's window and checksum settings.
#pragma once
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mcdc {
namespace host {

struct ZInBuf {
  const void *src;
  size_t size, pos;
};
struct ZOutBuf {
  void *dst;
  size_t size, pos;
};

// The libzstd entry points used (stable API since zstd 1.4.0).
struct ZstdApi {
  void *(*createCCtx)() = nullptr;
  size_t (*freeCCtx)(void *) = nullptr;
  size_t (*cctxSetParameter)(void *, int, int) = nullptr;
  size_t (*compressStream2)(void *, ZOutBuf *, ZInBuf *, int) = nullptr;
  size_t (*compressBound)(size_t) = nullptr;
  unsigned (*isError)(size_t) = nullptr;
  const char *(*getErrorName)(size_t) = nullptr;
  void *(*createDCtx)() = nullptr;
  size_t (*freeDCtx)(void *) = nullptr;
  size_t (*dctxSetParameter)(void *, int, int) = nullptr;
  size_t (*decompressStream)(void *, void *, void *) = nullptr;
  size_t (*dStreamOutSize)() = nullptr;
  bool ok = false;
  std::string why;
};

// ZSTD_cParameter / ZSTD_dParameter values (zstd.h, stable)
constexpr int kZstdCLevel = 100, kZstdCWindowLog = 101, kZstdCContentSize = 200, kZstdCChecksum = 201,
              kZstdDWindowLogMax = 100;
constexpr int kZstdLevel = 3, kZstdWindowLog = 20;
constexpr int kZstdEContinue = 0, kZstdEEnd = 2;  // ZSTD_EndDirective  // storage.rs:31,76-79 (zstd crate default level 3)

inline const ZstdApi &zstd_api() {
  static ZstdApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      api.why = "libzstd.so.1 not found";
      return;
    }
    auto sym = [&](const char *name) { return dlsym(h, name); };
    api.createCCtx = (void *(*)())sym("ZSTD_createCCtx");
    api.freeCCtx = (size_t(*)(void *))sym("ZSTD_freeCCtx");
    api.cctxSetParameter = (size_t(*)(void *, int, int))sym("ZSTD_CCtx_setParameter");
    api.compressStream2 = (size_t(*)(void *, ZOutBuf *, ZInBuf *, int))sym("ZSTD_compressStream2");
    api.compressBound = (size_t(*)(size_t))sym("ZSTD_compressBound");
    api.isError = (unsigned (*)(size_t))sym("ZSTD_isError");
    api.getErrorName = (const char *(*)(size_t))sym("ZSTD_getErrorName");
    api.createDCtx = (void *(*)())sym("ZSTD_createDCtx");
    api.freeDCtx = (size_t(*)(void *))sym("ZSTD_freeDCtx");
    api.dctxSetParameter = (size_t(*)(void *, int, int))sym("ZSTD_DCtx_setParameter");
    api.decompressStream = (size_t(*)(void *, void *, void *))sym("ZSTD_decompressStream");
    api.dStreamOutSize = (size_t(*)())sym("ZSTD_DStreamOutSize");
    api.ok = api.createCCtx && api.freeCCtx && api.cctxSetParameter && api.compressStream2 && api.compressBound &&
             api.isError && api.getErrorName && api.createDCtx && api.freeDCtx && api.dctxSetParameter &&
             api.decompressStream && api.dStreamOutSize;
    if (!api.ok) api.why = "libzstd.so.1 lacks the zstd 1.4 advanced API";
  });
  return api;
}

// Run fn(i, worker) for i in [0, n) on up to `threads` host threads (worker
// = thread index, for per-thread state); items are handed out one at a time.
template <class F>
void parallel_items(size_t n, int threads, F fn) {
  threads = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, n));
  std::atomic<size_t> next{0};
  auto run = [&](int w) {
    for (size_t i; (i = next.fetch_add(1)) < n;) fn(i, w);
  };
  std::vector<std::thread> pool;
  for (int w = 1; w < threads; ++w) pool.emplace_back(run, w);
  run(0);
  for (auto &t : pool) t.join();
}

// Compress blob i = in[off[i], + len[i]) for every i on up to `threads` host
// threads, one compression context per thread, exactly as the crate's
// ZstdEncoder writes a blob (storage.rs:74-84): level 3, window log 20, no
// checksum; write_all (ZSTD_e_continue), then finish (ZSTD_e_end until
// flushed), the size never pledged -- so the frames carry no content size and
// keep the window descriptor.  dst(i) -> (pointer, capacity >= its
// compressBound + 64) says where blob i goes, done(i, bytes) receives its size
// (not called for a blob that failed).  Returns "" or an error.  The one
// place the host encodes blobs: both entry points below are thin wrappers.
template <class Dst, class Done>
inline std::string zstd_compress_each(const uint8_t *in, const uint64_t *off, const uint64_t *len, size_t n,
                                      int threads, Dst dst, Done done) {
  const ZstdApi &z = zstd_api();
  if (!z.ok) return z.why;
  std::vector<void *> cctx((size_t)std::max(1, threads), nullptr);
  std::mutex emu;
  std::string err;
  parallel_items(n, threads, [&](size_t i, int w) {
    if (!cctx[w]) {
      cctx[w] = z.createCCtx();
      const bool ok = cctx[w] && !z.isError(z.cctxSetParameter(cctx[w], kZstdCLevel, kZstdLevel)) &&
                      !z.isError(z.cctxSetParameter(cctx[w], kZstdCWindowLog, kZstdWindowLog)) &&
                      !z.isError(z.cctxSetParameter(cctx[w], kZstdCChecksum, 0)) &&
                      !z.isError(z.cctxSetParameter(cctx[w], kZstdCContentSize, 0));
      if (!ok) {  // never compress with other settings than the reference's
        std::lock_guard<std::mutex> lk(emu);
        err = "zstd rejected level 3 / window log 20 / no checksum / no content size";
        if (cctx[w]) z.freeCCtx(cctx[w]);
        cctx[w] = nullptr;
        return;
      }
    }
    const std::pair<uint8_t *, size_t> d = dst(i, z.compressBound(len[i]) + 64);
    ZInBuf ib{in + off[i], (size_t)len[i], 0};
    ZOutBuf ob{d.first, d.second, 0};
    size_t r = z.compressStream2(cctx[w], &ob, &ib, kZstdEContinue);
    if (!z.isError(r)) {
      do {
        r = z.compressStream2(cctx[w], &ob, &ib, kZstdEEnd);
      } while (!z.isError(r) && r != 0 && ob.pos < ob.size);
    }
    if (z.isError(r) || r != 0) {  // (the context is mid-frame: drop it)
      std::lock_guard<std::mutex> lk(emu);
      err = std::string("zstd compression failed: ") + (z.isError(r) ? z.getErrorName(r) : "output bound");
      z.freeCCtx(cctx[w]);
      cctx[w] = nullptr;
      return;
    }
    done(i, ob.pos);
  });
  for (void *c : cctx)
    if (c) z.freeCCtx(c);
  return err;
}

// compress blob i into out_base[out_off[i], + its compressBound + 64), its
// size to out_len[i] (0 if it failed): one output region per blob, no
// per-blob allocation
inline std::string zstd_compress_into(const uint8_t *in, const uint64_t *off, const uint64_t *len, size_t n,
                                      int threads, uint8_t *out_base, const uint64_t *out_off, uint64_t *out_len) {
  for (size_t i = 0; i < n; ++i) out_len[i] = 0;
  return zstd_compress_each(
      in, off, len, n, threads, [&](size_t i, size_t cap) { return std::make_pair(out_base + out_off[i], cap); },
      [&](size_t i, size_t bytes) { out_len[i] = bytes; });
}

// compress blob i into out[i] (empty if it failed)
inline std::string zstd_compress_all(const uint8_t *in, const uint64_t *off, const uint64_t *len, size_t n,
                                     int threads, std::vector<std::vector<uint8_t>> &out) {
  out.assign(n, {});
  std::vector<uint8_t> ok(n, 0);
  std::string err = zstd_compress_each(
      in, off, len, n, threads,
      [&](size_t i, size_t cap) {
        out[i].resize(cap);
        return std::make_pair(out[i].data(), cap);
      },
      [&](size_t i, size_t bytes) {
        out[i].resize(bytes);
        ok[i] = 1;
      });
  for (size_t i = 0; i < n; ++i)
    if (!ok[i]) out[i].clear();
  return err;
}

// decompress frame i = in[off[i], + len[i]) into out[i] (window_log_max 20,
// as storage.rs:87-94); ok[i] = 0 or -2 (not a valid frame within the window)
inline std::string zstd_decompress_all(const uint8_t *in, const uint64_t *off, const uint64_t *len,
                                       const int32_t *skip, size_t n, int threads,
                                       std::vector<std::vector<uint8_t>> &out, std::vector<int32_t> &ok) {
  const ZstdApi &z = zstd_api();
  if (!z.ok) return z.why;
  out.assign(n, {});
  ok.assign(n, 0);
  std::vector<void *> dctx((size_t)std::max(1, threads), nullptr);
  parallel_items(n, threads, [&](size_t i, int w) {
    if ((skip && skip[i]) || len[i] == 0) return;  // (no frame: no bytes, as read_to_end of an empty reader)
    if (!dctx[w]) {
      dctx[w] = z.createDCtx();
      if (!dctx[w] || z.isError(z.dctxSetParameter(dctx[w], kZstdDWindowLogMax, kZstdWindowLog))) {
        if (dctx[w]) z.freeDCtx(dctx[w]);
        dctx[w] = nullptr;
        ok[i] = -2;
        return;
      }
    }
    std::vector<uint8_t> &o = out[i];
    const size_t step = z.dStreamOutSize();
    ZInBuf ib{in + off[i], (size_t)len[i], 0};
    for (;;) {
      const size_t at = o.size();
      o.resize(at + step);
      ZOutBuf ob{o.data() + at, step, 0};
      const size_t r = z.decompressStream(dctx[w], &ob, &ib);
      o.resize(at + ob.pos);
      if (z.isError(r)) {
        ok[i] = -2;
        o.clear();
        // a context left mid-frame is reset by recreating it
        z.freeDCtx(dctx[w]);
        dctx[w] = nullptr;
        return;
      }
      if (r == 0 && ib.pos == ib.size) return;   // frame complete, input consumed
      if (ib.pos == ib.size && ob.pos < step) {  // input ended inside a frame
        ok[i] = -2;
        o.clear();
        z.freeDCtx(dctx[w]);
        dctx[w] = nullptr;
        return;
      }
    }
  });
  for (void *d : dctx)
    if (d) z.freeDCtx(d);
  return "";
}

}  // namespace host
}  // namespace mcdc
