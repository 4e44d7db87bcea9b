// fastcdc_v2020.hpp — C++ host mirror of the chunker interface mapache uses,
// over the C ABI of libmcdc.so (include/mcdc.h).
//
// The reference (Rust) calls the crate `fastcdc` 3.2.1, module `v2020`, at
// /root/reference/src/archiver/processor.rs:173-202:
//     StreamCDC::with_level(reader, MIN, AVG, MAX, Normalization::Level1)
//     for result in chunker { let chunk = result?; ... chunk.data ... }
// This header keeps those names and meanings (namespace
// mapache_amd::fastcdc::v2020): Normalization, Chunk, ChunkData, Error,
// FastCDC (slice), StreamCDC<Reader>, with_level/new constructors, and an
// iterator whose items are Result<ChunkData, Error>; end of stream ends the
// iteration (the crate's Error::Empty).  Where the crate asserts (invalid
// sizes) the constructors throw std::invalid_argument.  Every boundary is
// computed on the GPU by libmcdc; nothing here chunks.
#pragma once

#include <mcdc.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

namespace mapache_amd::fastcdc::v2020 {

inline constexpr uint32_t MINIMUM_MIN = 64;
inline constexpr uint32_t MINIMUM_MAX = 1048576;
inline constexpr uint32_t AVERAGE_MIN = 256;
inline constexpr uint32_t AVERAGE_MAX = 4194304;
inline constexpr uint32_t MAXIMUM_MIN = 1024;
inline constexpr uint32_t MAXIMUM_MAX = 16777216;

enum class Normalization : uint32_t { Level0 = 0, Level1 = 1, Level2 = 2, Level3 = 3 };

struct Chunk {  // fastcdc::v2020::Chunk
  uint64_t hash;
  size_t offset;
  size_t length;
};

struct ChunkData {  // fastcdc::v2020::ChunkData
  uint64_t hash;
  uint64_t offset;
  size_t length;
  std::vector<uint8_t> data;
};

class Error : public std::runtime_error {  // fastcdc::v2020::Error
 public:
  enum class Kind { Empty, IoError, Other };
  Error(Kind k, const std::string &msg) : std::runtime_error(msg), kind_(k) {}
  Kind kind() const { return kind_; }

 private:
  Kind kind_;
};

template <class T>
using Result = std::variant<T, Error>;

// Thrown for failures of the GPU library itself (no CPU fallback exists).
class DeviceError : public std::runtime_error {
 public:
  DeviceError(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

namespace detail {
inline void check(int rc) {
  if (rc != MCDC_OK) throw DeviceError(rc, mcdc_last_error());
}
inline mcdc_params make_params(uint32_t min_size, uint32_t avg_size, uint32_t max_size,
                               Normalization level) {
  // the crate's assert!s, in its order (FastCDC/StreamCDC::with_level)
  if (!(min_size >= MINIMUM_MIN)) throw std::invalid_argument("assertion failed: min_size >= MINIMUM_MIN");
  if (!(min_size <= MINIMUM_MAX)) throw std::invalid_argument("assertion failed: min_size <= MINIMUM_MAX");
  if (!(avg_size >= AVERAGE_MIN)) throw std::invalid_argument("assertion failed: avg_size >= AVERAGE_MIN");
  if (!(avg_size <= AVERAGE_MAX)) throw std::invalid_argument("assertion failed: avg_size <= AVERAGE_MAX");
  if (!(max_size >= MAXIMUM_MIN)) throw std::invalid_argument("assertion failed: max_size >= MAXIMUM_MIN");
  if (!(max_size <= MAXIMUM_MAX)) throw std::invalid_argument("assertion failed: max_size <= MAXIMUM_MAX");
  mcdc_params p{min_size, avg_size, max_size, static_cast<uint32_t>(level)};
  check(mcdc_params_check(&p, nullptr, nullptr));
  return p;
}
}  // namespace detail

// RAII mcdc_ctx: one device, one stream, one workspace.  Not thread-safe;
// give each thread its own (mapache's rayon workers would each own one).
class Context {
 public:
  explicit Context(int device = 0, size_t max_bytes = size_t(1) << 30) : max_bytes_(max_bytes) {
    mcdc_ctx *c = nullptr;
    detail::check(mcdc_ctx_create(device, max_bytes, &c));
    ctx_.reset(c);
  }
  mcdc_ctx *get() const { return ctx_.get(); }
  size_t max_bytes() const { return max_bytes_; }
  mcdc_timing timing() const {
    mcdc_timing t{};
    detail::check(mcdc_ctx_timing(ctx_.get(), &t));
    return t;
  }
  std::vector<mcdc_chunk> chunk_host(const mcdc_params &p, const uint8_t *data, size_t n) {
    std::vector<mcdc_chunk> out(n / (p.min_size - 1) + 2);
    size_t k = 0;
    detail::check(mcdc_chunk_host(ctx_.get(), &p, data, n, out.data(), out.size(), &k));
    out.resize(k);
    return out;
  }

 private:
  struct Del {
    void operator()(mcdc_ctx *c) const { mcdc_ctx_destroy(c); }
  };
  std::unique_ptr<mcdc_ctx, Del> ctx_;
  size_t max_bytes_;
};

// Per-thread default context, grown on demand.
inline Context &default_context(size_t need) {
  thread_local std::unique_ptr<Context> ctx;
  if (!ctx || ctx->max_bytes() < need) {
    ctx.reset();
    ctx = std::make_unique<Context>(0, std::max<size_t>(need, size_t(1) << 30));
  }
  return *ctx;
}

// fastcdc::v2020::FastCDC — chunks of an in-memory slice.
class FastCDC {
 public:
  FastCDC(const uint8_t *source, size_t n, uint32_t min_size, uint32_t avg_size, uint32_t max_size,
          Normalization level = Normalization::Level1, Context *ctx = nullptr)
      : src_(source), n_(n), params_(detail::make_params(min_size, avg_size, max_size, level)), ctx_(ctx) {}
  static FastCDC new_(const uint8_t *source, size_t n, uint32_t min_size, uint32_t avg_size,
                      uint32_t max_size) {
    return FastCDC(source, n, min_size, avg_size, max_size, Normalization::Level1);
  }
  static FastCDC with_level(const uint8_t *source, size_t n, uint32_t min_size, uint32_t avg_size,
                            uint32_t max_size, Normalization level) {
    return FastCDC(source, n, min_size, avg_size, max_size, level);
  }

  std::optional<Chunk> next() {
    run();
    if (i_ >= chunks_.size()) return std::nullopt;
    const mcdc_chunk &c = chunks_[i_++];
    return Chunk{c.hash, static_cast<size_t>(c.offset), static_cast<size_t>(c.length)};
  }
  std::vector<Chunk> collect() {
    std::vector<Chunk> v;
    while (auto c = next()) v.push_back(*c);
    return v;
  }

 private:
  void run() {
    if (done_) return;
    Context &ctx = ctx_ ? *ctx_ : default_context(n_);
    chunks_ = ctx.chunk_host(params_, src_, n_);
    done_ = true;
  }
  const uint8_t *src_;
  size_t n_;
  mcdc_params params_;
  Context *ctx_;
  std::vector<mcdc_chunk> chunks_;
  size_t i_ = 0;
  bool done_ = false;
};

// fastcdc::v2020::StreamCDC over a Reader with `long read(uint8_t*, size_t)`
// returning bytes read, 0 at EOF, <0 on error (Error::IoError).  The source is
// consumed in windows >= 2*max; a chunk starting at c is final once c + max is
// inside the bytes read (cut_gear never looks further), so the result equals
// chunking the whole stream.
template <class Reader>
class StreamCDC {
 public:
  StreamCDC(Reader source, uint32_t min_size, uint32_t avg_size, uint32_t max_size,
            Normalization level = Normalization::Level1, size_t window = size_t(256) << 20,
            Context *ctx = nullptr)
      : src_(std::move(source)),
        params_(detail::make_params(min_size, avg_size, max_size, level)),
        window_(std::max<size_t>(window, 2 * size_t(max_size))),
        ctx_(ctx) {}
  static StreamCDC with_level(Reader source, uint32_t min_size, uint32_t avg_size, uint32_t max_size,
                              Normalization level) {
    return StreamCDC(std::move(source), min_size, avg_size, max_size, level);
  }
  static StreamCDC new_(Reader source, uint32_t min_size, uint32_t avg_size, uint32_t max_size) {
    return StreamCDC(std::move(source), min_size, avg_size, max_size, Normalization::Level1);
  }

  // None = iteration over (the crate maps Error::Empty to the end).
  std::optional<Result<ChunkData>> next() {
    while (q_ == pending_.size()) {
      if (eof_) return std::nullopt;
      if (auto err = fill()) return Result<ChunkData>(std::move(*err));
    }
    return Result<ChunkData>(std::move(pending_[q_++]));
  }

 private:
  std::optional<Error> fill() {
    pending_.clear();
    q_ = 0;
    buf_.resize(window_);
    size_t len = carry_;
    while (len < window_) {
      const long r = src_.read(buf_.data() + len, window_ - len);
      if (r < 0) return Error(Error::Kind::IoError, "read failed");
      if (r == 0) {
        eof_ = true;
        break;
      }
      len += static_cast<size_t>(r);
    }
    if (len == 0) return std::nullopt;
    Context &ctx = ctx_ ? *ctx_ : default_context(len);
    const std::vector<mcdc_chunk> ch = ctx.chunk_host(params_, buf_.data(), len);
    size_t keep_from = len;
    for (const mcdc_chunk &c : ch) {
      if (!eof_ && c.offset + params_.max_size > len) {
        keep_from = c.offset;
        break;
      }
      ChunkData d{c.hash, processed_ + c.offset, static_cast<size_t>(c.length), {}};
      d.data.assign(buf_.begin() + c.offset, buf_.begin() + c.offset + c.length);
      pending_.push_back(std::move(d));
    }
    processed_ += keep_from;
    carry_ = len - keep_from;
    std::memmove(buf_.data(), buf_.data() + keep_from, carry_);
    return std::nullopt;
  }

  Reader src_;
  mcdc_params params_;
  size_t window_;
  Context *ctx_;
  std::vector<uint8_t> buf_;
  size_t carry_ = 0;
  uint64_t processed_ = 0;
  bool eof_ = false;
  std::vector<ChunkData> pending_;
  size_t q_ = 0;
};

}  // namespace mapache_amd::fastcdc::v2020
