// batcher.hpp — the cross-worker batching front-end (host C++, header-only).
//
// mapache chunks files on `read_concurrency` rayon workers at once
// (/root/reference/src/archiver/mod.rs:162-215, default 4:
// src/global/defaults.rs:22); each worker builds its own StreamCDC per file
// (src/archiver/processor.rs:173).  On the GPU one call over many files costs
// about as much as one call over one (a batch amortises the launch chain and
// the synchronisation), so this front-end lets every worker submit its file
// and blocks it until a batch containing the file has been chunked:
//
//   * group commit: a submitting thread that finds no batch in flight becomes
//     the leader, waits up to `gather_us` for more submissions (or until the
//     batch is full), takes the pending files and runs ONE batch call for all
//     of them; files submitted meanwhile form the next batch;
//   * per-file results (the file's chains restart at its first byte, exactly
//     one StreamCDC per file) are copied into each caller's own array, with
//     the crate-shaped status per caller (a too-small array gets
//     MCDC_E_CAPACITY and the required count, like mcdc_chunk_host).
//
// The batch function is a parameter: libmcdc.so's C ABI (mcdc_batcher_*)
// instantiates it with mcdc_chunk_batch on the batcher's own context; the CPU
// tests instantiate it with the oracle (tests/cpp/test_batcher.cpp, also run
// under ThreadSanitizer and ASan/UBSan).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mcdc.h"

namespace mcdc {
namespace host {

// (bufs, lens, nbufs, out, cap, counts, n_out, err_message) -> MCDC_* status
using BatchFn = std::function<int(const uint8_t *const *, const size_t *, size_t, mcdc_chunk *, size_t, size_t *,
                                  size_t *, std::string *)>;

struct BatcherStats {
  uint64_t batches = 0, files = 0, bytes = 0, max_batch_files = 0;
};

class Batcher {
 public:
  // out_bound(len): an upper bound of the chunks of a len-byte file
  Batcher(BatchFn fn, std::function<size_t(size_t)> out_bound, size_t max_batch_bytes, size_t max_batch_files,
          uint32_t gather_us)
      : fn_(std::move(fn)),
        bound_(std::move(out_bound)),
        max_bytes_(max_batch_bytes),
        max_files_(max_batch_files ? max_batch_files : 1),
        gather_us_(gather_us) {}

  Batcher(const Batcher &) = delete;
  Batcher &operator=(const Batcher &) = delete;

  ~Batcher() {
    // no caller may still be inside chunk(); wait for a leader finishing up
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return !leader_; });
  }

  // Chunk one file; blocks until its batch completed.  Thread-safe.
  int chunk(const uint8_t *data, size_t n, mcdc_chunk *out, size_t cap, size_t *n_out, std::string *err) {
    if (n && !data) {
      if (err) *err = "data is NULL";
      return MCDC_E_INVALID;
    }
    if (n > max_bytes_) {
      if (err) *err = "file larger than the batcher's max_batch_bytes";
      return MCDC_E_TOOBIG;
    }
    Req r;
    r.data = data;
    r.n = n;
    r.out = out;
    r.cap = cap;
    std::unique_lock<std::mutex> lk(mu_);
    pending_.push_back(&r);
    pending_bytes_ += n;
    new_cv_.notify_all();
    while (!r.done) {
      if (!leader_) {
        leader_ = true;
        lead(lk);  // returns with the lock held; r may or may not be in that batch
        leader_ = false;
        done_cv_.notify_all();
      } else {
        done_cv_.wait(lk);
      }
    }
    if (n_out) *n_out = r.n_out;
    if (r.rc && err) *err = r.err;
    return r.rc;
  }

  BatcherStats stats() const {
    std::lock_guard<std::mutex> lk(mu_);
    return stats_;
  }

 private:
  struct Req {
    const uint8_t *data = nullptr;
    size_t n = 0;
    mcdc_chunk *out = nullptr;
    size_t cap = 0, n_out = 0;
    int rc = MCDC_OK;
    std::string err;
    bool done = false;
  };

  // Called with the lock held; gathers, runs one batch unlocked, publishes.
  void lead(std::unique_lock<std::mutex> &lk) {
    // (system_clock: libstdc++ waits on it with pthread_cond_timedwait, which
    // ThreadSanitizer intercepts; a steady_clock wait uses
    // pthread_cond_clockwait, which GCC 11's runtime does not)
    const auto deadline = std::chrono::system_clock::now() + std::chrono::microseconds(gather_us_);
    while (pending_bytes_ < max_bytes_ && pending_.size() < max_files_ &&
           new_cv_.wait_until(lk, deadline) != std::cv_status::timeout) {
    }
    // take a prefix that fits (always at least one file)
    std::vector<Req *> batch;
    size_t bytes = 0;
    while (!pending_.empty() && batch.size() < max_files_ &&
           (batch.empty() || bytes + pending_.front()->n <= max_bytes_)) {
      batch.push_back(pending_.front());
      bytes += pending_.front()->n;
      pending_bytes_ -= pending_.front()->n;
      pending_.pop_front();
    }
    lk.unlock();
    run(batch);
    lk.lock();
    for (Req *q : batch) q->done = true;
    ++stats_.batches;
    stats_.files += batch.size();
    stats_.bytes += bytes;
    if (batch.size() > stats_.max_batch_files) stats_.max_batch_files = batch.size();
  }

  // Only the leader runs this, so the scratch vectors need no lock.
  void run(const std::vector<Req *> &batch) {
    const size_t k = batch.size();
    bufs_.resize(k);
    lens_.resize(k);
    counts_.assign(k, 0);
    size_t cap = 0;
    for (size_t i = 0; i < k; ++i) {
      bufs_[i] = batch[i]->data;
      lens_[i] = batch[i]->n;
      cap += bound_(batch[i]->n);
    }
    if (out_.size() < cap) out_.resize(cap);
    size_t total = 0;
    std::string msg;
    const int rc = fn_(bufs_.data(), lens_.data(), k, out_.data(), out_.size(), counts_.data(), &total, &msg);
    size_t at = 0;
    for (size_t i = 0; i < k; ++i) {
      Req *q = batch[i];
      if (rc != MCDC_OK) {
        q->rc = rc;
        q->err = msg;
        continue;
      }
      const size_t c = counts_[i];
      q->n_out = c;
      if (c > q->cap || (c && !q->out)) {
        q->rc = MCDC_E_CAPACITY;
        q->err = "output capacity " + std::to_string(q->cap) + " < " + std::to_string(c) + " chunks";
      } else if (c) {
        std::memcpy(q->out, out_.data() + at, c * sizeof(mcdc_chunk));
      }
      at += c;
    }
  }

  BatchFn fn_;
  std::function<size_t(size_t)> bound_;
  const size_t max_bytes_, max_files_;
  const uint32_t gather_us_;
  mutable std::mutex mu_;
  std::condition_variable new_cv_, done_cv_;
  std::deque<Req *> pending_;
  size_t pending_bytes_ = 0;
  bool leader_ = false;
  BatcherStats stats_;
  // leader-only scratch
  std::vector<const uint8_t *> bufs_;
  std::vector<size_t> lens_, counts_;
  std::vector<mcdc_chunk> out_;
};

}  // namespace host
}  // namespace mcdc
