// mcdc_api.hip — host side of libmcdc.so: the C ABI declared in include/mcdc.h.
//
// Replaces, for mapache's Archiver, the construction and iteration of
// fastcdc::v2020::StreamCDC at /root/reference/src/archiver/processor.rs:173-202
// (see INTEGRATION.md for the Rust binding).  Device work is delegated to the
// kernels in mcdc_kernels.hip; nothing here computes chunk boundaries.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/mcdc.h"
#include "../host/batcher.hpp"
#include "gear_table.h"
#include "mcdc_aead.h"
#include "mcdc_blake3.h"
#include "mcdc_index.h"
#include "mcdc_zframe.h"
#include "mcdc_zcomp.h"
#include "mcdc_internal.h"
#include "../host/zstd_stage.hpp"

using namespace mcdc;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(MCDC_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                  __FILE__, __LINE__);                                                    \
  } while (0)

constexpr uint32_t MINIMUM_MIN = 64, MINIMUM_MAX = 1048576;


constexpr uint32_t AVERAGE_MIN = 256, AVERAGE_MAX = 4194304;
constexpr uint32_t MAXIMUM_MIN = 1024, MAXIMUM_MAX = 16777216;

// crate: fn logarithm2(value: u32) -> u32 { f64::from(value).log2().round() as u32 }
uint32_t logarithm2(uint32_t v) { return (uint32_t)std::lround(std::log2((double)v)); }

int check_params(const mcdc_params *p, uint64_t *ms, uint64_t *ml) {
  if (!p) return fail(MCDC_E_INVALID, "params is NULL");
  if (p->min_size < MINIMUM_MIN || p->min_size > MINIMUM_MAX)
    return fail(MCDC_E_PARAMS, "min_size %u outside [%u, %u]", p->min_size, MINIMUM_MIN, MINIMUM_MAX);
  if (p->avg_size < AVERAGE_MIN || p->avg_size > AVERAGE_MAX)
    return fail(MCDC_E_PARAMS, "avg_size %u outside [%u, %u]", p->avg_size, AVERAGE_MIN, AVERAGE_MAX);
  if (p->max_size < MAXIMUM_MIN || p->max_size > MAXIMUM_MAX)
    return fail(MCDC_E_PARAMS, "max_size %u outside [%u, %u]", p->max_size, MAXIMUM_MIN, MAXIMUM_MAX);
  if (p->level > 3) return fail(MCDC_E_PARAMS, "level %u not a Normalization", p->level);
  const uint32_t bits = logarithm2(p->avg_size);
  if (ms) *ms = kMasks[bits + p->level];
  if (ml) *ml = kMasks[bits - p->level];
  return MCDC_OK;
}

uint32_t next_pow2(uint32_t v) {
  uint32_t r = 1;
  while (r < v) r <<= 1;
  return r;
}

DevParams make_dev_params(const mcdc_params *p, uint64_t ms, uint64_t ml) {
  DevParams d{};
  d.min = p->min_size;
  d.avg = p->avg_size;
  d.max = p->max_size;
  d.ms = ms;
  d.ml = ml;
  d.ms16 = ms << 16;
  d.ml16 = ml << 16;
  d.pf_hi = (uint32_t)((ms & ml) >> 16);
  // candidate slots per run: ~4x the expected S|L count, at least 8
  const double dens = std::ldexp(1.0, -__builtin_popcountll(ms)) + std::ldexp(1.0, -__builtin_popcountll(ml));
  const uint32_t want = (uint32_t)std::ceil(4.0 * kRun * dens) + 4;
  d.cap = std::min<uint32_t>(128, std::max<uint32_t>(8, next_pow2(want)));
  return d;
}

// The lane walk (one lane per chain, DESIGN.md §5 "Resolution, round 3") when
// a chain step's window spans at most 64 runs (max <= 256 KiB): its steps
// read run summaries 16 runs per batch, so larger windows favour the group
// walk.  Single-part calls only (the staged pipeline keeps the group walk).
bool use_lane_walk(const mcdc_params *p, const Knobs &kn) {
  if (kn.parts != 1 || kn.lane_walk == 0) return false;
  return kn.lane_walk == 2 || p->max_size <= 64u * kRun;
}

// Segment length: ~16 expected chunks per speculative chain on the group walk
// (Knobs::seg_chunks, an A/B-build knob), ~4 on the lane walk (more, shorter
// chains: one lane each), >= 2 * max so that a single chunk never skips a
// whole segment.
uint64_t segment_bytes(const mcdc_params *p, const Knobs &kn) {
  const uint64_t k = (uint64_t)(use_lane_walk(p, kn) ? kn.lane_seg_chunks : kn.seg_chunks);
  uint64_t z = std::max<uint64_t>(2ull * p->max_size, k * ((uint64_t)p->min_size + p->avg_size));
  return (z + kRun - 1) / kRun * kRun;
}

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

constexpr int kMaxParts = 4;


// Host memcpy into the pinned staging slabs, split over a few threads: one
// thread copies pageable memory at ~10-15 GB/s, below the PCIe DMA rate the
// staged copy feeds (57.6 GB/s measured).  Persistent workers, created on the
// first pageable call of a context.
class CopyPool {
 public:
  struct Piece {
    uint8_t *dst;
    const uint8_t *src;
    size_t len;
  };
  explicit CopyPool(int threads) : nthreads_(threads) {
    for (int t = 0; t < threads; ++t) workers_.emplace_back([this, t] { loop(t); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &w : workers_) w.join();
  }
  // copy every piece; the calling thread takes share 0, the workers the rest
  void copy(const std::vector<Piece> &pieces) {
    size_t total = 0;
    for (const Piece &p : pieces) total += p.len;
    if (total < (4u << 20)) {  // not worth a hand-off
      for (const Piece &p : pieces) std::memcpy(p.dst, p.src, p.len);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      pieces_ = &pieces;
      total_ = total;
      pending_ = nthreads_;
      ++gen_;
    }
    cv_.notify_all();
    run_share(pieces, total, 0, nthreads_ + 1);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  static void run_share(const std::vector<Piece> &pieces, size_t total, int share, int nshares) {
    // bytes [a, b) of the concatenated pieces, cache-line aligned shares
    const size_t per = ((total + nshares - 1) / nshares + 63) / 64 * 64;  // shares cover all of total
    const size_t a = std::min(total, per * share), b = std::min(total, a + per);
    size_t at = 0;
    for (const Piece &p : pieces) {
      const size_t lo = std::max(a, at), hi = std::min(b, at + p.len);
      if (lo < hi) std::memcpy(p.dst + (lo - at), p.src + (lo - at), hi - lo);
      at += p.len;
      if (at >= b) break;
    }
  }
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::vector<Piece> *pieces;
      size_t total;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        pieces = pieces_;
        total = total_;
      }
      run_share(*pieces, total, t + 1, nthreads_ + 1);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  const int nthreads_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::vector<Piece> *pieces_ = nullptr;
  size_t total_ = 0;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

struct mcdc_ctx {
  int device = 0;
  int num_cus = 256;
  size_t max_bytes = 0;
  hipStream_t stream = nullptr;   // scan (and input copies)
  hipStream_t stream2 = nullptr;  // chain resolution, overlapping the scan's later parts
  hipStream_t stream3 = nullptr;  // the GPU save path's seals and pack assembly, beside the compressor
  hipStream_t stream4 = nullptr;  // the GPU save path's pack copies to the host, beside the seals
  hipEvent_t ev_start = nullptr, ev_scan = nullptr, ev_end = nullptr, ev_h2d0 = nullptr,
             ev_h2d1 = nullptr;
  hipEvent_t ev_part[kMaxParts] = {};
  hipEvent_t ev_tab = nullptr;    // after the last async upload out of h_tab
  hipEvent_t ev_prep = nullptr;   // after a call's table uploads and workspace resets on stream2
  bool tab_inflight = false;
  Knobs knobs;                    // read once at creation (read_knobs)
  uint64_t *d_gear = nullptr, *d_gear16 = nullptr;
  // workspace
  DevBuf arena, run_cnt, run_sum, run_ent, run_bits, punt, segs, files, nodes, node_off, node_cnt, seg_exit, cont, cont_cnt, cont_rep,
      cont_ent, long_list,
      link_seg, link_idx, link_pos, file_flags, seg_true, entry_idx, seg_count, seg_off, out, err,
      scan_tmp, seg_incl, irr, tile_ctr, b3_chunks, b3_gcnt, b3_goff, b3_owner, b3_nodes, b3_ids, b3_tmp, b3_hist, enc_in, enc_out, zf_sz, zf_off, zf_tmp, zf_ext,
      ae_ext, ae_nonce, ae_olen, ae_tcnt, ae_ooff, ae_toff, ae_tmp, ae_rec, ae_keys, ae_owner, ae_tsum, ae_status,
      sv_in, sv_pack, sv_comp, sv_seal, sv_ext, zc_cnt, zc_cls, zc_first, zc_wcnt, zc_wfirst, zc_blocks, zc_stage, zc_piece, zc_poff, zc_misc, zc_tmp, zc_words,
      zc_extra, zc_blocks2, zc_stage2, zc_piece2, zc_poff2, zc_tmp2, zc_words2, zc_extra2,  // (the second batch set)
      sv_zch, sv_zpre, sv_zext,  // (the GPU save path's compressor input: all blobs, prefixes, frame extents)
      sv_ids,  // (the save path's blob IDs in HBM)
      rl_ent, run_list,  // (the list-mode scan: its range entries and run list)
      plan_in, plan_tmp;  // (the GPU plan's extents and block sums)
  // pinned host staging (two slabs; stage_busy: an async copy out of slab k
  // may still be in flight, ev_h2d0/1 mark its completion)
  void *h_stage = nullptr;
  size_t h_stage_cap = 0;
  bool stage_busy[2] = {false, false};
  hipEvent_t ev_copy0 = nullptr;  // before the first input copy of a host call
  std::unique_ptr<CopyPool> pool;
  std::vector<Seg> h_segs;
  std::vector<File> h_files;
  std::vector<uint64_t> h_node_off;
  void *h_tab = nullptr;  // pinned copy of the segment tables (async H2D)
  size_t h_tab_cap = 0;
  // Plan cache: the segment tables depend only on the file ranges and the
  // parameters (never on the bytes), so a call with the same layout as the
  // previous one reuses the uploaded tables.
  uint64_t plan_n = 0, plan_z = 0, plan_min = 0;  // (the plan's key: these and the files' extents, in h_files
                                                  // or, planned on the GPU, staged in h_tab)
  bool plan_gpu = false;
  uint64_t plan_nsegs = 0, plan_nodes = 0;
  bool plan_valid = false;
  std::vector<uint64_t> bx_fs, bx_fe;
  DevBuf bits_zero;          // run_bits words [bits_zero_at * 2, + cap bytes) zeroed after the last call
  uint64_t bits_zero_at = 0;
  double call_t0 = 0;  // host entry time of the running call (host_pre_ms)  // mcdc_chunk_batch_device's file ranges (reused: no page faults per call)
  uint64_t *h_res = nullptr;  // pinned call summary written by k_finish
  uint64_t *h_fcnt = nullptr;  // pinned chunks-per-file, written by k_file_counts
  uint64_t *d_fcnt = nullptr;  // its device alias
  size_t h_fcnt_cap = 0;       // entries
  void *h_save = nullptr;      // pinned staging of the save path's new blobs (host zstd mode, device input)
  size_t h_save_cap = 0;       // bytes
  void *h_zarena = nullptr;    // pinned: mcdc_encode_blobs' frames back to back (its H2D source)
  size_t h_zarena_cap = 0;
  std::unique_ptr<uint8_t[]> h_zbuf;  // mcdc_encode_blobs' per-frame bound regions (kept: no page faults per call)
  size_t h_zbuf_cap = 0;
  void *h_encb = nullptr;      // pinned: mcdc_save_files' encoded blobs (host zstd mode)
  size_t h_encb_cap = 0;
  void *h_meta = nullptr;      // pinned: the GPU save path's encoded pack headers (their H2D source)
  size_t h_meta_cap = 0;
  std::vector<hipEvent_t> ev_pool;  // timing-free events the compressor and the save path take per call (kept)
  std::mutex ev_pool_mu;
  void *h_list = nullptr;      // pinned: mcdc_save_files' blob list (the IDs' upload source)
  size_t h_list_cap = 0;
  void *h_rl = nullptr;        // pinned: the list-mode scan's range entries (their H2D source)
  size_t h_rl_cap = 0;
  int list_state = 0;          // run list of the plan's layout: 0 none, 1 built (run_list), 2 not worth it
  uint64_t list_n = 0, list_nal = 0, list_min = 0;  // its runs, the arena length and min_size it was built for
  uint64_t *d_res = nullptr;  // its device alias
  mcdc_timing timing{};
};

namespace {

double now_ms();
#ifdef MCDC_SAVE_TRACE  // (A/B builds only: host time of the save path's stages, to stderr)
#define SAVE_T(name) fprintf(stderr, "SAVE %-14s %8.3f ms\n", name, now_ms() - t_trace0)
#else
#define SAVE_T(name) ((void)0)
#endif
static double t_trace0 = 0;

// The bytes ensure() allocates for a request (headroom against regrowth):
// mcdc_zstd_compress_scratch reports the same.
size_t ensure_bytes(size_t bytes) {
  if (bytes == 0) bytes = 16;
  return (bytes + bytes / 8 + 255) / 256 * 256;
}

int ensure(mcdc_ctx *ctx, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return MCDC_OK;
  if (b.p) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream3));
    HIP_TRY(hipStreamSynchronize(ctx->stream4));
    HIP_TRY(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  const size_t alloc = ensure_bytes(bytes);
#ifdef MCDC_SAVE_TRACE
  fprintf(stderr, "ENSURE %p %zu -> %zu\n", (void *)&b, b.cap, alloc);
#endif
  if (hipMalloc(&b.p, alloc) != hipSuccess) {
    b.p = nullptr;
    (void)hipGetLastError();
    return fail(MCDC_E_NOMEM, "hipMalloc(%zu) failed", alloc);
  }
  b.cap = alloc;
  return MCDC_OK;
}

int ensure_stage(mcdc_ctx *ctx, size_t bytes) {
  if (ctx->h_stage_cap >= bytes) return MCDC_OK;
  if (ctx->h_stage) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream3));
    HIP_TRY(hipStreamSynchronize(ctx->stream4));
    HIP_TRY(hipHostFree(ctx->h_stage));
    ctx->h_stage = nullptr;
    ctx->h_stage_cap = 0;
  }
  SAVE_T("pinned alloc");
  if (hipHostMalloc(&ctx->h_stage, bytes, hipHostMallocDefault) != hipSuccess) {
    ctx->h_stage = nullptr;
    (void)hipGetLastError();
    return fail(MCDC_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
  }
  ctx->h_stage_cap = bytes;
  ctx->stage_busy[0] = ctx->stage_busy[1] = false;
  return MCDC_OK;
}

int ensure_tab(mcdc_ctx *ctx, size_t bytes) {
  if (ctx->h_tab_cap >= bytes) return MCDC_OK;
  if (ctx->h_tab) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream3));
    HIP_TRY(hipStreamSynchronize(ctx->stream4));
    HIP_TRY(hipHostFree(ctx->h_tab));
    ctx->h_tab = nullptr;
    ctx->h_tab_cap = 0;
  }
  const size_t alloc = (bytes + bytes / 4 + 4095) / 4096 * 4096;
  SAVE_T("pinned alloc");
  if (hipHostMalloc(&ctx->h_tab, alloc, hipHostMallocDefault) != hipSuccess) {
    ctx->h_tab = nullptr;
    (void)hipGetLastError();
    return fail(MCDC_E_NOMEM, "hipHostMalloc(%zu) failed", alloc);
  }
  ctx->h_tab_cap = alloc;
  return MCDC_OK;
}

int ensure_fcnt(mcdc_ctx *ctx, size_t n) {
  if (ctx->h_fcnt_cap >= n) return MCDC_OK;
  if (ctx->h_fcnt) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream3));
    HIP_TRY(hipStreamSynchronize(ctx->stream4));
    HIP_TRY(hipHostFree(ctx->h_fcnt));
    ctx->h_fcnt = nullptr;
    ctx->h_fcnt_cap = 0;
  }
  const size_t alloc = (n + n / 4 + 511) / 512 * 512;
  SAVE_T("pinned alloc");
  if (hipHostMalloc((void **)&ctx->h_fcnt, alloc * 8, hipHostMallocDefault) != hipSuccess) {
    ctx->h_fcnt = nullptr;
    (void)hipGetLastError();
    return fail(MCDC_E_NOMEM, "hipHostMalloc(%zu) failed", alloc * 8);
  }
  HIP_TRY(hipHostGetDevicePointer((void **)&ctx->d_fcnt, ctx->h_fcnt, 0));
  ctx->h_fcnt_cap = alloc;
  return MCDC_OK;
}

// A pinned host buffer of the context, grown (never shrunk) and kept.
int ensure_pinned(mcdc_ctx *ctx, void *&p, size_t &cap, size_t bytes) {
  if (cap >= bytes) return MCDC_OK;
  if (p) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream3));
    HIP_TRY(hipStreamSynchronize(ctx->stream4));
    HIP_TRY(hipHostFree(p));
    p = nullptr;
    cap = 0;
  }
  const size_t alloc = (bytes + bytes / 8 + 4095) / 4096 * 4096;
  SAVE_T("pinned alloc");
  if (hipHostMalloc(&p, alloc, hipHostMallocDefault) != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return fail(MCDC_E_NOMEM, "hipHostMalloc(%zu) failed", alloc);
  }
  cap = alloc;
  return MCDC_OK;
}
int ensure_hsave(mcdc_ctx *ctx, size_t bytes) { return ensure_pinned(ctx, ctx->h_save, ctx->h_save_cap, bytes); }

// Where k_emit can write the caller's output array directly: a device
// pointer on the context's device (the boundary list stays in HBM for a
// device-side consumer), or the device alias of pinned host memory
// (hipHostMalloc / registered: written straight over PCIe, no separate copy).
// nullptr for pageable host memory (staged through ctx->out + one D2H copy).
void *direct_out(const mcdc_ctx *ctx, void *out) {
  if (!out) return nullptr;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, out) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type == hipMemoryTypeDevice) return a.device == ctx->device ? out : nullptr;
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  return a.devicePointer;
}

bool is_device_ptr(const void *p) {
  if (!p) return false;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// x / d for one divisor d and many x < 2^53 (the plan's segment and node
// counts): a double-precision estimate corrected to the exact quotient.
struct FastDiv {
  uint64_t d;
  double inv;
  explicit FastDiv(uint64_t dv) : d(dv), inv(1.0 / (double)dv) {}
  uint64_t div(uint64_t x) const {
    if (x >= (1ull << 52)) return x / d;
    uint64_t q = (uint64_t)((double)x * inv);
    if (q * d > x) --q;
    else if ((q + 1) * d <= x) ++q;
    return q;
  }
};

// The list-mode scan's run list for a layout (run_pipeline): per file longer
// than min_size the full runs holding [start + min_size, end) -- every run a
// chunk window of the file reads (lane_next, group_next, forced_run and
// run_first_hit read runs at or after a chunk start + min_size of the file;
// the restart positions before it are re-hashed from bytes) -- merged while
// the files ascend (files that do not: no list), as entries of <= 64 runs, the
// list expanded by k_run_list on stream2.  Kept (list_state 1) when it skips
// at least 20 % of the runs (MCDC_RUN_LIST=2: always).
int build_run_list(mcdc_ctx *ctx, const mcdc_params *params, uint64_t n_al, const uint64_t *fstart,
                   const uint64_t *fend, size_t nfiles) {
  const Knobs &kn = ctx->knobs;
  const uint64_t nfull = n_al / kRun, mn = params->min_size;
  ctx->list_state = 2;
  uint32_t *e = nullptr;
  int rc = MCDC_OK;
  uint64_t tot = 0, k = 0;
  // two passes: the runs it would list (the decision), then the entries
  auto pass = [&](bool write) -> bool {
    uint64_t c0 = 0, c1 = 0;
    tot = k = 0;
    auto flush = [&]() {
      if (!write) {
        tot += c1 - c0;
        return;
      }
      for (uint64_t r = c0; r < c1; r += 64, ++k) {
        e[2 * k] = (uint32_t)r;
        e[2 * k + 1] = (uint32_t)tot;
        tot += std::min<uint64_t>(64, c1 - r);
      }
    };
    for (size_t i = 0; i < nfiles; ++i) {
      if (fend[i] - fstart[i] <= mn) continue;  // (one chunk, hash 0: nothing of it is hashed)
      const uint64_t r0 = (fstart[i] + mn) / kRun, r1 = std::min<uint64_t>((fend[i] + kRun - 1) / kRun, nfull);
      if (r0 >= r1) continue;
      if (r0 < c0) return false;  // (files not ascending: the flat scan)
      if (r0 <= c1 && c1 > c0) {
        c1 = std::max(c1, r1);
      } else {
        flush();
        c0 = r0;
        c1 = r1;
      }
    }
    flush();
    return true;
  };
  if (!pass(false) || tot >= (1ull << 32) || !(kn.run_list == 2 || (nfull >= 2048 && tot * 5 <= nfull * 4)))
    return MCDC_OK;
  if ((rc = ensure_pinned(ctx, ctx->h_rl, ctx->h_rl_cap, (nfiles + tot / 64 + 2) * 8))) return rc;
  e = (uint32_t *)ctx->h_rl;
  pass(true);
  if ((rc = ensure(ctx, ctx->rl_ent, k * 8)) || (rc = ensure(ctx, ctx->run_list, (tot + 64) * 4))) return rc;
  if (k) HIP_TRY(hipMemcpyAsync(ctx->rl_ent.p, ctx->h_rl, k * 8, hipMemcpyHostToDevice, ctx->stream2));
  launch_run_list((const uint32_t *)ctx->rl_ent.p, k, tot, (uint32_t *)ctx->run_list.p, nullptr, 0, ctx->stream2);
  HIP_TRY(hipGetLastError());
  ctx->list_state = 1;
  ctx->list_n = tot;
  ctx->list_nal = n_al;
  ctx->list_min = mn;
  return MCDC_OK;
}

// Core: files are [fstart[i], fend[i]) in an arena at `base` (16-aligned),
// arena length n_al (multiple of 16, all reads stay below it).
// after_scan (optional) runs once the scan is enqueued, before fstart /
// fend are read: a caller prepares (and validates) the file ranges there,
// overlapping the scan.
int run_pipeline(mcdc_ctx *ctx, const mcdc_params *params, const uint8_t *base, uint64_t n_al,
                 const uint64_t *fstart, const uint64_t *fend, size_t nfiles, mcdc_chunk *out,
                 size_t cap, size_t *counts, size_t *n_out, const std::function<int()> &after_scan = {}) {
  SAVE_T("pipe: start");
  uint64_t ms = 0, ml = 0;
  int rc = check_params(params, &ms, &ml);
  if (rc) return rc;
  const DevParams P = make_dev_params(params, ms, ml);
  const Knobs &kn = ctx->knobs;
  const uint64_t Z = segment_bytes(params, kn);
  // one attribute query classifies `out`: device memory of this device
  // (used in place), pinned host memory (k_emit writes it over PCIe by
  // default; with MCDC_PINNED_DIRECT=0 the list is emitted into HBM and one
  // DMA copies it), pageable host memory (one D2H copy)
  void *out_dev = nullptr;
  if (out) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, out) != hipSuccess) {
      (void)hipGetLastError();
    } else if (a.type == hipMemoryTypeDevice) {
      if (a.device != ctx->device) return fail(MCDC_E_INVALID, "out is a device pointer of another device");
      out_dev = out;
    } else if (a.type == hipMemoryTypeHost && a.devicePointer && kn.pinned_direct) {
      out_dev = a.devicePointer;
    }
  }

  // ---- scan workspace, and the scan itself for a single-part call ----
  // The scan reads none of the segment tables, so a single-part call enqueues
  // it before the host plans segments: planning (O(files)) overlaps the scan.
  const uint64_t nruns = (n_al + kRun - 1) / kRun;
  const uint64_t ntiles_full = (n_al / kRun) / 64;
  if ((rc = ensure(ctx, ctx->run_cnt, nruns))) return rc;
  // (+ one 16-run batch: the lane walk loads summaries a batch past its window)
  if ((rc = ensure(ctx, ctx->run_sum, (nruns + 32) * 4))) return rc;
  if ((rc = ensure(ctx, ctx->run_ent, nruns * P.cap * sizeof(uint32_t)))) return rc;
  // candidate-bitmap word pairs (+ read-ahead), then the scan's tile counter:
  // the bitmap words of the partial last tile (set with atomics) and the
  // counter are zeroed by one memset before the scan
  const uint64_t nbitw = nruns / 64 + 4;
  const size_t rb_cap = ctx->run_bits.cap;
  if ((rc = ensure(ctx, ctx->run_bits, nbitw * 16 + 64))) return rc;
  if (ctx->run_bits.cap != rb_cap) ctx->bits_zero = DevBuf{};  // (reallocated: the zeroed words are gone)
  SAVE_T("pipe: ensured");
  if ((rc = ensure(ctx, ctx->err, 32))) return rc;  // (zeroed by the first scan launch)
  Work W{};
  W.base = base;
  W.n_al = n_al;
  W.nruns = nruns;
  W.gear = ctx->d_gear;
  W.gear16 = ctx->d_gear16;
  W.run_cnt = (uint8_t *)ctx->run_cnt.p;
  W.run_sum = (uint32_t *)ctx->run_sum.p;
  W.run_ent = (uint32_t *)ctx->run_ent.p;
  W.run_bits = (uint64_t *)ctx->run_bits.p;
  W.err = (uint32_t *)ctx->err.p;
  W.tile_ctr = kn.dyn_tiles ? W.run_bits + 2 * nbitw : nullptr;
  W.first_static = kn.first_static ? 1u : 0u;
  hipStream_t st = ctx->stream;
  const bool early = kn.parts == 1;
  // the bitmap words the partial last tile's runs share (set with atomics)
  // through the tile counter
  const uint64_t bw0 = nruns / 64 >= 2 ? nruns / 64 - 2 : 0;
  const size_t zero_bytes = (nbitw - bw0) * 16 + 8;
  const double t_pre = now_ms();
  // The bitmap words of the partial last tile and the tile counter were zeroed
  // at the end of the previous call if it had this layout (off the next
  // call's path: two fill kernels of ~4 us each before the scan otherwise)
  const bool zeroed = ctx->bits_zero.p == ctx->run_bits.p && ctx->bits_zero_at == bw0 &&
                      ctx->bits_zero.cap == zero_bytes;
  ctx->bits_zero = DevBuf{};
  if (!zeroed) SAVE_T("pipe: cold");
  // List-mode scan: cut_gear hashes a chunk from min_size on (v2020), so a
  // file's first min_size bytes, less the 48-byte window warm-up, are read by
  // no chunk window -- every byte of a file up to min_size long: half the
  // bytes of the configs[3] stand-in.  The run list (build_run_list) depends
  // only on the layout, like the segment plan, and is kept with it: a call
  // whose layout repeats the previous call's builds it (on the host, while its
  // scan runs) and the calls after it scan through it, speculatively -- the
  // layout is compared with the plan's while the scan runs, and a call whose
  // layout turns out different re-scans flat (one wasted list scan; a
  // workload whose layouts change never builds a list, so never speculates).
  const bool spec_list = early && ctx->list_state == 1 && ctx->list_nal == n_al && ctx->list_min == params->min_size &&
                         (kn.scan_pieces ? kn.scan_pieces : scan_pieces(n_al / kRun, ctx->num_cus)) == 2;
  auto scan_flat = [&](bool cold) -> int {
    // (the scan's start and end events are recorded by its dispatch: an event
    // record between two kernels delays the second by ~5 us, kernel traces
    // of tools/small_probe.py)
#ifndef MCDC_COLD_EVENT  // (A/B: 1 = the start event recorded before the cold path's memset, as in round 5)
#define MCDC_COLD_EVENT 0
#endif
    if (cold) {
      if (MCDC_COLD_EVENT) HIP_TRY(hipEventRecord(ctx->ev_start, st));
      HIP_TRY(hipMemsetAsync(W.run_bits + 2 * bw0, 0, zero_bytes, st));
    }
    const int pc = kn.scan_pieces ? kn.scan_pieces : scan_pieces(n_al / kRun, ctx->num_cus);
    launch_scan(W, P, ctx->num_cus, st, 0, n_al > 0 ? (n_al / kRun) / (64 / pc) : 0, n_al > 0, pc, kn.scan_cold,
                !cold || !MCDC_COLD_EVENT ? ctx->ev_start : nullptr, ctx->ev_scan);
    HIP_TRY(hipGetLastError());
    return MCDC_OK;
  };
  if (spec_list) {  // (the bitmap words and the tile counter zeroed, then the listed runs and the partial last run)
    launch_run_list(nullptr, 0, 0, nullptr, W.run_bits, 2 * nbitw + 1, st, ctx->ev_start);
    W.run_list = (const uint32_t *)ctx->run_list.p;
    W.list_n = ctx->list_n;
    launch_scan(W, P, ctx->num_cus, st, 0, (ctx->list_n + 31) / 32, true, 2, false, nullptr, ctx->ev_scan);
    HIP_TRY(hipGetLastError());
    W.run_list = nullptr;  // (the resolution kernels take W by value: the scan's fields only)
    W.list_n = 0;
  } else if (early) {
    if ((rc = scan_flat(!zeroed))) return rc;
  }
  SAVE_T("pipe: scan queued");
  if (after_scan && (rc = after_scan())) return rc;
  SAVE_T("pipe: ranges");

  // ---- plan segments (host; reused when the layout repeats) ----
  // (no division per file: the output bound from the total -- it bounds the
  // per-file sum -- and the plan's quotients by FastDiv; the plan key is the
  // kept file table itself.  80 000 files: ~0.3 ms of 64-bit divisions before)
  uint64_t total_bytes = 0;
  for (size_t i = 0; i < nfiles; ++i) total_bytes += fend[i] - fstart[i];
  const uint64_t out_bound = total_bytes / (params->min_size - 1) + 2 * (uint64_t)nfiles + 1;
  bool same_plan = ctx->plan_valid && ctx->plan_n == nfiles && ctx->plan_z == Z && ctx->plan_min == params->min_size;
  if (same_plan && ctx->plan_gpu) {  // (the key: the extents staged for the GPU plan, starts then ends)
    const uint64_t *ks = (const uint64_t *)ctx->h_tab, *ke = ks + nfiles;
    for (size_t i = 0; same_plan && i < nfiles; ++i) same_plan = ks[i] == fstart[i] && ke[i] == fend[i];
  } else {
    for (size_t i = 0; same_plan && i < nfiles; ++i)
      same_plan = ctx->h_files[i].start == fstart[i] && ctx->h_files[i].end == fend[i];
  }
  SAVE_T("pipe: compared");
  if (!same_plan) {
    ctx->plan_valid = false;
    ctx->plan_n = nfiles;
    ctx->plan_z = Z;
    ctx->plan_min = params->min_size;
    const FastDiv dz(Z), dm(params->min_size - 1);
    const uint64_t ncap_full = dm.div(Z) + 2;  // (a whole segment's node capacity)
    // A single-part call of many files plans on the GPU (launch_plan, after
    // the extents' upload below): here only the totals the workspace needs,
    // and the extents staged (pinned) as the upload's source and the key.
    ctx->plan_gpu = early && nfiles >= 2048;
    ctx->h_files.clear();
    ctx->h_segs.clear();
    ctx->h_node_off.clear();
    if (ctx->plan_gpu) {
      if (ctx->tab_inflight) {  // (the previous upload out of the stage)
        HIP_TRY(hipEventSynchronize(ctx->ev_tab));
        ctx->tab_inflight = false;
      }
      if ((rc = ensure_tab(ctx, 16 * nfiles))) return rc;
      uint64_t *ks = (uint64_t *)ctx->h_tab, *ke = ks + nfiles;
      uint64_t ns = 0, kmax = 0;
      for (size_t i = 0; i < nfiles; ++i) {  // (one pass: staged and counted; a division only past one segment)
        const uint64_t a = fstart[i], e = fend[i], len = e - a;
        const uint64_t k = len == 0 ? 0 : len <= Z ? 1 : dz.div(len + Z - 1);
        ks[i] = a;
        ke[i] = e;
        ns += k;
        kmax = std::max(kmax, k);
      }
      ctx->plan_nsegs = ns;
      // (the node buffer's size: a bound of the per-segment capacities'
      // sum, floor(len / (min_size - 1)) + 2 each, which k_plan_write lays out)
      ctx->plan_nodes = total_bytes / (params->min_size - 1) + 2 * ns + 1;
      SAVE_T("pipe: staged extents");
      // (k_plan_write writes a file's segments on one lane: a batch holding a
      // file of thousands of segments is planned on the host)
      if (kmax > 1024) ctx->plan_gpu = false;
    }
    if (!ctx->plan_gpu) {
      ctx->h_files.resize(nfiles);
      ctx->h_segs.reserve(nfiles + total_bytes / Z + 1);
      ctx->h_node_off.reserve(nfiles + total_bytes / Z + 2);
      ctx->h_node_off.push_back(0);
      uint64_t noff = 0;
      for (size_t i = 0; i < nfiles; ++i) {
        const uint64_t fs0 = fstart[i], fe0 = fend[i], len = fe0 - fs0;
        const uint32_t nseg = (uint32_t)dz.div(len + Z - 1);
        ctx->h_files[i] = File{fs0, fe0, (uint32_t)ctx->h_segs.size(), nseg};
        for (uint32_t k = 0; k < nseg; ++k) {
          Seg S;
          S.start = fs0 + (uint64_t)k * Z;
          S.end = k + 1 < nseg ? S.start + Z : fe0;
          S.file = (uint32_t)i;
          S.flags = (k == 0 ? kSegFirst : 0) | (k + 1 == nseg ? kSegLast : 0);
          ctx->h_segs.push_back(S);
          noff += k + 1 < nseg ? ncap_full : dm.div(S.end - S.start) + 2;
          ctx->h_node_off.push_back(noff);
        }
      }
      ctx->plan_nsegs = ctx->h_segs.size();
      ctx->plan_nodes = noff;
    }
  }
  const uint32_t nsegs = (uint32_t)ctx->plan_nsegs;
  SAVE_T(same_plan ? "pipe: plan same" : "pipe: planned");
  // the run list follows the plan: a new layout drops it; a speculative list
  // scan of another layout's runs is replaced by the flat scan (same stream:
  // every kernel after it reads the flat scan's run data)
  if (!same_plan) ctx->list_state = 0;
  if (spec_list && !same_plan && (rc = scan_flat(true))) return rc;
  bool list_built = false;
  if (early && same_plan && ctx->list_state == 0 && kn.run_list && n_al >= kRun &&
      (kn.scan_pieces ? kn.scan_pieces : scan_pieces(n_al / kRun, ctx->num_cus)) == 2) {
    if ((rc = build_run_list(ctx, params, n_al, fstart, fend, nfiles))) return rc;
    list_built = ctx->list_state == 1;
  }

  SAVE_T("pipe: list checked");
  // ---- workspace ----
  const void *tabs_before[3] = {ctx->segs.p, ctx->files.p, ctx->node_off.p};
  if ((rc = ensure(ctx, ctx->segs, nsegs * sizeof(Seg)))) return rc;
  if ((rc = ensure(ctx, ctx->files, nfiles * sizeof(File)))) return rc;
  if ((rc = ensure(ctx, ctx->nodes, ctx->plan_nodes * sizeof(uint64_t)))) return rc;
  if ((rc = ensure(ctx, ctx->node_off, (nsegs + 1) * sizeof(uint64_t)))) return rc;
  if (tabs_before[0] != ctx->segs.p || tabs_before[1] != ctx->files.p || tabs_before[2] != ctx->node_off.p)
    ctx->plan_valid = false;  // reallocated: the uploaded tables are gone
  if ((rc = ensure(ctx, ctx->node_cnt, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->seg_exit, nsegs * 8))) return rc;
  if ((rc = ensure(ctx, ctx->cont, (size_t)nsegs * kContMax * 8))) return rc;
  if ((rc = ensure(ctx, ctx->cont_cnt, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->cont_rep, (size_t)nsegs * kContMax * 4))) return rc;
  if ((rc = ensure(ctx, ctx->cont_ent, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->long_list, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->link_seg, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->link_idx, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->link_pos, nsegs * 8))) return rc;
  if ((rc = ensure(ctx, ctx->file_flags, nfiles * 4))) return rc;
  if ((rc = ensure(ctx, ctx->seg_true, nsegs))) return rc;
  if ((rc = ensure(ctx, ctx->entry_idx, nsegs * 4))) return rc;
  if ((rc = ensure(ctx, ctx->seg_count, (nsegs + 1) * 8))) return rc;
  if ((rc = ensure(ctx, ctx->seg_off, (nsegs + 1) * 8))) return rc;
  if (!out_dev && (rc = ensure(ctx, ctx->out, out_bound * sizeof(DevChunk)))) return rc;
  const size_t tmpb = scan_tmp_bytes(nsegs);
  if ((rc = ensure(ctx, ctx->scan_tmp, tmpb))) return rc;

  W.segs = (const Seg *)ctx->segs.p;
  W.nsegs = nsegs;
  W.nfiles = (uint32_t)nfiles;
  W.files = (const File *)ctx->files.p;
  W.zseg = Z;
  W.nodes = (uint64_t *)ctx->nodes.p;
  W.node_off = (const uint64_t *)ctx->node_off.p;
  W.node_cnt = (uint32_t *)ctx->node_cnt.p;
  W.seg_exit = (uint64_t *)ctx->seg_exit.p;
  W.cont = (uint64_t *)ctx->cont.p;
  W.cont_cnt = (uint32_t *)ctx->cont_cnt.p;
  W.cont_rep = (uint32_t *)ctx->cont_rep.p;
  W.cont_ent = (uint32_t *)ctx->cont_ent.p;
  W.long_list = (uint32_t *)ctx->long_list.p;
  W.link_seg = (uint32_t *)ctx->link_seg.p;
  W.link_idx = (uint32_t *)ctx->link_idx.p;
  W.link_pos = (uint64_t *)ctx->link_pos.p;
  W.file_flags = (uint32_t *)ctx->file_flags.p;
  W.seg_true = (uint8_t *)ctx->seg_true.p;
  W.entry_idx = (uint32_t *)ctx->entry_idx.p;
  W.seg_count = (uint64_t *)ctx->seg_count.p;
  W.seg_off = (uint64_t *)ctx->seg_off.p;
  W.out = out_dev ? (DevChunk *)out_dev : (DevChunk *)ctx->out.p;
  W.out_cap = out_dev ? std::min<uint64_t>(out_bound, cap) : out_bound;
  W.err = (uint32_t *)ctx->err.p;
  W.long_n = W.err + 3;

  if ((rc = ensure(ctx, ctx->seg_incl, (size_t)nsegs * 8))) return rc;
  if ((rc = ensure(ctx, ctx->irr, (size_t)nsegs * 5 + 16))) return rc;
  W.irr_n = (uint32_t *)ctx->irr.p;
  W.irr_list = (uint32_t *)ctx->irr.p + 4;
  W.irr_flag = (uint8_t *)ctx->irr.p + 16 + (size_t)nsegs * 4;
  const bool lane = use_lane_walk(params, kn);
  if (lane) {
    if ((rc = ensure(ctx, ctx->punt, (size_t)nsegs * 8 + 16 + lb_tiles(nsegs) * 8))) return rc;
    W.punt_spec = (uint32_t *)ctx->punt.p;
    W.punt_link = (uint32_t *)ctx->punt.p + nsegs;
    // look-back status words after the lists (16-byte aligned: nsegs*8 + 16 bytes in)
    W.lb_status = (uint64_t *)((char *)ctx->punt.p + (size_t)nsegs * 8 + 16);
  }
  W.ncu = (uint32_t)(ctx->num_cus > 0 ? ctx->num_cus : 256);

  // ---- staged pipeline plan ----
  // parts: full tiles [tb[i], tb[i+1]); the last part also scans the partial tile
  const uint64_t tile_bytes = 64ull * kRun;
  // (part_tiles / min_rounds shrink the round unit and the size threshold so
  // that tests exercise the staged path on small inputs)
  const uint64_t waves =
      kn.part_tiles ? (uint64_t)kn.part_tiles : std::max<uint64_t>(1, scan_waves(ntiles_full, ctx->num_cus));
  int K = std::min(kn.parts, kMaxParts);
  const uint64_t tail_rounds = (uint64_t)kn.tail_rounds;
  const uint64_t min_rounds = (uint64_t)kn.min_rounds;
  uint64_t tb[kMaxParts + 1];
  {
    uint64_t rounds_needed = 0, r = tail_rounds;
    for (int k = 1; k < K; ++k, r *= 3) rounds_needed += r;
    if (nsegs == 0 || ntiles_full < (rounds_needed + min_rounds) * waves || ntiles_full <= rounds_needed * waves)
      K = 1;
    tb[0] = 0;
    tb[K] = ntiles_full;
    r = tail_rounds;
    for (int k = K - 1; k >= 1; --k, r *= 3) tb[k] = tb[k + 1] - r * waves;
  }
  // resolution batches: spec/link/emit of segments [hi[i-1], hi[i]) after part i
  uint32_t spec_hi[kMaxParts], link_hi[kMaxParts];
  {
    const uint64_t mx = params->max_size;
    auto ceil_run = [](uint64_t x) { return (x + kRun - 1) / kRun * kRun; };
    uint32_t sp = 0, lk = 0;
    for (int i = 0; i < K; ++i) {
      if (i == K - 1) {
        sp = lk = nsegs;
      } else {
        const uint64_t B = tb[i + 1] * tile_bytes;
        while (sp < nsegs) {  // k_spec reads candidates up to S.end + max
          const Seg &S = ctx->h_segs[sp];
          if (ceil_run(std::min<uint64_t>(S.end + mx, ctx->h_files[S.file].end)) > B) break;
          ++sp;
        }
        while (lk < sp) {  // k_link: <= kContMax steps past S.end, merging into segments < sp
          const Seg &S = ctx->h_segs[lk];
          if (!(S.flags & kSegLast)) {
            const File &F = ctx->h_files[S.file];
            const uint64_t x = std::min<uint64_t>(S.end + (kContMax + 1) * mx, F.end);
            const uint64_t j = F.first_seg + (std::min<uint64_t>(x, F.end - 1) - F.start) / Z;
            if (ceil_run(x) > B || j >= sp) break;
          }
          ++lk;
        }
      }
      spec_hi[i] = sp;
      link_hi[i] = lk;
    }
  }

  // ---- launches: scan parts on `stream`, resolution on `stream2` ----
  // The scan needs none of the segment tables, so it is enqueued first; the
  // table uploads and workspace resets run on stream2 beside it.
  hipStream_t st2 = ctx->stream2;
  if (!early) {
    HIP_TRY(hipEventRecord(ctx->ev_start, st));
    for (int i = 0; i < K; ++i) {
      if (i == 0) HIP_TRY(hipMemsetAsync(W.run_bits + 2 * bw0, 0, zero_bytes, st));
      else if (W.tile_ctr) HIP_TRY(hipMemsetAsync(W.tile_ctr, 0, 8, st));
      if (n_al > 0) launch_scan(W, P, ctx->num_cus, st, tb[i], tb[i + 1], i == K - 1, 1, false);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(ctx->ev_part[i], st));
    }
    HIP_TRY(hipEventRecord(ctx->ev_scan, st));
  }
  bool uploaded = false;
  if (!ctx->plan_valid && ctx->plan_gpu) {  // the extents (staged at planning) -> the plan kernels on stream2
    uploaded = true;
    if ((rc = ensure(ctx, ctx->plan_in, 16 * nfiles)) || (rc = ensure(ctx, ctx->plan_tmp, 16 * (nfiles / 256 + 1))))
      return rc;
    HIP_TRY(hipMemcpyAsync(ctx->plan_in.p, ctx->h_tab, 16 * nfiles, hipMemcpyHostToDevice, st2));
    HIP_TRY(hipEventRecord(ctx->ev_tab, st2));
    ctx->tab_inflight = true;
    launch_plan((const uint64_t *)ctx->plan_in.p, nfiles, Z, params->min_size - 1, (uint64_t *)ctx->plan_tmp.p,
                (File *)ctx->files.p, (Seg *)ctx->segs.p, (uint64_t *)ctx->node_off.p, st2);
    HIP_TRY(hipGetLastError());
    ctx->plan_valid = true;
    SAVE_T("pipe: plan queued");
  } else if (!ctx->plan_valid) {  // tables -> pinned stage -> one async copy each
    uploaded = true;
    const size_t b_segs = nsegs * sizeof(Seg), b_files = nfiles * sizeof(File),
                 b_noff = ctx->h_node_off.size() * 8;
    const size_t o_files = (b_segs + 255) / 256 * 256, o_noff = o_files + (b_files + 255) / 256 * 256;
    // (staging on the host overlaps the scan just enqueued; the previous
    // uploads out of the pinned stage are waited for first: a call that
    // failed after enqueuing them returned without synchronising)
    if (ctx->tab_inflight) {
      SAVE_T("pipe: wait tab");
      HIP_TRY(hipEventSynchronize(ctx->ev_tab));
      ctx->tab_inflight = false;
    }
    if ((rc = ensure_tab(ctx, o_noff + b_noff))) return rc;
    char *tbuf = (char *)ctx->h_tab;
    if (b_segs) std::memcpy(tbuf, ctx->h_segs.data(), b_segs);
    if (b_files) std::memcpy(tbuf + o_files, ctx->h_files.data(), b_files);
    std::memcpy(tbuf + o_noff, ctx->h_node_off.data(), b_noff);
    SAVE_T("pipe: staged");
    if (b_segs) HIP_TRY(hipMemcpyAsync(ctx->segs.p, tbuf, b_segs, hipMemcpyHostToDevice, st2));
    if (b_files) HIP_TRY(hipMemcpyAsync(ctx->files.p, tbuf + o_files, b_files, hipMemcpyHostToDevice, st2));
    HIP_TRY(hipMemcpyAsync(ctx->node_off.p, tbuf + o_noff, b_noff, hipMemcpyHostToDevice, st2));
    HIP_TRY(hipEventRecord(ctx->ev_tab, st2));
    ctx->tab_inflight = true;
    ctx->plan_valid = true;
  }
  const bool want_counts = counts && nfiles;
  if (want_counts && (rc = ensure_fcnt(ctx, nfiles))) return rc;
  const bool lane_all = lane && K == 1;
  // A single-part call resolves on the scan's own stream (either walk): its
  // kernels follow the scan at a same-queue kernel boundary instead of a
  // cross-queue event (~13 us measured), and wait for stream2 only for this
  // call's table uploads / plan; the staged pipeline resolves part i on
  // stream2 behind the scan's part-i event, overlapping the later parts.
  hipStream_t rs = K == 1 ? st : st2;
  if (lane_all && n_al == 0) HIP_TRY(hipMemsetAsync(ctx->err.p, 0, 32, st));  // (no scan launch to clear them)
  if (!lane_all) {  // (the lane walk's first kernels reset these: k_scan_q, k_spec_lane; the scan only clears err)
    if (nfiles) HIP_TRY(hipMemsetAsync(ctx->file_flags.p, 0, nfiles * 4, rs));
    HIP_TRY(hipMemsetAsync(ctx->err.p, 0, 32, rs));
    HIP_TRY(hipMemsetAsync((uint64_t *)ctx->seg_count.p + nsegs, 0, 8, rs));
    HIP_TRY(hipMemsetAsync(ctx->seg_off.p, 0, 8, rs));
  }
  if (K == 1 && uploaded) {
    HIP_TRY(hipEventRecord(ctx->ev_prep, st2));
    HIP_TRY(hipStreamWaitEvent(st, ctx->ev_prep, 0));
  }
  if (lane_all) {
    launch_resolve_lane(W, P, (uint64_t *)ctx->seg_incl.p, ctx->scan_tmp.p, tmpb, st,
                        want_counts ? ctx->d_fcnt : nullptr);
    HIP_TRY(hipGetLastError());
  }
  for (int i = 0; i < (lane_all ? 0 : K); ++i) {
    if (K > 1) HIP_TRY(hipStreamWaitEvent(st2, ctx->ev_part[i], 0));
    const uint32_t a_s = i ? spec_hi[i - 1] : 0, a_l = i ? link_hi[i - 1] : 0;
    launch_spec(W, P, kn, a_s, spec_hi[i], rs);
    // parts before the last: link_hi assumes <= kContMax continuation steps
    launch_link(W, P, kn, a_l, link_hi[i], i == K - 1 ? ~0ull : (uint64_t)kContMax, rs);
    launch_emit_incremental(W, P, a_l, link_hi[i], (uint64_t *)ctx->seg_incl.p, ctx->scan_tmp.p, tmpb, rs);
    HIP_TRY(hipGetLastError());
  }
  if (want_counts && !(lane_all && nsegs)) launch_file_counts(W, ctx->d_fcnt, rs);  // (else by the emit)
  // (a whole-call scan: its bitmap words zeroed for the next call by k_finish)
  const bool rezero = early && n_al > 0;
  launch_finish(W, ctx->d_res, rs, ctx->ev_end, rezero ? W.run_bits + 2 * bw0 : nullptr, (uint32_t)(zero_bytes / 8));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(rs));
  const double t_dev = now_ms();
  if (rezero && !((volatile uint64_t *)ctx->h_res)[3]) {
    ctx->bits_zero.p = ctx->run_bits.p;
    ctx->bits_zero.cap = zero_bytes;
    ctx->bits_zero_at = bw0;
  }
  if (((volatile uint64_t *)ctx->h_res)[3]) {
    // some continuation did not merge into the next segment: resolve the whole
    // call with the general path (serial fallback / serial walk), which
    // rewrites every count, offset and boundary of the incremental pass
    HIP_TRY(hipMemsetAsync(ctx->err.p, 0, 4, rs));  // incremental capacity bits are void
    launch_resolve_general(W, P, ctx->scan_tmp.p, tmpb, rs);
    HIP_TRY(hipGetLastError());
    if (want_counts) launch_file_counts(W, ctx->d_fcnt, rs);
    launch_finish(W, ctx->d_res, rs, ctx->ev_end);
    HIP_TRY(hipGetLastError());
  }

  SAVE_T("pipe: finish queued");
  // ---- results: one synchronisation in the common case ----
  const double t_d2h0 = now_ms();
  HIP_TRY(hipStreamSynchronize(rs));
  if (list_built && rs != st2) HIP_TRY(hipStreamSynchronize(st2));  // (the run list's build, long done)
  SAVE_T("pipe: synced");
  const uint64_t total = ((volatile uint64_t *)ctx->h_res)[0];
  const uint32_t err = (uint32_t)((volatile uint64_t *)ctx->h_res)[1];
  const uint64_t nfallback = ((volatile uint64_t *)ctx->h_res)[2];
  if (n_out) *n_out = (size_t)total;
  if (total > cap || (total && !out))
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %llu chunks", cap, (unsigned long long)total);
  if (err) return fail(MCDC_E_INTERNAL, "device consistency error 0x%x", err);
  bool copies = false;
  if (total && !out_dev) {
    HIP_TRY(hipMemcpyAsync(out, ctx->out.p, total * sizeof(mcdc_chunk), hipMemcpyDeviceToHost, rs));
    copies = true;
  }
  if (copies) HIP_TRY(hipStreamSynchronize(rs));
  const double t_d2h1 = now_ms();
  static_assert(sizeof(size_t) == sizeof(uint64_t), "counts are 64-bit");
  if (want_counts) std::memcpy(counts, ctx->h_fcnt, nfiles * sizeof(uint64_t));
  float scan_ms = 0, dev_ms = 0;
  // (the resolution stream waited for the scan's last part event, not for
  // ev_scan recorded after it on the scan's stream: it may still be pending)
  if (rs != st) HIP_TRY(hipEventSynchronize(ctx->ev_scan));
  HIP_TRY(hipEventElapsedTime(&scan_ms, ctx->ev_start, ctx->ev_scan));
  HIP_TRY(hipEventElapsedTime(&dev_ms, ctx->ev_start, ctx->ev_end));
  ctx->timing.scan_ms = scan_ms;
  ctx->timing.device_ms = dev_ms;
  ctx->timing.resolve_ms = dev_ms - scan_ms;
  ctx->timing.d2h_ms = t_d2h1 - t_d2h0;
  ctx->timing.bytes = total_bytes;
  ctx->timing.chunks = total;
  ctx->timing.scan_launches = n_al > 0 ? (uint64_t)K : 0;
  ctx->timing.fallback_files = nfallback;
  ctx->timing.lane_walk = lane_all ? 1 : 0;
  ctx->timing.handed_back = lane_all ? ((volatile uint64_t *)ctx->h_res)[4] : 0;
  ctx->timing.host_pre_ms = ctx->call_t0 > 0 ? t_pre - ctx->call_t0 : 0;
  ctx->call_t0 = 0;
  ctx->timing.host_post_ms = now_ms() - t_dev;
  return MCDC_OK;
}

int check_ctx(mcdc_ctx *ctx) {
  if (!ctx) return fail(MCDC_E_INVALID, "ctx is NULL");
  (void)hipGetLastError();  // a failure of an earlier call on this thread must not be reported by this one
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return fail(MCDC_E_DEVICE, "hipSetDevice: %s", hipGetErrorString(e));
  return MCDC_OK;
}

// ------------------------------------------------------------- sealing --
// Copy an argument array (host or device memory) into a context buffer.
int stage_arg(mcdc_ctx *ctx, DevBuf &b, const void *src, size_t bytes) {
  int rc = ensure(ctx, b, bytes);
  if (rc) return rc;
  if (!bytes) return MCDC_OK;
  HIP_TRY(hipMemcpyAsync(b.p, src, bytes, is_device_ptr(src) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                         ctx->stream));
  return MCDC_OK;
}

// Copy n entries of a device result array to the caller's array (host or device).
int give_back(mcdc_ctx *ctx, void *dst, const void *d_src, size_t bytes) {
  if (!dst || !bytes) return MCDC_OK;
  HIP_TRY(hipMemcpyAsync(dst, d_src, bytes, is_device_ptr(dst) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                         ctx->stream));
  return MCDC_OK;
}

// mcdc_seal_device (open = 0) / mcdc_open_device (open = 1); chunks != nullptr:
// the extents come from a boundary list instead (mcdc_seal_chunks_device).
int aead_run(mcdc_ctx *ctx, int open, const uint8_t *key, const void *d_in, size_t n_in, const mcdc_blob *blobs,
             size_t nblobs, const uint8_t *nonces, void *d_out, size_t out_cap, uint64_t *out_offsets,
             int32_t *status, const mcdc_chunk *chunks = nullptr, bool wait_done = true,
             const uint64_t *place = nullptr) {
  // (wait_done false, seal only: returns once the kernels are enqueued and
  // out_offsets is written; the caller orders later work on the context's
  // stream and synchronises it.  place, seal only: host array of nblobs + 1,
  // blob i's output at d_out + place[i] instead of back to back, place[n] the
  // end of the furthest one -- the GPU save path seals into the pack layout)
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!key || (!d_in && n_in) || (nblobs && !blobs && !chunks) || (!open && nblobs && !nonces))
    return fail(MCDC_E_INVALID, "NULL argument");
  if (d_in && !is_device_ptr(d_in)) return fail(MCDC_E_INVALID, "d_in is not a device pointer");
  if (d_out && !is_device_ptr(d_out)) return fail(MCDC_E_INVALID, "d_out is not a device pointer");
  if (nblobs >= (1ull << 31)) return fail(MCDC_E_TOOBIG, "too many blobs (%zu)", nblobs);
  const double t0 = now_ms();
  hipStream_t st = ctx->stream;
  ctx->timing = mcdc_timing{};
  if (nblobs == 0) {
    const uint64_t zero = 0;
    if (out_offsets) {
      HIP_TRY(hipMemcpyAsync(out_offsets, &zero, 8, is_device_ptr(out_offsets) ? hipMemcpyHostToDevice
                                                                               : hipMemcpyHostToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
    }
    ctx->timing.total_ms = now_ms() - t0;
    return MCDC_OK;
  }
  const size_t n = nblobs;
  const size_t tmpb = aead_scan_tmp_bytes(n);
  if (chunks) {  // a boundary list: to the device if needed, then (offset, length) pairs
    if ((rc = stage_arg(ctx, ctx->b3_chunks, chunks, n * sizeof(mcdc_chunk))) ||
        (rc = ensure(ctx, ctx->ae_ext, n * sizeof(mcdc_blob))))
      return rc;
    launch_aead_from_chunks(ctx->b3_chunks.p, n, (uint64_t *)ctx->ae_ext.p, ctx->stream);
  } else if ((rc = stage_arg(ctx, ctx->ae_ext, blobs, n * sizeof(mcdc_blob)))) {
    return rc;
  }
  if ((!open && (rc = stage_arg(ctx, ctx->ae_nonce, nonces, n * kAeadNonce))) ||
      (rc = ensure(ctx, ctx->ae_olen, (n + 1) * 8)) || (rc = ensure(ctx, ctx->ae_tcnt, (n + 1) * 8)) ||
      (rc = ensure(ctx, ctx->ae_ooff, (n + 1) * 8)) || (rc = ensure(ctx, ctx->ae_toff, (n + 1) * 8)) ||
      (rc = ensure(ctx, ctx->ae_tmp, tmpb)) || (rc = ensure(ctx, ctx->err, 32)))
    return rc;
  uint32_t *err = (uint32_t *)ctx->err.p + 2;  // (words 4-5: the tile counters)
  uint64_t *ooff = (uint64_t *)ctx->ae_ooff.p, *toff = (uint64_t *)ctx->ae_toff.p;
  HIP_TRY(hipMemsetAsync(err, 0, 4, st));
  HIP_TRY(hipEventRecord(ctx->ev_start, st));
  launch_aead_sizes(open, (const uint64_t *)ctx->ae_ext.p, n, n_in, (uint64_t *)ctx->ae_olen.p,
                    (uint64_t *)ctx->ae_tcnt.p, ooff, toff, err, ctx->ae_tmp.p, tmpb, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev_scan, st));
  uint32_t herr = 0;
  uint64_t total = 0, ntiles = 0;
  HIP_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&total, ooff + n, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&ntiles, toff + n, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (herr) return fail(MCDC_E_INVALID, "a blob extent lies outside the %zu-byte input", n_in);
  if (place && !open) {  // (the sizes' scan is kept for the tile offsets; the output offsets replaced)
    HIP_TRY(hipMemcpyAsync(ooff, place, (n + 1) * 8, hipMemcpyHostToDevice, st));
    total = place[n];
  } else if ((rc = give_back(ctx, out_offsets, ooff, (n + 1) * 8))) {
    return rc;
  }
  if (!wait_done && !open) HIP_TRY(hipStreamSynchronize(st));  // (the offsets before the seal is enqueued)
  if (total > out_cap || (total && !d_out)) {
    HIP_TRY(hipStreamSynchronize(st));
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %llu bytes", out_cap, (unsigned long long)total);
  }
  if (ntiles >= (1ull << 32)) return fail(MCDC_E_TOOBIG, "input too large (%llu tiles)", (unsigned long long)ntiles);
  if ((rc = ensure(ctx, ctx->ae_rec, n * sizeof(AeadRec))) || (rc = ensure(ctx, ctx->ae_keys, n * sizeof(AeadKeys))) ||
      (rc = ensure(ctx, ctx->ae_owner, ntiles * 4)) || (rc = ensure(ctx, ctx->ae_tsum, ntiles * 16)) ||
      (rc = ensure(ctx, ctx->ae_status, n * 4)))
    return rc;
  AeadMaster mk;
  aead_expand_key256(key, mk.rk);
  HIP_TRY(hipEventRecord(ctx->ev_h2d0, st));
  if (!open)
    launch_aead_seal(mk, (const uint8_t *)d_in, (const uint64_t *)ctx->ae_ext.p, (const uint32_t *)ctx->ae_nonce.p, n,
                     (uint8_t *)d_out, ooff, toff, ntiles, (AeadRec *)ctx->ae_rec.p, (AeadKeys *)ctx->ae_keys.p,
                     (uint32_t *)ctx->ae_owner.p, (uint4 *)ctx->ae_tsum.p, (uint32_t *)ctx->err.p + 4,
                     ctx->num_cus, st);
  else
    launch_aead_open(mk, (const uint8_t *)d_in, (const uint64_t *)ctx->ae_ext.p, n, (uint8_t *)d_out, ooff, toff,
                     ntiles, (AeadRec *)ctx->ae_rec.p, (AeadKeys *)ctx->ae_keys.p, (uint32_t *)ctx->ae_owner.p,
                     (uint4 *)ctx->ae_tsum.p, (int32_t *)ctx->ae_status.p, (uint32_t *)ctx->err.p + 4,
                     ctx->num_cus, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev_end, st));
  std::memset(mk.rk, 0, sizeof mk.rk);
  if (!wait_done && !open) {
    ctx->timing.total_ms = now_ms() - t0;
    return MCDC_OK;
  }
  std::vector<int32_t> hstat;
  if (open) {
    hstat.resize(n);
    HIP_TRY(hipMemcpyAsync(hstat.data(), ctx->ae_status.p, n * 4, hipMemcpyDeviceToHost, st));
    if ((rc = give_back(ctx, status, ctx->ae_status.p, n * 4))) return rc;
  }
  HIP_TRY(hipStreamSynchronize(st));
  float ms0 = 0, ms1 = 0;
  HIP_TRY(hipEventElapsedTime(&ms0, ctx->ev_start, ctx->ev_scan));
  HIP_TRY(hipEventElapsedTime(&ms1, ctx->ev_h2d0, ctx->ev_end));
  ctx->timing.aead_ms = ms1;
  ctx->timing.device_ms = ms0 + ms1;
  ctx->timing.bytes = open ? total : 0;
  ctx->timing.chunks = n;
  ctx->timing.total_ms = now_ms() - t0;
  if (!open) {
    ctx->timing.bytes = total - (uint64_t)n * kAeadOverhead;
    return MCDC_OK;
  }
  size_t bad = 0;
  for (int32_t v : hstat) bad += v != 0;
  if (bad) return fail(MCDC_E_AUTH, "%zu of %zu blobs failed authentication", bad, n);
  return MCDC_OK;
}

}  // namespace

// ================================================================= C ABI ==
extern "C" {

int mcdc_abi_version(void) { return MCDC_ABI_VERSION; }

const char *mcdc_last_error(void) { return g_last_error.c_str(); }

int mcdc_params_check(const mcdc_params *params, uint64_t *mask_s, uint64_t *mask_l) {
  return check_params(params, mask_s, mask_l);
}

int mcdc_ctx_create(int device, size_t max_bytes, mcdc_ctx **out) {
  if (!out) return fail(MCDC_E_INVALID, "out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    return fail(MCDC_E_DEVICE, "no HIP device available");
  }
  if (device < 0 || device >= ndev) return fail(MCDC_E_INVALID, "device %d out of range (%d)", device, ndev);
  mcdc_ctx *ctx = new (std::nothrow) mcdc_ctx();
  if (!ctx) return fail(MCDC_E_NOMEM, "host allocation failed");
  ctx->device = device;
  ctx->max_bytes = max_bytes;
  auto bail = [&](int rc) {
    mcdc_ctx_destroy(ctx);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(fail(MCDC_E_DEVICE, "hipSetDevice(%d)", device));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream3, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream4, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(MCDC_E_DEVICE, "hipStreamCreate failed"));
  hipEvent_t *evs[] = {&ctx->ev_start, &ctx->ev_scan, &ctx->ev_end, &ctx->ev_h2d0, &ctx->ev_h2d1};
  for (hipEvent_t *e : evs)
    if (hipEventCreate(e) != hipSuccess) return bail(fail(MCDC_E_DEVICE, "hipEventCreate failed"));
  for (hipEvent_t &e : ctx->ev_part)  // ordering only: no timestamps
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return bail(fail(MCDC_E_DEVICE, "hipEventCreate failed"));
  if (hipEventCreateWithFlags(&ctx->ev_tab, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_prep, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&ctx->ev_copy0) != hipSuccess)
    return bail(fail(MCDC_E_DEVICE, "hipEventCreate failed"));
  ctx->knobs = read_knobs();
  uint64_t g16[256];
  for (int i = 0; i < 256; ++i) g16[i] = kGear[i] << 16;
  if (hipMalloc(&ctx->d_gear, 2048) != hipSuccess || hipMalloc(&ctx->d_gear16, 2048) != hipSuccess)
    return bail(fail(MCDC_E_NOMEM, "hipMalloc(tables) failed"));
  if (hipMemcpy(ctx->d_gear, kGear, 2048, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(ctx->d_gear16, g16, 2048, hipMemcpyHostToDevice) != hipSuccess)
    return bail(fail(MCDC_E_DEVICE, "table upload failed"));
  // (words 0-4: the chunker's call summary; 8-11: the compressor's per-batch counts)
  if (hipHostMalloc((void **)&ctx->h_res, 128, hipHostMallocDefault) != hipSuccess ||
      hipHostGetDevicePointer((void **)&ctx->d_res, ctx->h_res, 0) != hipSuccess)
    return bail(fail(MCDC_E_NOMEM, "pinned result word allocation failed"));
  *out = ctx;
  return MCDC_OK;
}

void mcdc_ctx_destroy(mcdc_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  if (ctx->stream3) (void)hipStreamSynchronize(ctx->stream3);
  if (ctx->stream4) (void)hipStreamSynchronize(ctx->stream4);
  if (ctx->h_tab) (void)hipHostFree(ctx->h_tab);
  if (ctx->h_res) (void)hipHostFree(ctx->h_res);
  if (ctx->h_fcnt) (void)hipHostFree(ctx->h_fcnt);
  if (ctx->h_save) (void)hipHostFree(ctx->h_save);
  if (ctx->h_zarena) (void)hipHostFree(ctx->h_zarena);
  if (ctx->h_encb) (void)hipHostFree(ctx->h_encb);
  if (ctx->h_meta) (void)hipHostFree(ctx->h_meta);
  if (ctx->h_rl) (void)hipHostFree(ctx->h_rl);
  if (ctx->h_list) (void)hipHostFree(ctx->h_list);
  DevBuf *bufs[] = {&ctx->arena, &ctx->run_cnt, &ctx->run_sum, &ctx->run_ent, &ctx->run_bits, &ctx->punt, &ctx->segs, &ctx->files, &ctx->nodes,
                    &ctx->node_off, &ctx->node_cnt, &ctx->seg_exit, &ctx->cont, &ctx->cont_cnt, &ctx->cont_rep,
                    &ctx->cont_ent, &ctx->long_list,
                    &ctx->link_seg, &ctx->link_idx, &ctx->link_pos, &ctx->file_flags,
                    &ctx->seg_true, &ctx->entry_idx, &ctx->seg_count, &ctx->seg_off, &ctx->out,
                    &ctx->err, &ctx->scan_tmp, &ctx->seg_incl, &ctx->irr, &ctx->tile_ctr, &ctx->b3_chunks, &ctx->b3_gcnt,
                    &ctx->b3_goff, &ctx->b3_owner, &ctx->b3_nodes, &ctx->b3_ids, &ctx->b3_tmp, &ctx->b3_hist, &ctx->enc_in, &ctx->enc_out, &ctx->zf_sz,
                    &ctx->zf_off, &ctx->zf_tmp, &ctx->zf_ext,
                    &ctx->ae_ext, &ctx->ae_nonce, &ctx->ae_olen, &ctx->ae_tcnt, &ctx->ae_ooff, &ctx->ae_toff,
                    &ctx->ae_tmp, &ctx->ae_rec, &ctx->ae_keys, &ctx->ae_owner, &ctx->ae_tsum, &ctx->ae_status,
                    &ctx->sv_in, &ctx->sv_pack, &ctx->sv_comp, &ctx->sv_seal, &ctx->sv_ext, &ctx->zc_cnt, &ctx->zc_cls, &ctx->zc_first, &ctx->zc_wcnt, &ctx->zc_wfirst, &ctx->zc_blocks, &ctx->zc_stage,
                    &ctx->zc_piece, &ctx->zc_poff, &ctx->zc_misc, &ctx->zc_tmp, &ctx->zc_words, &ctx->zc_extra,
                    &ctx->zc_blocks2, &ctx->zc_stage2, &ctx->zc_piece2, &ctx->zc_poff2, &ctx->zc_tmp2,
                    &ctx->zc_words2, &ctx->zc_extra2, &ctx->sv_zch, &ctx->sv_zpre, &ctx->sv_zext, &ctx->rl_ent,
                    &ctx->run_list, &ctx->plan_in, &ctx->plan_tmp, &ctx->sv_ids};
  for (DevBuf *b : bufs)
    if (b->p) (void)hipFree(b->p);
  if (ctx->d_gear) (void)hipFree(ctx->d_gear);
  if (ctx->d_gear16) (void)hipFree(ctx->d_gear16);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  hipEvent_t evs[] = {ctx->ev_start, ctx->ev_scan, ctx->ev_end, ctx->ev_h2d0, ctx->ev_h2d1};
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ev_part)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  if (ctx->ev_tab) (void)hipEventDestroy(ctx->ev_tab);
  if (ctx->ev_prep) (void)hipEventDestroy(ctx->ev_prep);
  if (ctx->ev_copy0) (void)hipEventDestroy(ctx->ev_copy0);
  ctx->pool.reset();
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->stream3) (void)hipStreamDestroy(ctx->stream3);
  if (ctx->stream4) (void)hipStreamDestroy(ctx->stream4);
  delete ctx;
}

int mcdc_ctx_timing(const mcdc_ctx *ctx, mcdc_timing *out) {
  if (!ctx || !out) return fail(MCDC_E_INVALID, "NULL argument");
  *out = ctx->timing;
  return MCDC_OK;
}

int mcdc_chunk_device(mcdc_ctx *ctx, const mcdc_params *params, const void *d_data, size_t n,
                      mcdc_chunk *out, size_t cap, size_t *n_out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!d_data && n) return fail(MCDC_E_INVALID, "d_data is NULL");
  if (n > ctx->max_bytes) return fail(MCDC_E_TOOBIG, "n=%zu > max_bytes=%zu", n, ctx->max_bytes);
  const double t0 = now_ms();
  const uintptr_t addr = (uintptr_t)d_data;
  const uint8_t *base = (const uint8_t *)(addr & ~(uintptr_t)15);
  const uint64_t delta = addr & 15;
  const uint64_t n_al = n ? (delta + n + 15) / 16 * 16 : 0;
  const uint64_t fs = delta, fe = delta + n;
  rc = run_pipeline(ctx, params, base, n_al, &fs, &fe, 1, out, cap, nullptr, n_out);
  ctx->timing.h2d_ms = 0;
  ctx->timing.total_ms = now_ms() - t0;
  return rc;
}

int mcdc_chunk_batch_device(mcdc_ctx *ctx, const mcdc_params *params, const void *d_arena,
                            const uint64_t *offsets, const uint64_t *lens, size_t nbufs,
                            mcdc_chunk *out, size_t cap, size_t *counts, size_t *n_out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (nbufs && (!d_arena || !offsets || !lens)) return fail(MCDC_E_INVALID, "NULL argument");
  const double t0 = now_ms();
  ctx->call_t0 = t0;
  struct ClearT0 {  // (every exit, failures included: a later call never reads a stale start)
    mcdc_ctx *c;
    ~ClearT0() { c->call_t0 = 0; }
  } clear_t0{ctx};
  const uintptr_t addr = (uintptr_t)d_arena;
  const uint8_t *base = (const uint8_t *)(addr & ~(uintptr_t)15);
  const uint64_t delta = addr & 15;
  // The scan needs only the arena span.  It is taken from the last non-empty
  // buffer (files laid out in arena order, the usual case) and the scan
  // enqueued at once; the per-file ranges, their overlap check and the true
  // span are built while it runs.  A layout whose last buffer does not end
  // furthest is found there and the call restarts with the true span (the
  // speculative scan read a prefix of it).  Before, a pass over all extents
  // for the span (~0.02 ms for 80 000 files) and the whole range loop
  // (~0.1 ms) preceded the first launch (tools/small_probe.py).
  size_t last = nbufs;
  while (last > 0 && lens[last - 1] == 0) --last;
  uint64_t span = last ? offsets[last - 1] + lens[last - 1] : 0;
  if (last && span < offsets[last - 1]) span = 0;  // (wraps: rejected by ranges() below)
  std::vector<uint64_t> &fs = ctx->bx_fs, &fe = ctx->bx_fe;
  fs.resize(nbufs);
  fe.resize(nbufs);
  bool respan = false;
  auto ranges = [&]() -> int {
    uint64_t hi = 0;
    bool sorted = true;
    for (size_t i = 0; i < nbufs; ++i) {
      if (offsets[i] > UINT64_MAX - 32 - lens[i])
        return fail(MCDC_E_INVALID, "buffer %zu: offset + length overflows", i);
      fs[i] = delta + offsets[i];
      fe[i] = fs[i] + lens[i];
      if (lens[i] == 0) continue;
      sorted = sorted && fs[i] >= hi;  // non-empty ranges in increasing order, disjoint
      hi = std::max(hi, fe[i]);
    }
    if (hi > delta + span) {  // (the span was not the last buffer's end)
      respan = true;
      span = hi - delta;
      return MCDC_E_INTERNAL;
    }
    if (!sorted) {  // any order is allowed, overlaps are not (one chunk chain per byte range)
      std::vector<size_t> idx;
      idx.reserve(nbufs);
      for (size_t i = 0; i < nbufs; ++i)
        if (lens[i]) idx.push_back(i);
      std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return fs[a] < fs[b]; });
      for (size_t k = 1; k < idx.size(); ++k)
        if (fs[idx[k]] < fe[idx[k - 1]])
          return fail(MCDC_E_INVALID, "buffers %zu and %zu overlap", idx[k - 1], idx[k]);
    }
    return MCDC_OK;
  };
  for (int attempt = 0;; ++attempt) {
    // the workspace is sized from the arena span (gaps included), so the span
    // is what the context bound limits
    if (span > ctx->max_bytes)
      return fail(MCDC_E_TOOBIG, "arena span %llu > max_bytes=%zu", (unsigned long long)span, ctx->max_bytes);
    const uint64_t n_al = span ? (span + delta + 15) / 16 * 16 : 0;
    rc = run_pipeline(ctx, params, base, n_al, fs.data(), fe.data(), nbufs, out, cap, counts, n_out, ranges);
    if (!(respan && attempt == 0)) break;
    respan = false;  // (once: ranges() now sees the true span)
  }
  ctx->timing.h2d_ms = 0;
  ctx->timing.total_ms = now_ms() - t0;
  return rc;
}

// Host buffers are packed back to back into the context's device arena
// through two pinned staging slabs: the host copy into slab k + 1 (split over
// the copy pool's threads) runs while slab k's DMA is in flight.  Everything
// is enqueued on the context stream and the scan follows in stream order, so
// the host does not wait for the last DMA before planning the call.
static int stage_to_arena(mcdc_ctx *ctx, const uint8_t *const *bufs, const size_t *lens, size_t nbufs,
                          uint64_t total) {
  int rc = ensure(ctx, ctx->arena, total + 16);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(ctx->ev_copy0, ctx->stream));
  const size_t slab = (size_t)std::min<uint64_t>(total ? total : 1, 256ull << 20);
  hipEvent_t done[2] = {ctx->ev_h2d0, ctx->ev_h2d1};
  uint64_t dst = 0;
  size_t bi = 0, boff = 0;
  int k = 0;
  // Buffers that already live in pinned (or device) memory are DMA'd directly.
  auto direct = [&](const void *p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return at.type == hipMemoryTypeHost || at.type == hipMemoryTypeDevice;
  };
  bool all_direct = nbufs > 0;
  for (size_t i = 0; i < nbufs && all_direct; ++i) all_direct = lens[i] == 0 || direct(bufs[i]);
  if (all_direct) {
    for (size_t i = 0; i < nbufs; ++i) {
      if (lens[i])
        HIP_TRY(hipMemcpyAsync((uint8_t *)ctx->arena.p + dst, bufs[i], lens[i], hipMemcpyDefault, ctx->stream));
      dst += lens[i];
    }
    return MCDC_OK;
  }
  if ((rc = ensure_stage(ctx, 2 * slab))) return rc;
  if (!ctx->pool) {
    const unsigned hw = std::thread::hardware_concurrency();
    ctx->pool.reset(new (std::nothrow) CopyPool((int)std::min(7u, hw > 1 ? hw - 1 : 1u)));
    if (!ctx->pool) return fail(MCDC_E_NOMEM, "host allocation failed");
  }
  uint8_t *stage[2] = {(uint8_t *)ctx->h_stage, (uint8_t *)ctx->h_stage + slab};
  std::vector<CopyPool::Piece> pieces;
  while (dst < total) {
    if (ctx->stage_busy[k]) HIP_TRY(hipEventSynchronize(done[k]));
    pieces.clear();
    size_t fill = 0;
    while (fill < slab && bi < nbufs) {
      const size_t take = std::min(slab - fill, lens[bi] - boff);
      if (take) pieces.push_back({stage[k] + fill, bufs[bi] + boff, take});
      fill += take;
      boff += take;
      if (boff == lens[bi]) { ++bi; boff = 0; }
    }
    ctx->pool->copy(pieces);
    HIP_TRY(hipMemcpyAsync((uint8_t *)ctx->arena.p + dst, stage[k], fill, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipEventRecord(done[k], ctx->stream));
    ctx->stage_busy[k] = true;
    dst += fill;
    k ^= 1;
  }
  return MCDC_OK;
}

int mcdc_chunk_batch(mcdc_ctx *ctx, const mcdc_params *params, const uint8_t *const *bufs,
                     const size_t *lens, size_t nbufs, mcdc_chunk *out, size_t cap, size_t *counts,
                     size_t *n_out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (nbufs && (!bufs || !lens)) return fail(MCDC_E_INVALID, "NULL argument");
  if ((rc = check_params(params, nullptr, nullptr))) return rc;
  const double t0 = now_ms();
  uint64_t total = 0;
  std::vector<uint64_t> offs(nbufs), ls(nbufs);
  for (size_t i = 0; i < nbufs; ++i) {
    if (lens[i] && !bufs[i]) return fail(MCDC_E_INVALID, "bufs[%zu] is NULL", i);
    offs[i] = total;
    ls[i] = lens[i];
    total += lens[i];
  }
  if (total > ctx->max_bytes) return fail(MCDC_E_TOOBIG, "batch bytes %llu > max_bytes", (unsigned long long)total);
  if ((rc = stage_to_arena(ctx, bufs, lens, nbufs, total))) {
    (void)hipStreamSynchronize(ctx->stream);  // nothing may still read the caller's buffers
    return rc;
  }
  std::vector<uint64_t> fs(nbufs), fe(nbufs);
  for (size_t i = 0; i < nbufs; ++i) { fs[i] = offs[i]; fe[i] = offs[i] + ls[i]; }
  const uint64_t n_al = (total + 15) / 16 * 16;
  rc = run_pipeline(ctx, params, (const uint8_t *)ctx->arena.p, n_al, fs.data(), fe.data(), nbufs,
                    out, cap, counts, n_out);
  if (rc) (void)hipStreamSynchronize(ctx->stream);
  float h2d = 0;  // first input copy to the scan's start, on the stream
  if (!rc && hipEventElapsedTime(&h2d, ctx->ev_copy0, ctx->ev_start) != hipSuccess) {
    (void)hipGetLastError();
    h2d = 0;
  }
  ctx->timing.h2d_ms = h2d;
  ctx->timing.total_ms = now_ms() - t0;
  return rc;
}

int mcdc_chunk_host(mcdc_ctx *ctx, const mcdc_params *params, const void *h_data, size_t n,
                    mcdc_chunk *out, size_t cap, size_t *n_out) {
  const uint8_t *b = (const uint8_t *)h_data;
  if (!h_data && n) return fail(MCDC_E_INVALID, "h_data is NULL");
  return mcdc_chunk_batch(ctx, params, &b, &n, 1, out, cap, nullptr, n_out);
}

int mcdc_device_alloc(mcdc_ctx *ctx, size_t bytes, void **d_ptr) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!d_ptr) return fail(MCDC_E_INVALID, "d_ptr is NULL");
  if (hipMalloc(d_ptr, bytes ? bytes : 16) != hipSuccess) {
    (void)hipGetLastError();
    *d_ptr = nullptr;
    return fail(MCDC_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  }
  return MCDC_OK;
}

int mcdc_device_free(mcdc_ctx *ctx, void *d_ptr) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (d_ptr) HIP_TRY(hipFree(d_ptr));
  return MCDC_OK;
}

int mcdc_ctx_synchronize(mcdc_ctx *ctx) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  // the context's own streams (every call of the library enqueues on them),
  // then the null stream (the plain copies of the utilities): other
  // contexts' work on the device is not waited for
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream2));
  HIP_TRY(hipStreamSynchronize(ctx->stream3));
  HIP_TRY(hipStreamSynchronize(ctx->stream4));
  HIP_TRY(hipStreamSynchronize(nullptr));
  return MCDC_OK;
}

int mcdc_ctx_set_option(mcdc_ctx *ctx, const char *name, long long value) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!name) return fail(MCDC_E_INVALID, "option name is NULL");
  const std::string n(name);
  if (n == "zc_batch_blocks") {
    if (value < (long long)kZcSegBlocks || value > (1ll << 24))
      return fail(MCDC_E_INVALID, "zc_batch_blocks %lld outside [%u, 2^24]", value, kZcSegBlocks);
    ctx->knobs.zc_batch = (uint64_t)value;
  } else if (n == "zc_two") {
    ctx->knobs.zc_two = value != 0;
  } else if (n == "zc_small") {
    ctx->knobs.zc_small = value != 0;
  } else if (n == "save_group_blocks") {
    if (value < 0) return fail(MCDC_E_INVALID, "save_group_blocks %lld < 0", value);
    ctx->knobs.save_group_blocks = (uint64_t)value;
  } else if (n == "test_fail_after_index") {
    ctx->knobs.test_fail_after_index = value != 0;
  } else {
    return fail(MCDC_E_INVALID, "unknown option '%s'", name);
  }
  return MCDC_OK;
}

int mcdc_host_alloc(mcdc_ctx *ctx, size_t bytes, void **h_ptr) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!h_ptr) return fail(MCDC_E_INVALID, "h_ptr is NULL");
  if (hipHostMalloc(h_ptr, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *h_ptr = nullptr;
    return fail(MCDC_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
  }
  return MCDC_OK;
}

int mcdc_host_free(mcdc_ctx *ctx, void *h_ptr) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (h_ptr) HIP_TRY(hipHostFree(h_ptr));
  return MCDC_OK;
}

int mcdc_memcpy_h2d(mcdc_ctx *ctx, void *d_dst, const void *h_src, size_t bytes) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MCDC_OK;
}

int mcdc_chunk_ids_device(mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks, size_t nchunks,
                          uint8_t *ids) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!d_data && n) || (nchunks && (!chunks || !ids))) return fail(MCDC_E_INVALID, "NULL argument");
  // (chunk indices are 32-bit in the group owners and the wide-tree list; the scan counts in int)
  if (nchunks >= (1ull << 31)) return fail(MCDC_E_TOOBIG, "too many chunks (%zu)", nchunks);
  const double t0 = now_ms();
  hipStream_t st = ctx->stream;
  ctx->timing = mcdc_timing{};
  if (nchunks == 0) {
    ctx->timing.total_ms = now_ms() - t0;
    return MCDC_OK;
  }
  const DevChunk *dch = nullptr;
  if (is_device_ptr(chunks)) {
    if (!direct_out(ctx, (void *)chunks)) return fail(MCDC_E_INVALID, "chunks is a device pointer of another device");
    dch = (const DevChunk *)chunks;
  } else {
    if ((rc = ensure(ctx, ctx->b3_chunks, nchunks * sizeof(DevChunk)))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->b3_chunks.p, chunks, nchunks * sizeof(DevChunk), hipMemcpyHostToDevice, st));
    dch = (const DevChunk *)ctx->b3_chunks.p;
  }
  uint8_t *ids_dev = (uint8_t *)direct_out(ctx, ids);
  if (!ids_dev && is_device_ptr(ids)) return fail(MCDC_E_INVALID, "ids is a device pointer of another device");
  // groups of disjoint chunks never exceed this bound; overlapping or repeated
  // chunks can, and are then hashed again with the exact count read back
  uint64_t bound = b3_group_bound(n, nchunks);
  const size_t tmpb = b3_tmp_bytes(nchunks);
  if ((rc = ensure(ctx, ctx->b3_gcnt, (nchunks + 1) * 8)) || (rc = ensure(ctx, ctx->b3_goff, (nchunks + 1) * 8)) ||
      (rc = ensure(ctx, ctx->b3_owner, bound * 4)) || (rc = ensure(ctx, ctx->b3_nodes, bound * 32)) ||
      (rc = ensure(ctx, ctx->b3_tmp, tmpb)) || (rc = ensure(ctx, ctx->err, 16)) ||
      (rc = ensure(ctx, ctx->b3_hist, kB3HistWords * 4)))
    return rc;
  uint32_t *hist = (uint32_t *)ctx->b3_hist.p;
  if (!ids_dev) {
    if ((rc = ensure(ctx, ctx->b3_ids, nchunks * 32))) return rc;
    ids_dev = (uint8_t *)ctx->b3_ids.p;
  }
  uint32_t *err = (uint32_t *)ctx->err.p + 3;
  const uint64_t *goff = (const uint64_t *)ctx->b3_goff.p;
  HIP_TRY(hipMemsetAsync(err, 0, 4, st));
  HIP_TRY(hipEventRecord(ctx->ev_start, st));
  launch_b3_prepare(dch, nchunks, n, (uint64_t *)ctx->b3_gcnt.p, (uint64_t *)ctx->b3_goff.p, hist, err, ctx->b3_tmp.p,
                    tmpb, st);
  launch_b3_hash((const uint8_t *)d_data, dch, nchunks, goff, bound, hist, (uint32_t *)ctx->b3_owner.p,
                 (uint32_t *)ctx->b3_nodes.p, ids_dev, (uint64_t *)ctx->b3_gcnt.p, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev_end, st));
  uint32_t herr = 0;
  uint64_t groups = 0;
  HIP_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&groups, goff + nchunks, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  groups = b3_groups_total(groups);
  if (herr) return fail(MCDC_E_INVALID, "a chunk lies outside the %zu-byte buffer", n);
  if (groups > bound) {  // overlapping / repeated chunks: the kernels skipped; hash with the exact bound
    bound = groups;
    if ((rc = ensure(ctx, ctx->b3_owner, bound * 4)) || (rc = ensure(ctx, ctx->b3_nodes, bound * 32))) return rc;
    HIP_TRY(hipEventRecord(ctx->ev_start, st));
    launch_b3_hash((const uint8_t *)d_data, dch, nchunks, goff, bound, hist, (uint32_t *)ctx->b3_owner.p,
                   (uint32_t *)ctx->b3_nodes.p, ids_dev, (uint64_t *)ctx->b3_gcnt.p, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->ev_end, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  if (ids_dev == ctx->b3_ids.p) {
    HIP_TRY(hipMemcpyAsync(ids, ids_dev, nchunks * 32, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_end));
  ctx->timing.ids_ms = ms;
  ctx->timing.device_ms = ms;
  ctx->timing.bytes = n;
  ctx->timing.chunks = nchunks;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

int mcdc_seal_device(mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in, const mcdc_blob *blobs,
                     size_t nblobs, const uint8_t *nonces, void *d_out, size_t out_cap, uint64_t *out_offsets) {
  return aead_run(ctx, 0, key, d_in, n_in, blobs, nblobs, nonces, d_out, out_cap, out_offsets, nullptr);
}

int mcdc_seal_chunks_device(mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in,
                            const mcdc_chunk *chunks, size_t nchunks, const uint8_t *nonces, void *d_out,
                            size_t out_cap, uint64_t *out_offsets) {
  if (nchunks && !chunks) return fail(MCDC_E_INVALID, "chunks is NULL");
  return aead_run(ctx, 0, key, d_in, n_in, nullptr, nchunks, nonces, d_out, out_cap, out_offsets, nullptr, chunks);
}

int mcdc_open_device(mcdc_ctx *ctx, const uint8_t key[32], const void *d_in, size_t n_in, const mcdc_blob *sealed,
                     size_t nblobs, void *d_out, size_t out_cap, uint64_t *out_offsets, int32_t *status) {
  return aead_run(ctx, 1, key, d_in, n_in, sealed, nblobs, nullptr, d_out, out_cap, out_offsets, status);
}

}  // extern "C"

// ------------------------------------------------------------ dedup index --
// The blob-exists check of Repository::save_blob for a batch
// (/root/reference/src/repository/repository_v1.rs:169-180), csrc/mcdc_index.hip.
struct mcdc_index {
  int device = 0;
  DevBuf pfx[2], ids[2];  // sorted by prefix; [cur] is live, the other is the merge target
  int cur = 0;
  uint64_t size = 0;
  // per-call scratch
  DevBuf keys, skeys, pos, spos, sflag, is_new, count, tmp, ids_in, chunks_in, chunks_out;
};

extern "C" {

int mcdc_index_create(mcdc_ctx *ctx, mcdc_index **out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out) return fail(MCDC_E_INVALID, "NULL argument");
  *out = new (std::nothrow) mcdc_index;
  if (!*out) return fail(MCDC_E_NOMEM, "out of host memory");
  (*out)->device = ctx->device;
  return MCDC_OK;
}

void mcdc_index_destroy(mcdc_index *ix) {
  if (!ix) return;
  (void)hipSetDevice(ix->device);
  DevBuf *bufs[] = {&ix->pfx[0], &ix->pfx[1], &ix->ids[0], &ix->ids[1], &ix->keys, &ix->skeys, &ix->pos,
                    &ix->spos, &ix->sflag, &ix->is_new, &ix->count, &ix->tmp, &ix->ids_in, &ix->chunks_in,
                    &ix->chunks_out};
  for (DevBuf *b : bufs)
    if (b->p) (void)hipFree(b->p);
  delete ix;
}

size_t mcdc_index_size(const mcdc_index *ix) { return ix ? (size_t)ix->size : 0; }

int mcdc_index_add(mcdc_ctx *ctx, mcdc_index *ix, const uint8_t *ids, size_t n, uint8_t *is_new,
                   const mcdc_chunk *chunks, mcdc_chunk *new_chunks, size_t *n_new) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!ix || (n && !ids) || (!chunks != !new_chunks)) return fail(MCDC_E_INVALID, "NULL argument");
  if (ix->device != ctx->device) return fail(MCDC_E_INVALID, "the index lives on device %d", ix->device);
  if (n >= (1ull << 31)) return fail(MCDC_E_TOOBIG, "too many IDs (%zu)", n);
  const double t0 = now_ms();
  hipStream_t st = ctx->stream;
  ctx->timing = mcdc_timing{};
  if (n_new) *n_new = 0;
  if (n == 0) {
    ctx->timing.total_ms = now_ms() - t0;
    return MCDC_OK;
  }
  const size_t tmpb = idx_tmp_bytes(n);
  if ((rc = stage_arg(ctx, ix->ids_in, ids, n * 32)) || (rc = ensure(ctx, ix->keys, n * 8)) ||
      (rc = ensure(ctx, ix->skeys, n * 8)) || (rc = ensure(ctx, ix->pos, n * 4)) || (rc = ensure(ctx, ix->spos, n * 4)) ||
      (rc = ensure(ctx, ix->sflag, n)) || (rc = ensure(ctx, ix->is_new, n)) || (rc = ensure(ctx, ix->count, 16)) ||
      (rc = ensure(ctx, ix->tmp, tmpb)))
    return rc;
  const uint8_t *d_ids = (const uint8_t *)ix->ids_in.p;
  IdxScratch sc{(uint64_t *)ix->keys.p, (uint64_t *)ix->skeys.p, (uint32_t *)ix->pos.p, (uint32_t *)ix->spos.p,
                (uint8_t *)ix->sflag.p, (uint64_t *)ix->count.p, ix->tmp.p, tmpb};
  IdxIndexView view{(const uint64_t *)ix->pfx[ix->cur].p, (const uint8_t *)ix->ids[ix->cur].p, ix->size};
  HIP_TRY(hipEventRecord(ctx->ev_start, st));
  launch_idx_mark(d_ids, n, view, sc, (uint8_t *)ix->is_new.p, st);
  HIP_TRY(hipGetLastError());
  uint64_t m = 0;
  HIP_TRY(hipMemcpyAsync(&m, sc.count, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int nxt = ix->cur ^ 1;
  if ((rc = ensure(ctx, ix->pfx[nxt], (ix->size + m) * 8)) || (rc = ensure(ctx, ix->ids[nxt], (ix->size + m) * 32)))
    return rc;
  launch_idx_merge(d_ids, m, view, sc, (uint64_t *)ix->pfx[nxt].p, (uint8_t *)ix->ids[nxt].p, st);
  HIP_TRY(hipGetLastError());
  if (chunks) {
    if ((rc = stage_arg(ctx, ix->chunks_in, chunks, n * sizeof(mcdc_chunk))) ||
        (rc = ensure(ctx, ix->chunks_out, n * sizeof(mcdc_chunk))))
      return rc;
    launch_idx_compact_chunks((const DevChunk *)ix->chunks_in.p, (const uint8_t *)ix->is_new.p, n,
                              (DevChunk *)ix->chunks_out.p, sc.count + 1, sc.tmp, tmpb, st);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(ctx->ev_end, st));
  if ((rc = give_back(ctx, is_new, ix->is_new.p, n)) ||
      (chunks && (rc = give_back(ctx, new_chunks, ix->chunks_out.p, m * sizeof(mcdc_chunk)))))
    return rc;
  HIP_TRY(hipStreamSynchronize(st));
  ix->cur = nxt;
  ix->size += m;
  if (n_new) *n_new = (size_t)m;
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_end));
  ctx->timing.device_ms = ms;
  ctx->timing.chunks = n;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

// ------------------------------------------------------ SecureStorage ---
// encode / decode of many host blobs: zstd on host threads (host/zstd_stage.hpp),
// AES-256-GCM-SIV on the GPU (aead_run).
static int zstd_threads() {
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, hw ? hw : 1u));
}

static int check_extents(const mcdc_blob *b, size_t n, size_t n_in) {
  for (size_t i = 0; i < n; ++i)
    if (b[i].offset > n_in || b[i].length > n_in - b[i].offset)
      return fail(MCDC_E_INVALID, "blob %zu lies outside the %zu-byte input", i, n_in);
  return MCDC_OK;
}

int mcdc_encode_blobs(mcdc_ctx *ctx, const uint8_t key[32], const void *h_in, size_t n_in, const mcdc_blob *blobs,
                      size_t nblobs, const uint8_t *nonces, void *h_out, size_t out_cap, uint64_t *out_offsets) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!h_in && n_in) || (nblobs && (!blobs || (key && !nonces)))) return fail(MCDC_E_INVALID, "NULL argument");
  if ((h_in && is_device_ptr(h_in)) || (h_out && is_device_ptr(h_out)))
    return fail(MCDC_E_INVALID, "h_in / h_out must be host memory");
  if ((rc = check_extents(blobs, nblobs, n_in))) return rc;
  const double t0 = now_ms();
  std::vector<uint64_t> off(nblobs), len(nblobs);
  for (size_t i = 0; i < nblobs; ++i) off[i] = blobs[i].offset, len[i] = blobs[i].length;
  // every frame into its own bound-sized region of one buffer (no per-blob
  // allocation or zero fill), then packed back to back
  const mcdc::host::ZstdApi &za = mcdc::host::zstd_api();
  if (!za.ok) return fail(MCDC_E_INTERNAL, "%s", za.why.c_str());
  std::vector<uint64_t> bo(nblobs + 1, 0), clen(nblobs, 0);
  for (size_t i = 0; i < nblobs; ++i) bo[i + 1] = bo[i] + za.compressBound(len[i]) + 64;
  if (ctx->h_zbuf_cap < bo[nblobs]) {  // (kept by the context: a fresh multi-GB buffer per call page-faults)
    const size_t alloc = (size_t)(bo[nblobs] + bo[nblobs] / 8 + 4096);
    ctx->h_zbuf.reset(new (std::nothrow) uint8_t[alloc]);
    ctx->h_zbuf_cap = ctx->h_zbuf ? alloc : 0;
    if (!ctx->h_zbuf) return fail(MCDC_E_NOMEM, "host allocation of %zu bytes failed", alloc);
  }
  uint8_t *const cbuf = ctx->h_zbuf.get();
  const std::string zerr = mcdc::host::zstd_compress_into((const uint8_t *)h_in, off.data(), len.data(), nblobs,
                                                          zstd_threads(), cbuf, bo.data(), clen.data());
  if (!zerr.empty()) return fail(MCDC_E_INTERNAL, "%s", zerr.c_str());
  std::vector<mcdc_blob> ext(nblobs);
  size_t total = 0;
  for (size_t i = 0; i < nblobs; ++i) ext[i] = mcdc_blob{total, clen[i]}, total += clen[i];
  if ((rc = ensure_pinned(ctx, ctx->h_zarena, ctx->h_zarena_cap, std::max<size_t>(total, 1)))) return rc;
  uint8_t *const arena = (uint8_t *)ctx->h_zarena;  // (pinned: the H2D below runs at the DMA rate)
  mcdc::host::parallel_items(nblobs, zstd_threads(), [&](size_t i, int) {
    if (clen[i]) std::memcpy(arena + ext[i].offset, cbuf + bo[i], clen[i]);
  });
  if (!key) {  // SecureStorage::build(): no key, encrypt() returns the compressed bytes (storage.rs:120-125)
    if (out_offsets) {
      for (size_t i = 0; i < nblobs; ++i) out_offsets[i] = ext[i].offset;
      out_offsets[nblobs] = total;
    }
    if (total > out_cap || (total && !h_out))
      return fail(MCDC_E_CAPACITY, "output capacity %zu < %zu bytes", out_cap, total);
    if (total) std::memcpy(h_out, arena, total);
    ctx->timing = mcdc_timing{};
    ctx->timing.bytes = n_in;
    ctx->timing.total_ms = now_ms() - t0;
    return MCDC_OK;
  }
  const size_t cap = total + (size_t)kAeadOverhead * nblobs;
  if ((rc = ensure(ctx, ctx->enc_in, total)) || (rc = ensure(ctx, ctx->enc_out, cap))) return rc;
  if (total) HIP_TRY(hipMemcpyAsync(ctx->enc_in.p, arena, total, hipMemcpyHostToDevice, ctx->stream));
  std::vector<uint64_t> oo(nblobs + 1);
  if ((rc = aead_run(ctx, 0, key, ctx->enc_in.p, total, ext.data(), nblobs, nonces, ctx->enc_out.p, cap, oo.data(),
                     nullptr)))
    return rc;
  const mcdc_timing tm = ctx->timing;
  if (out_offsets) std::memcpy(out_offsets, oo.data(), (nblobs + 1) * 8);
  if (oo[nblobs] > out_cap || (oo[nblobs] && !h_out))
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %llu bytes", out_cap, (unsigned long long)oo[nblobs]);
  if (oo[nblobs]) {
    HIP_TRY(hipMemcpyAsync(h_out, ctx->enc_out.p, oo[nblobs], hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  ctx->timing = tm;
  ctx->timing.bytes = n_in;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

int mcdc_decode_blobs(mcdc_ctx *ctx, const uint8_t key[32], const void *h_in, size_t n_in, const mcdc_blob *sealed,
                      size_t nblobs, void *h_out, size_t out_cap, uint64_t *out_offsets, int32_t *status) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!h_in && n_in) || (nblobs && !sealed)) return fail(MCDC_E_INVALID, "NULL argument");
  if ((h_in && is_device_ptr(h_in)) || (h_out && is_device_ptr(h_out)))
    return fail(MCDC_E_INVALID, "h_in / h_out must be host memory");
  if ((rc = check_extents(sealed, nblobs, n_in))) return rc;
  const double t0 = now_ms();
  std::vector<uint64_t> poff(nblobs), plen(nblobs);
  std::vector<int32_t> st(std::max<size_t>(nblobs, 1), 0);
  const uint8_t *zin = (const uint8_t *)h_in;
  mcdc_timing tm{};
  if (key) {
    if ((rc = ensure(ctx, ctx->enc_in, n_in)) || (rc = ensure(ctx, ctx->enc_out, n_in))) return rc;
    if (n_in) HIP_TRY(hipMemcpyAsync(ctx->enc_in.p, h_in, n_in, hipMemcpyHostToDevice, ctx->stream));
    std::vector<uint64_t> oo(nblobs + 1);
    rc = aead_run(ctx, 1, key, ctx->enc_in.p, n_in, sealed, nblobs, nullptr, ctx->enc_out.p, n_in, oo.data(),
                  st.data());
    if (rc && rc != MCDC_E_AUTH) return rc;
    tm = ctx->timing;
    // (the opened frames into a pinned buffer the context keeps: DMA rate, no
    // zero fill or page faults per call)
    if ((rc = ensure_pinned(ctx, ctx->h_zarena, ctx->h_zarena_cap, std::max<uint64_t>(oo[nblobs], 1)))) return rc;
    uint8_t *const plain = (uint8_t *)ctx->h_zarena;
    if (oo[nblobs]) {
      HIP_TRY(hipMemcpyAsync(plain, ctx->enc_out.p, oo[nblobs], hipMemcpyDeviceToHost, ctx->stream));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    for (size_t i = 0; i < nblobs; ++i) poff[i] = oo[i], plen[i] = oo[i + 1] - oo[i];
    zin = plain;
  } else {  // SecureStorage::build(): decrypt() is the identity, only decompress (storage.rs:67-69)
    for (size_t i = 0; i < nblobs; ++i) poff[i] = sealed[i].offset, plen[i] = sealed[i].length;
  }
  std::vector<std::vector<uint8_t>> dec;
  std::vector<int32_t> zok;
  const std::string zerr = mcdc::host::zstd_decompress_all(zin, poff.data(), plen.data(), st.data(),
                                                           nblobs, zstd_threads(), dec, zok);
  if (!zerr.empty()) return fail(MCDC_E_INTERNAL, "%s", zerr.c_str());
  size_t total = 0, bad = 0;
  std::vector<uint64_t> doff(nblobs + 1);
  for (size_t i = 0; i < nblobs; ++i) {
    const int32_t s = st[i] ? -1 : zok[i];
    if (status) status[i] = s;
    bad += s != 0;
    doff[i] = total;
    total += dec[i].size();
  }
  doff[nblobs] = total;
  if (out_offsets) std::memcpy(out_offsets, doff.data(), (nblobs + 1) * 8);
  if (total > out_cap || (total && !h_out))
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %zu bytes", out_cap, total);
  mcdc::host::parallel_items(nblobs, zstd_threads(), [&](size_t i, int) {
    if (!dec[i].empty()) std::memcpy((uint8_t *)h_out + doff[i], dec[i].data(), dec[i].size());
  });
  ctx->timing = tm;
  ctx->timing.total_ms = now_ms() - t0;
  if (bad) return fail(MCDC_E_AUTH, "%zu of %zu blobs failed to decode", bad, nblobs);
  return MCDC_OK;
}

// The GPU save path's seal of n blobs of d_in (extents ext, host, relative to
// d_in; nonces: 12 B each) into d_out at host-given places, enqueued on
// `st` with no host wait: the output and tile offsets (k_aead_sizes' rule)
// computed on the host, the records staged from pinned memory `stage` (at
// least seal_stage_bytes(n), untouched until `st` has run the copies), the
// context's AEAD workspace reused in stream order (ensured beforehand for
// the largest call: ensure() would wait for every stream).
static size_t seal_stage_bytes(size_t n) { return n * (16 + 12) + 2 * (n + 1) * 8 + 64; }
static uint64_t seal_tiles(uint64_t len) {  // (k_aead_sizes, seal: tiles of a blob of len bytes)
  const uint64_t T = len + kAeadOverhead;
  const uint64_t ct = ((T - 1) / 16 + 2 + kAeadTileBlocks - 1) / kAeadTileBlocks;
  const uint64_t nblk = (len + 15) / 16, rows = (nblk + 63) / 64;
  uint64_t pt = (rows + kAeadRows - 1) / kAeadRows;
  if (pt > 1 && rows - kAeadRows * (pt - 1) < kAeadRows / 2) --pt;
  return ct > pt ? ct : pt;
}
static int seal_workspace(mcdc_ctx *ctx, size_t n, uint64_t ntiles) {
  int rc;
  if ((rc = ensure(ctx, ctx->ae_ext, n * 16)) || (rc = ensure(ctx, ctx->ae_nonce, n * kAeadNonce)) ||
      (rc = ensure(ctx, ctx->ae_ooff, (n + 1) * 8)) || (rc = ensure(ctx, ctx->ae_toff, (n + 1) * 8)) ||
      (rc = ensure(ctx, ctx->ae_rec, n * sizeof(AeadRec))) || (rc = ensure(ctx, ctx->ae_keys, n * sizeof(AeadKeys))) ||
      (rc = ensure(ctx, ctx->ae_owner, ntiles * 4)) || (rc = ensure(ctx, ctx->ae_tsum, ntiles * 16)) ||
      (rc = ensure(ctx, ctx->err, 32)))
    return rc;
  return MCDC_OK;
}
static int seal_placed(mcdc_ctx *ctx, hipStream_t st, const uint8_t *key, const uint8_t *d_in, const mcdc_blob *ext,
                       size_t n, const uint8_t *nonces, uint8_t *d_out, const uint64_t *place, uint8_t *stage) {
  if (n == 0) return MCDC_OK;
  uint64_t *sx = reinterpret_cast<uint64_t *>(stage);  // ext pairs, then ooff, toff; nonces after
  uint64_t *so = sx + 2 * n, *stt = so + n + 1;
  uint8_t *sn = reinterpret_cast<uint8_t *>(stt + n + 1);
  uint64_t nt = 0;
  for (size_t i = 0; i < n; ++i) {
    sx[2 * i] = ext[i].offset;
    sx[2 * i + 1] = ext[i].length;
    so[i] = place[i];
    stt[i] = nt;
    nt += seal_tiles(ext[i].length);
  }
  so[n] = place[n];
  stt[n] = nt;
  std::memcpy(sn, nonces, n * kAeadNonce);
  if (nt >= (1ull << 32)) return fail(MCDC_E_TOOBIG, "input too large (%llu tiles)", (unsigned long long)nt);
  if (ctx->ae_owner.cap < nt * 4 || ctx->ae_tsum.cap < nt * 16 || ctx->ae_ext.cap < n * 16 ||
      ctx->ae_rec.cap < n * sizeof(AeadRec) || ctx->ae_keys.cap < n * sizeof(AeadKeys))
    return fail(MCDC_E_INTERNAL, "save path: seal workspace not reserved");
  HIP_TRY(hipMemcpyAsync(ctx->ae_ext.p, sx, n * 16, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->ae_ooff.p, so, (n + 1) * 8, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->ae_toff.p, stt, (n + 1) * 8, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->ae_nonce.p, sn, n * kAeadNonce, hipMemcpyHostToDevice, st));
  AeadMaster mk;
  aead_expand_key256(key, mk.rk);
  launch_aead_seal(mk, d_in, (const uint64_t *)ctx->ae_ext.p, (const uint32_t *)ctx->ae_nonce.p, n, d_out,
                   (const uint64_t *)ctx->ae_ooff.p, (const uint64_t *)ctx->ae_toff.p, nt, (AeadRec *)ctx->ae_rec.p,
                   (AeadKeys *)ctx->ae_keys.p, (uint32_t *)ctx->ae_owner.p, (uint4 *)ctx->ae_tsum.p,
                   (uint32_t *)ctx->err.p + 4, ctx->num_cus, st);
  std::memset(mk.rk, 0, sizeof mk.rk);
  HIP_TRY(hipGetLastError());
  return MCDC_OK;
}


// ------------------------------------------------------------ pack plan --
// Packer::add_blob / flush over a run of encoded blob lengths
// (packer.rs:101-186, flush rule repository_v1.rs:185-193): which blobs go in
// which pack, each pack's header (generate_header: 37-byte entries, padded to
// a multiple of 64 with the caller's random entries) SecureStorage-encoded
// (mcdc_encode_blobs), and the pack extents: blobs || encode(header) ||
// le32(len).  Shared by the host packer (mcdc_pack_blobs) and the GPU save
// path, which assembles the same layout in HBM.
static constexpr size_t kHeaderEntry = 37, kHeaderMultiple = 64;  // packer.rs:30, defaults.rs:32

struct PackPlan {
  std::vector<size_t> first;    // first blob of each pack, + nblobs
  std::vector<uint8_t> meta;    // per pack: encode(header) || le32(len), back to back
  std::vector<uint64_t> moff;   // pack k's meta = meta[moff[k], moff[k + 1])
  std::vector<uint64_t> body;   // body bytes per pack
  std::vector<mcdc_chunk> pk;   // pack extents in the output (offset, length)
  size_t total = 0;
  size_t np() const { return first.empty() ? 0 : first.size() - 1; }
};

static int plan_packs(mcdc_ctx *ctx, const uint8_t key[32], const uint64_t *lens, const uint8_t *ids,
                      const uint8_t *types, size_t nblobs, uint64_t max_pack_size, const uint8_t *header_nonces,
                      size_t nnonces, const uint8_t *padding, size_t npadding, PackPlan &P) {
  for (size_t i = 0; i < nblobs; ++i)
    if (lens[i] > 0xffffffffull) return fail(MCDC_E_INVALID, "blob %zu exceeds the header's u32 length", i);
  // add, then flush once the packer holds more than max_pack_size bytes; the
  // rest is flushed last
  P.first.clear();
  uint64_t size = 0;
  bool open = false;
  for (size_t i = 0; i < nblobs; ++i) {
    if (!open) P.first.push_back(i), open = true;
    size += lens[i];
    if (size > max_pack_size) size = 0, open = false;
  }
  const size_t np = P.first.size();
  P.first.push_back(nblobs);
  if (key && np > nnonces)  // (without a key the headers are only compressed: no nonces)
    return fail(MCDC_E_INVALID, "%zu packs need %zu header nonces (%zu given)", np, np, nnonces);
  std::vector<uint8_t> hdr;
  std::vector<mcdc_blob> hext(np);
  size_t pad_used = 0;
  for (size_t k = 0; k < np; ++k) {
    const size_t cnt = P.first[k + 1] - P.first[k];
    const size_t pad = cnt % kHeaderMultiple ? kHeaderMultiple - cnt % kHeaderMultiple : 0;
    if (pad_used + pad > npadding)
      return fail(MCDC_E_INVALID, "the padding pool holds %zu entries, the headers need more", npadding);
    hext[k] = mcdc_blob{hdr.size(), (cnt + pad) * kHeaderEntry};
    for (size_t i = P.first[k]; i < P.first[k + 1]; ++i) {
      const uint32_t len = (uint32_t)lens[i];
      hdr.insert(hdr.end(), ids + 32 * i, ids + 32 * i + 32);
      for (int b = 0; b < 4; ++b) hdr.push_back((uint8_t)(len >> (8 * b)));
      hdr.push_back(types[i]);
    }
    for (size_t j = 0; j < pad; ++j, ++pad_used) {
      hdr.insert(hdr.end(), padding + 36 * pad_used, padding + 36 * pad_used + 36);
      hdr.push_back(0xff);
    }
  }
  SAVE_T("plan headers");
  // SecureStorage::encode of every header (zstd on host threads, sealing on the GPU)
  size_t enc_cap = hdr.size() + hdr.size() / 64 + 1024 * np + 64;
  std::vector<uint8_t> enc(enc_cap);
  std::vector<uint64_t> eo(np + 1, 0);
  if (np) {
    int rc = mcdc_encode_blobs(ctx, key, hdr.data(), hdr.size(), hext.data(), np, header_nonces, enc.data(), enc_cap,
                               eo.data());
    if (rc == MCDC_E_CAPACITY) {
      enc.resize(eo[np]);
      enc_cap = enc.size();
      rc = mcdc_encode_blobs(ctx, key, hdr.data(), hdr.size(), hext.data(), np, header_nonces, enc.data(), enc_cap,
                             eo.data());
    }
    if (rc) return rc;
  }
  SAVE_T("plan encoded");
  P.meta.clear();
  P.moff.assign(np + 1, 0);
  P.body.assign(np, 0);
  P.pk.assign(np, mcdc_chunk{});
  P.total = 0;
  for (size_t k = 0; k < np; ++k) {
    const uint32_t hl = (uint32_t)(eo[k + 1] - eo[k]);
    P.meta.insert(P.meta.end(), enc.data() + eo[k], enc.data() + eo[k + 1]);
    for (int b = 0; b < 4; ++b) P.meta.push_back((uint8_t)(hl >> (8 * b)));
    P.moff[k + 1] = P.meta.size();
    for (size_t i = P.first[k]; i < P.first[k + 1]; ++i) P.body[k] += lens[i];
    P.pk[k] = mcdc_chunk{P.total, P.body[k] + hl + 4, 0};
    P.total += P.body[k] + hl + 4;
  }
  return MCDC_OK;
}

static void fill_pack_records(const PackPlan &P, const uint8_t *pid, mcdc_pack *packs) {
  for (size_t k = 0; k < P.np(); ++k) {
    packs[k].offset = P.pk[k].offset;
    packs[k].length = P.pk[k].length;
    packs[k].nblobs = P.first[k + 1] - P.first[k];
    packs[k].meta_size = P.moff[k + 1] - P.moff[k];
    std::memcpy(packs[k].id, pid + 32 * k, 32);
  }
}

// ------------------------------------------------------------ save path --

// ---------------------------------------------------- zstd compression --
// The compressor's batches: whole chunks, in order, each within `cap_w` words
// (zc_span, ~ its input bytes) and `cap_b` blocks unless one chunk is
// longer.  Two scratch sets on two streams (batches alternate) when the list
// takes more than one set of "zc_batch_blocks" / 2 x 32 KiB of words; one
// set of up to the whole batch otherwise.  first / wfirst: the chunks'
// block and word prefixes (n + 1 entries, relative: only differences count).
struct ZcBatches {
  std::vector<size_t> cut;  // batch k: chunks [cut[k], cut[k + 1])
  uint64_t mw = 0, mb = 0;  // the largest batch's words and blocks (the scratch sets' sizes)
  bool two = false;
};
static ZcBatches zc_batches(const uint64_t *first, const uint64_t *wfirst, size_t n, const Knobs &kn) {
  ZcBatches r;
  uint64_t longest_w = 0, longest_b = 0;
  for (size_t i = 0; i < n; ++i) {
    longest_w = std::max(longest_w, wfirst[i + 1] - wfirst[i]);
    longest_b = std::max(longest_b, first[i + 1] - first[i]);
  }
  const uint64_t zb = kn.zc_batch, set_w = std::min<uint64_t>(zb / 2 * kZcBlock, 1ull << 31);
  const uint64_t total_w = wfirst[n] - wfirst[0], total_b = first[n] - first[0];
  r.two = kn.zc_two && total_w > set_w && longest_w <= set_w;
  // (blocks: twice the words' full blocks, so that a set of shorter blocks
  // -- small files -- still holds the words' worth of input.  Two half
  // batches for a call of one set or less, on the two streams, measured no
  // faster: tools/tree_probe.py 29.8-31.1 vs 29.6-31.1 ms, 256 MiB of text
  // 59.6 vs 60.7 GiB/s, the same box)
  const uint64_t cap_w = r.two ? set_w : std::max(std::min<uint64_t>(total_w, 2 * set_w), longest_w);
  const uint64_t cap_b = r.two ? zb : std::max(std::min<uint64_t>(total_b, 2 * zb), longest_b);
  for (size_t c0 = 0; c0 < n;) {
    size_t c1 = c0 + 1;
    while (c1 < n && wfirst[c1 + 1] - wfirst[c0] <= cap_w && first[c1 + 1] - first[c0] <= cap_b) ++c1;
    r.cut.push_back(c0);
    r.mw = std::max(r.mw, wfirst[c1] - wfirst[c0]);
    r.mb = std::max(r.mb, first[c1] - first[c0]);
    c0 = c1;
  }
  r.cut.push_back(n);
  return r;
}
// A scratch set's buffers for batches of up to mw words and mb blocks.
static uint64_t zc_set_words_bytes(uint64_t mw) { return (mw + 1024) * 4; }
static uint64_t zc_set_stage_bytes(uint64_t mw, uint64_t mb) { return mw + 64 * mb + kZcStagePad; }

// The scratch sets for batches of up to mw words and mb blocks (set 1 only
// with two streams); set 0's tmp also holds the call's own scans (tmpb).
static int zc_ensure_sets(mcdc_ctx *ctx, uint64_t mw, uint64_t mb, bool two, size_t tmpb) {
  DevBuf *const sets[2][7] = {{&ctx->zc_blocks, &ctx->zc_stage, &ctx->zc_piece, &ctx->zc_poff, &ctx->zc_tmp,
                               &ctx->zc_words, &ctx->zc_extra},
                              {&ctx->zc_blocks2, &ctx->zc_stage2, &ctx->zc_piece2, &ctx->zc_poff2, &ctx->zc_tmp2,
                               &ctx->zc_words2, &ctx->zc_extra2}};
  const size_t bytes[7] = {mb * sizeof(ZcBlock), zc_set_stage_bytes(mw, mb), (mb + 1) * 8, (mb + 1) * 8,
                           std::max(tmpb, zc_tmp_bytes(mb)), zc_set_words_bytes(mw), mb * kZcExtra};
  for (int k = 0; k < (two ? 2 : 1); ++k)
    for (int b = 0; b < 7; ++b) {
      const int rc = ensure(ctx, *sets[k][b], bytes[b]);
      if (rc) return rc;
    }
  return MCDC_OK;
}

// One compression call's batches enqueued on the context's streams, no host
// wait: chunks [0, nchunks) of dch with their block / word prefixes (first /
// wfirst on the device, hfirst / hwfirst on the host, same base) and the
// k_zc_small classes hcls; frames back to back from d_out (the running offset
// in misc[2], reset here), extents to ext.  The sets must hold zbt's batches
// (zc_ensure_sets); on return ctx->stream is ordered after every batch.
// Timing-free events of a call (compressor batches, save-path groups) from the
// context's pool, returned at the call's end: created once per context, not
// per call (a call used ~18; a later record supersedes any earlier one a
// stream wait already captured).
static hipError_t take_event(mcdc_ctx *ctx, hipEvent_t *e) {
  {
    std::lock_guard<std::mutex> g(ctx->ev_pool_mu);
    if (!ctx->ev_pool.empty()) {
      *e = ctx->ev_pool.back();
      ctx->ev_pool.pop_back();
      return hipSuccess;
    }
  }
  return hipEventCreateWithFlags(e, hipEventDisableTiming);
}
static void give_event(mcdc_ctx *ctx, hipEvent_t e) {
  if (!e) return;
  std::lock_guard<std::mutex> g(ctx->ev_pool_mu);
  ctx->ev_pool.push_back(e);
}

static int zc_enqueue(mcdc_ctx *ctx, const uint8_t *d_data, size_t n, const DevChunk *dch, const uint64_t *first,
                      const uint64_t *wfirst, const uint64_t *hfirst, const uint64_t *hwfirst, const uint8_t *hcls,
                      const ZcBatches &zbt, uint8_t *d_out, uint64_t *ext, uint64_t *misc) {
  static const zs::ZTables T = zs::build_tables();
  hipStream_t st = ctx->stream;
  const bool two = zbt.two;
  const size_t tmpb = ctx->zc_tmp.cap;
  const size_t tmpb2 = ctx->zc_tmp2.cap;
  struct Set {
    DevBuf *blocks, *stage, *piece, *poff, *tmp, *words, *extra;
    size_t tmpb;
  } sets[2] = {{&ctx->zc_blocks, &ctx->zc_stage, &ctx->zc_piece, &ctx->zc_poff, &ctx->zc_tmp, &ctx->zc_words,
                &ctx->zc_extra, tmpb},
               {&ctx->zc_blocks2, &ctx->zc_stage2, &ctx->zc_piece2, &ctx->zc_poff2, &ctx->zc_tmp2, &ctx->zc_words2,
                &ctx->zc_extra2, tmpb2}};
  HIP_TRY(hipMemsetAsync(misc + 2, 0, 8, st));
  // [0] setup done on st; [1 + k] set k's last final copy
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  auto destroy = [&]() {
    for (auto &e : ev) give_event(ctx, e);
  };
  for (auto &e : ev)
    if (take_event(ctx, &e) != hipSuccess)
      return e = nullptr, destroy(), fail(MCDC_E_DEVICE, "event creation failed");
  hipStream_t ss[2] = {st, ctx->stream2};
  if (two) {
    const int rc = hipEventRecord(ev[0], st) == hipSuccess && hipStreamWaitEvent(ss[1], ev[0], 0) == hipSuccess
                       ? MCDC_OK
                       : fail(MCDC_E_DEVICE, "stream ordering failed");
    if (rc) return destroy(), rc;
  }
  int k = 0, prev = -1;  // set of the batch, set of the batch before
  for (size_t bt = 0; bt + 1 < zbt.cut.size(); ++bt, k ^= two ? 1 : 0) {
    const size_t c0 = zbt.cut[bt], c1 = zbt.cut[bt + 1];
    uint64_t nseg = 0, nsmall[4] = {0, 0, 0, 0};  // (chunks of one block per k_zc_small class)
    uint64_t blongest = 0;  // (the batch's longest chunk in blocks: k_zc_far only above one segment)
    for (size_t c = c0; c < c1; ++c) {
      const uint64_t nbk = hfirst[c + 1] - hfirst[c];
      blongest = std::max(blongest, nbk);
      nseg += (nbk + kZcSegBlocks - 1) / kZcSegBlocks;
      if (hcls[c] < 4) ++nsmall[hcls[c]];
    }
    const uint64_t nblk = hfirst[c1] - hfirst[c0];
    const Set &z = sets[k];
    if (nblk > zbt.mb || hwfirst[c1] - hwfirst[c0] > zbt.mw || z.words->cap < zc_set_words_bytes(hwfirst[c1] - hwfirst[c0]) ||
        z.extra->cap < nblk * kZcExtra || z.stage->cap < zc_set_stage_bytes(hwfirst[c1] - hwfirst[c0], nblk))
      return destroy(), fail(MCDC_E_INTERNAL, "compressor batch beyond its scratch set");
    launch_zc_batch(d_data, n, dch, first, wfirst, c0, c1, hfirst[c0], nblk, (ZcBlock *)z.blocks->p,
                    (uint8_t *)z.stage->p, (uint32_t *)z.words->p, (uint8_t *)z.extra->p, T, (uint64_t *)z.piece->p,
                    (uint64_t *)z.poff->p, misc + 2, d_out, ext, z.tmp->p, z.tmpb, ss[k], ctx->knobs.zc_huf,
                    two && prev >= 0 && prev != k ? ev[1 + prev] : nullptr, two ? ev[1 + k] : nullptr,
                    blongest > kZcSegBlocks, nseg, ctx->knobs.zc_small ? nsmall : nullptr);
    if (hipGetLastError() != hipSuccess) return destroy(), fail(MCDC_E_DEVICE, "compress launch failed");
    prev = k;
  }
  if (two && prev == 1 && hipStreamWaitEvent(st, ev[2], 0) != hipSuccess)
    return destroy(), fail(MCDC_E_DEVICE, "stream ordering failed");
  destroy();
  return MCDC_OK;
}

// The Archiver's save path for a run of files (processor.rs:138-205 +
// Repository::save_blob, repository_v1.rs:155-195), composed from the stages
// above: size gate, chunking (GPU), chunk IDs (GPU), dedup (GPU index),
// SecureStorage::encode (zstd on host threads or on the GPU, sealing on the
// GPU), packer.
static constexpr uint64_t kMinChunkSize = 512 * 1024;  // global::defaults::MIN_CHUNK_SIZE (defaults.rs:35)

// GPU encode (store->gpu_compress): the stored blobs of the device copy d are
// compressed and sealed in HBM straight into the packs' layout, hashed there,
// and copied out pack by pack while the next blobs compress.
//   * Groups of blobs (in storing order, 1 GiB of 32 KiB blocks or the
//     compressor's batch, the larger; the last ones halving) are compressed
//     by zc_enqueue one after the other on the compressor's streams, every
//     input uploaded once, so the next group's batches queue before the host
//     waits for a group: no gap between groups.  After a group, its
//     blobs' encoded sizes are known (frame + kAeadOverhead), so the packer's
//     flush rule (Packer::add_blob / flush, packer.rs:101-186,
//     repository_v1.rs:185-193) places every blob of the group: a blob's pack
//     starts where the packs before it end, and a pack's header follows its
//     body.
//   * Headers (generate_header: 37-byte entries padded to a multiple of 64)
//     are SecureStorage-encoded with their zstd frame holding raw blocks
//     (decode-equal: mapache's decoder reads any frame; ~10 % larger than
//     level 3 on IDs, which are random bytes -- 0.1 % of the packs), so a
//     header's encoded size follows from its entry count and the layout is
//     fixed before anything is sealed.
//   * The group's blobs and the headers of the packs it closes are sealed by
//     aead_run into their places in sv_pack, the trailers (le32 of the
//     encoded header's length) copied beside them; then the closed packs
//     cross PCIe on stream3 while the next group compresses (the D2H was ~7
//     ms after everything else for the kernel-tree stand-in).
//   * The pack IDs (BLAKE3 of each pack) over sv_pack at the end.
// A too small packs_out / packs capacity is found as the packs close: no
// further copy is issued, the sizes are still computed, and MCDC_E_CAPACITY
// returns with the totals.

static int save_encode_gpu(mcdc_ctx *ctx, const mcdc_store *store, const uint8_t *d, size_t n,
                           const std::vector<mcdc_blob> &sext, const std::vector<uint8_t> &sids,
                           const std::vector<uint8_t> &types, void *packs_out, size_t packs_out_cap,
                           size_t *packs_bytes, mcdc_pack *packs, size_t packs_cap, size_t *npacks) {
  const size_t m = sext.size();
  const bool keyed = store->key != nullptr;
  const uint64_t over = keyed ? kAeadOverhead : 0;
  std::vector<mcdc_chunk> sch(m);
  uint64_t bound = 0;  // (the raw frames k_zc_nblocks reports, from the lengths)
  for (size_t k = 0; k < m; ++k) {
    sch[k] = mcdc_chunk{sext[k].offset, sext[k].length, 0};
    const uint64_t len = sext[k].length, nb = len ? (len + kZcBlock - 1) / kZcBlock : 1;
    bound += zs::kFrameHdr + zs::kBlockHdr * nb + len;
  }
  for (size_t k = 0; k < m; ++k)
    if (sext[k].length + over + zs::kFrameHdr + 3 * (sext[k].length / kZcBlock + 1) > 0xffffffffull)
      return fail(MCDC_E_INVALID, "blob %zu exceeds the header's u32 length", k);
  // the packs' bound: every blob at its raw frame, every header entry (padding
  // included: fewer than 64 per pack) raw-framed and sealed, the trailers
  const uint64_t mps = std::max<uint64_t>(store->max_pack_size, 1);
  const uint64_t np_max = (bound + over * m) / mps + 2;
  const uint64_t pack_bound = bound + over * m + (m + 64 * np_max) * kHeaderEntry +
                              np_max * (zs::kFrameHdr + over + 4 + 3 * ((m * kHeaderEntry) / (128 << 10) + 2));
  // sv_comp: every group's frames, each followed by the framed headers of the
  // packs it closes
  const uint64_t comp_cap = pack_bound + 64;
  int rc = MCDC_OK;
  if ((rc = ensure(ctx, ctx->sv_comp, comp_cap)) || (rc = ensure(ctx, ctx->sv_pack, std::max<uint64_t>(pack_bound, 1))))
    return rc;
  uint8_t *C = (uint8_t *)ctx->sv_comp.p, *D = (uint8_t *)ctx->sv_pack.p;
  std::vector<mcdc_blob> fr(m);   // frames, offsets from their group's start in C
  std::vector<uint64_t> lens(m);  // encoded sizes
  std::vector<uint64_t> place(m); // blob k at D + place[k]
  // the packs: first blob of each (+ m), extents, header sizes
  std::vector<size_t> first;
  std::vector<mcdc_chunk> pk;
  std::vector<uint64_t> meta;  // encoded header + 4
  uint64_t at = 0, body = 0;   // the open pack's start in D, its body so far
  bool open = false, overflow = false;
  size_t pad_used = 0, copied = 0;  // padding entries drawn; packs handed to stream3
  std::vector<uint8_t> hbuf;        // host: raw-framed headers of the packs closing in a group
  std::vector<hipEvent_t> evs;
  auto cleanup = [&]() {  // (every exit: nothing queued may still write the caller's buffer)
    (void)hipStreamSynchronize(ctx->stream4);
    (void)hipStreamSynchronize(ctx->stream3);
    (void)hipStreamSynchronize(ctx->stream);
    for (hipEvent_t e : evs) give_event(ctx, e);
  };
  // a header's raw zstd frame: frame header, then raw blocks of <= 128 KiB
  auto frame_len = [](uint64_t hl) {
    const uint64_t nb = hl ? (hl + (128 << 10) - 1) / (128 << 10) : 1;
    return zs::kFrameHdr + zs::kBlockHdr * nb + hl;
  };
  // close pack [first.back(), e): its extent, header, its place in D
  struct Closing {
    size_t k;
    uint64_t hpos, hlen;  // the header's frame at hbuf[hpos, + hlen)
  };
  std::vector<Closing> closing;
  auto close_pack = [&](size_t e) -> int {
    const size_t k = pk.size(), b0 = first.back(), cnt = e - b0;
    const size_t pad = cnt % kHeaderMultiple ? kHeaderMultiple - cnt % kHeaderMultiple : 0;
    if (pad_used + pad > store->npadding)
      return fail(MCDC_E_INVALID, "the padding pool holds %zu entries, the headers need more", store->npadding);
    if (keyed && k >= store->nheader_nonces)
      return fail(MCDC_E_INVALID, "more packs than the %zu header nonces given", store->nheader_nonces);
    const uint64_t hl = (cnt + pad) * kHeaderEntry, fl = frame_len(hl);
    const uint64_t hpos = hbuf.size();
    hbuf.resize(hpos + fl);
    uint8_t *h = hbuf.data() + hpos;
    zs::put_frame_header(h);
    uint64_t o = zs::kFrameHdr, left = hl;
    std::vector<uint8_t> hdr(hl);  // generate_header (packer.rs:113-150)
    uint8_t *q = hdr.data();
    for (size_t i = b0; i < e; ++i, q += kHeaderEntry) {
      const uint32_t len = (uint32_t)lens[i];
      std::memcpy(q, sids.data() + 32 * i, 32);
      std::memcpy(q + 32, &len, 4);
      q[36] = types[i];
    }
    for (size_t j = 0; j < pad; ++j, ++pad_used, q += kHeaderEntry) {
      std::memcpy(q, store->padding + 36 * pad_used, 36);
      q[36] = 0xff;
    }
    const uint8_t *src = hdr.data();
    do {
      const uint32_t bs = (uint32_t)std::min<uint64_t>(left, 128 << 10);
      zs::put_block_header(h + o, left == bs, 0, bs);
      std::memcpy(h + o + zs::kBlockHdr, src, bs);
      o += zs::kBlockHdr + bs, src += bs, left -= bs;
    } while (left);
    const uint64_t enc = fl + over;
    (void)e;
    pk.push_back(mcdc_chunk{at, body + enc + 4, 0});
    meta.push_back(enc + 4);
    closing.push_back(Closing{k, hpos, fl});
    at += body + enc + 4;
    body = 0;
    open = false;
    return MCDC_OK;
  };
  hipStream_t st = ctx->stream, s3 = ctx->stream3, s4 = ctx->stream4;
  // Groups of at least 1 GiB of blocks, the last ones halving: a group's
  // seals and pack copies (stream3, about half its compression time) hide
  // behind the next group's compression, and only the last, small group's
  // are left after the compressor finishes.
  const uint64_t group_blocks =
      ctx->knobs.save_group_blocks ? ctx->knobs.save_group_blocks : std::max<uint64_t>(ctx->knobs.zc_batch, 32768);
  constexpr uint64_t kTailBlocks = 8192;  // (the halving stops here: a seal call has ~0.3 ms of fixed latency)
  uint64_t left = 0;
  for (size_t k = 0; k < m; ++k) left += sext[k].length ? (sext[k].length + kZcBlock - 1) / kZcBlock : 1;
  // the groups, and what their seals need at most: the AEAD workspace is
  // reserved here (ensure() would wait for every stream mid-pipeline), the
  // seals' records and the headers staged in one pinned buffer, a region per
  // group (nothing the queued copies read is overwritten within the call)
  SAVE_T("gpu: buffers");
  std::vector<size_t> gstart;
  size_t gmax = 0;
  uint64_t tmax = 0;
  for (size_t g0 = 0; g0 < m;) {
    size_t g1 = g0;
    uint64_t gblk = 0, gt = 0;
    const uint64_t target = left > 2 * group_blocks ? group_blocks
                            : left > 2 * kTailBlocks ? std::max<uint64_t>(left / 2, kTailBlocks)
                                                     : left;
    while (g1 < m && gblk < target) {
      const uint64_t len = sext[g1].length, nb = len ? (len + kZcBlock - 1) / kZcBlock : 1;
      gblk += nb;
      gt += seal_tiles(zs::kFrameHdr + zs::kBlockHdr * nb + len);  // (the raw frame: the longest encoding)
      ++g1;
    }
    gstart.push_back(g0);
    gmax = std::max(gmax, g1 - g0);
    tmax = std::max(tmax, gt);
    left -= std::min(left, gblk);
    g0 = g1;
  }
  gstart.push_back(m);
  const size_t G = gstart.size() - 1;
  const uint64_t hdr_bound = pack_bound - bound - over * m;  // (the headers' and trailers' share)
  const uint64_t hmax = np_max + 1;                           // (headers per seal, at most)
  uint64_t htiles = 0;
  {
    const uint64_t per = (hdr_bound + hmax - 1) / hmax;
    htiles = hmax * seal_tiles(per + 1) + seal_tiles(hdr_bound);
  }
  const size_t stage_bytes =
      seal_stage_bytes(m) + G * (seal_stage_bytes(hmax) + 256) + hdr_bound + 8 * hmax + 16 * m + 4096;
  if ((keyed && (rc = seal_workspace(ctx, gmax + hmax, tmax + htiles))) ||
      (rc = ensure_pinned(ctx, ctx->h_meta, ctx->h_meta_cap, stage_bytes)))
    return cleanup(), rc;
  SAVE_T("gpu: groups");
  uint8_t *const hstage = (uint8_t *)ctx->h_meta;
  size_t hcur = 0;
  auto take = [&](size_t bytes) {  // a region of the pinned staging, 64-byte aligned
    uint8_t *p = hstage + hcur;
    hcur += (bytes + 63) / 64 * 64;
    return hcur <= stage_bytes ? p : nullptr;
  };
  // The compressor's input for every group, uploaded once (no upload or host
  // wait between groups): the blobs, their block / word prefixes and classes
  // on the host and in HBM, each group's batches, the scratch sets for the
  // largest; group g's frames at C + cstart[g] (its raw bound reserved), the
  // headers after all of them (at C + bound).
  std::vector<uint64_t> zpre(2 * (m + 1), 0);
  std::vector<uint8_t> zcls(m);
  uint64_t *const zfirst = zpre.data(), *const zwfirst = zpre.data() + m + 1;
  for (size_t k = 0; k < m; ++k) {
    const uint64_t len = sext[k].length, nb = len ? (len + kZcBlock - 1) / kZcBlock : 1;
    zfirst[k + 1] = zfirst[k] + nb;
    zwfirst[k + 1] = zwfirst[k] + zc_span(len);
    zcls[k] = nb == 1 ? (uint8_t)zc_small_class(len) : (uint8_t)4;
  }
  std::vector<ZcBatches> zbs(G);
  std::vector<uint64_t> cstart(G + 1, 0);
  uint64_t zmw = 0, zmb = 0;
  bool ztwo = false;
  for (size_t g = 0; g < G; ++g) {
    const size_t g0 = gstart[g], g1 = gstart[g + 1];
    zbs[g] = zc_batches(zfirst + g0, zwfirst + g0, g1 - g0, ctx->knobs);
    zmw = std::max(zmw, zbs[g].mw), zmb = std::max(zmb, zbs[g].mb), ztwo |= zbs[g].two;
    uint64_t gb = 0;
    for (size_t k = g0; k < g1; ++k)
      gb += zs::kFrameHdr + zs::kBlockHdr * (zfirst[k + 1] - zfirst[k]) + sext[k].length;
    cstart[g + 1] = cstart[g] + gb;
  }
  SAVE_T("gpu: batches");
  if ((rc = stage_arg(ctx, ctx->sv_zch, sch.data(), m * sizeof(mcdc_chunk))) ||
      (rc = stage_arg(ctx, ctx->sv_zpre, zpre.data(), zpre.size() * 8)) || (rc = ensure(ctx, ctx->sv_zext, 16 * m)) ||
      (rc = ensure(ctx, ctx->zc_misc, 32)) || (rc = zc_ensure_sets(ctx, zmw, zmb, ztwo, 0)))
    return cleanup(), rc;
  HIP_TRY(hipStreamSynchronize(st));  // (the uploads read pageable host memory)
  SAVE_T("gpu: uploads");
  const DevChunk *zch = (const DevChunk *)ctx->sv_zch.p;
  const uint64_t *dzfirst = (const uint64_t *)ctx->sv_zpre.p, *dzwfirst = dzfirst + m + 1;
  uint64_t *const zext = (uint64_t *)ctx->sv_zext.p, *const zmisc = (uint64_t *)ctx->zc_misc.p;
  uint64_t *const hext = (uint64_t *)take(16 * m);
  if (!hext) return cleanup(), fail(MCDC_E_INTERNAL, "save path: frame staging full");
  std::vector<hipEvent_t> evg(G, nullptr);  // group g's frames and extents complete (on st)
  hipEvent_t ev_s3 = nullptr, ev_cp = nullptr;
  for (auto &e : evg) {
    if (take_event(ctx, &e) != hipSuccess)
      return e = nullptr, cleanup(), fail(MCDC_E_DEVICE, "event creation failed");
    evs.push_back(e);
  }
  if (take_event(ctx, &ev_s3) != hipSuccess) return cleanup(), fail(MCDC_E_DEVICE, "event creation failed");
  evs.push_back(ev_s3);
  if (take_event(ctx, &ev_cp) != hipSuccess) return cleanup(), fail(MCDC_E_DEVICE, "event creation failed");
  evs.push_back(ev_cp);
  auto enqueue = [&](size_t g) -> int {  // group g's compression, then its extents to the host
    const size_t g0 = gstart[g], gm = gstart[g + 1] - g0;
    int r = zc_enqueue(ctx, d, n, zch + g0, dzfirst + g0, dzwfirst + g0, zfirst + g0, zwfirst + g0, zcls.data() + g0,
                       zbs[g], C + cstart[g], zext + 2 * g0, zmisc);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(hext + 2 * g0, zext + 2 * g0, 16 * gm, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(evg[g], st));
    return MCDC_OK;
  };
  uint64_t hoff = 0;  // the headers' running offset after the frames (C + bound)
  if (G && (rc = enqueue(0))) return cleanup(), rc;
  for (size_t g = 0; g < G; ++g) {  // compress a group; its seals, headers and closed packs on stream3
    const size_t g0 = gstart[g], g1 = gstart[g + 1], gm = g1 - g0;
    // the next group's batches queue behind this one's on the compressor's
    // streams before the host waits: no gap between groups
    if (g + 1 < G && (rc = enqueue(g + 1))) return cleanup(), rc;
    HIP_TRY(hipEventSynchronize(evg[g]));
    for (size_t i = g0; i < g1; ++i) fr[i] = mcdc_blob{hext[2 * i], hext[2 * i + 1]};
    SAVE_T("group compressed");
    HIP_TRY(hipStreamWaitEvent(s3, evg[g], 0));
    // place the group's blobs; close the packs the flush rule closes
    closing.clear();
    hbuf.clear();
    for (size_t i = g0; i < g1; ++i) {
      lens[i] = fr[i].length + over;
      if (!open) first.push_back(i), open = true;
      place[i] = at + body;
      body += lens[i];
      if (body > mps && (rc = close_pack(i + 1))) return cleanup(), rc;
    }
    if (g1 == m && open && (rc = close_pack(m))) return cleanup(), rc;
    // headers of the closing packs, framed on the host, to HBM after every group's frames
    const uint64_t hin = bound + hoff;
    if (hin + hbuf.size() > comp_cap)  // (frames within their raw bound, headers within pack_bound's share)
      return cleanup(), fail(MCDC_E_INTERNAL, "save path: header staging beyond the compressor buffer");
    uint8_t *hm = hbuf.empty() ? nullptr : take(hbuf.size()), *tr = closing.empty() ? nullptr : take(4 * closing.size());
    if ((!hbuf.empty() && !hm) || (!closing.empty() && !tr))
      return cleanup(), fail(MCDC_E_INTERNAL, "save path: header staging full");
    if (hm) {
      std::memcpy(hm, hbuf.data(), hbuf.size());
      HIP_TRY(hipMemcpyAsync(C + hin, hm, hbuf.size(), hipMemcpyHostToDevice, s3));
    }
    for (size_t c = 0; c < closing.size(); ++c) {  // trailers: le32(encoded header length)
      const uint32_t el = (uint32_t)(meta[closing[c].k] - 4);
      std::memcpy(tr + 4 * c, &el, 4);
    }
    if (keyed) {  // the group's blobs and the closing packs' headers: one seal into their places
      const size_t nc = closing.size(), ns = gm + nc;
      std::vector<mcdc_blob> sx(ns);
      std::vector<uint64_t> pl(ns + 1);
      std::vector<uint8_t> sn(12 * ns);
      uint64_t end = 0;
      for (size_t i = 0; i < gm; ++i) {
        sx[i] = fr[g0 + i];
        pl[i] = place[g0 + i];
        end = std::max(end, place[g0 + i] + lens[g0 + i]);
      }
      std::memcpy(sn.data(), store->nonces + 12 * g0, 12 * gm);
      for (size_t c = 0; c < nc; ++c) {  // (header frames at C + hin: offsets from the group's frames)
        const size_t k = closing[c].k;
        sx[gm + c] = mcdc_blob{hin - cstart[g] + closing[c].hpos, closing[c].hlen};
        pl[gm + c] = pk[k].offset + pk[k].length - meta[k];
        end = std::max(end, pl[gm + c] + closing[c].hlen + over);
        std::memcpy(sn.data() + 12 * (gm + c), store->header_nonces + 12 * k, 12);
      }
      pl[ns] = end;
      uint8_t *sst = take(seal_stage_bytes(ns));
      if (!sst) return cleanup(), fail(MCDC_E_INTERNAL, "save path: seal staging full");
      if ((rc = seal_placed(ctx, s3, store->key, C + cstart[g], sx.data(), ns, sn.data(), D, pl.data(), sst)))
        return cleanup(), rc;
    } else {  // frames as they are: the group's frames run by run of one pack, the headers
      for (size_t i = g0; i < g1;) {
        size_t e = i + 1;
        while (e < g1 && place[e] == place[e - 1] + lens[e - 1]) ++e;
        HIP_TRY(hipMemcpyAsync(D + place[i], C + cstart[g] + fr[i].offset, place[e - 1] + lens[e - 1] - place[i],
                               hipMemcpyDeviceToDevice, s3));
        i = e;
      }
      for (const Closing &c : closing)
        HIP_TRY(hipMemcpyAsync(D + pk[c.k].offset + pk[c.k].length - meta[c.k], C + hin + c.hpos, c.hlen,
                               hipMemcpyDeviceToDevice, s3));
    }
    for (size_t c = 0; c < closing.size(); ++c) {
      const size_t k = closing[c].k;
      HIP_TRY(hipMemcpyAsync(D + pk[k].offset + pk[k].length - 4, tr + 4 * c, 4, hipMemcpyHostToDevice, s3));
    }
    // the closed packs to the host on stream4, behind their seals and
    // trailers (stream3): the next group's seals do not wait for the copy
    if (!closing.empty()) {
      const size_t k1 = pk.size();
      overflow |= k1 > packs_cap || (packs_out == nullptr) ||
                  pk[k1 - 1].offset + pk[k1 - 1].length > packs_out_cap;
      if (!overflow) {
        const uint64_t lo = pk[copied].offset, hi = pk[k1 - 1].offset + pk[k1 - 1].length;
        HIP_TRY(hipEventRecord(ev_cp, s3));
        HIP_TRY(hipStreamWaitEvent(s4, ev_cp, 0));
        HIP_TRY(hipMemcpyAsync((uint8_t *)packs_out + lo, D + lo, hi - lo, hipMemcpyDeviceToHost, s4));
        copied = k1;
      }
    }
    hoff += hbuf.size();
  }
  // the pack IDs (on st) after the last seals and copies into D (stream3),
  // beside the last packs' copy to the host (stream4)
  HIP_TRY(hipEventRecord(ev_s3, s3));
  HIP_TRY(hipStreamWaitEvent(st, ev_s3, 0));
  const size_t np = pk.size();
  first.push_back(m);
  *npacks = np;
  if (packs_bytes) *packs_bytes = at;
  if (np > packs_cap || (np && !packs)) {
    HIP_TRY(hipStreamSynchronize(s3));
    HIP_TRY(hipStreamSynchronize(st));
    return cleanup(), fail(MCDC_E_CAPACITY, "%zu packs, capacity %zu", np, packs_cap);
  }
  if (overflow || at > packs_out_cap) {
    HIP_TRY(hipStreamSynchronize(s3));
    HIP_TRY(hipStreamSynchronize(st));
    return cleanup(), fail(MCDC_E_CAPACITY, "output capacity %zu < %llu bytes", packs_out_cap,
                           (unsigned long long)at);
  }
  SAVE_T("sealed enqueued");
  std::vector<uint8_t> pid(32 * np);
  rc = np ? mcdc_chunk_ids_device(ctx, D, at, pk.data(), np, pid.data()) : MCDC_OK;
  HIP_TRY(hipStreamSynchronize(s4));
  HIP_TRY(hipStreamSynchronize(s3));
  HIP_TRY(hipStreamSynchronize(st));
  cleanup();
  if (rc) return rc;
  SAVE_T("packs out");
  for (size_t k = 0; k < np; ++k) {
    packs[k].offset = pk[k].offset;
    packs[k].length = pk[k].length;
    packs[k].nblobs = first[k + 1] - first[k];
    packs[k].meta_size = meta[k];
    std::memcpy(packs[k].id, pid.data() + 32 * k, 32);
  }
  return MCDC_OK;
}

// Host encode (the crate's exact bytes): zstd level 3 / window 20 on host
// threads, the seal on the GPU (mcdc_encode_blobs), packs on the host.
static int save_encode_host(mcdc_ctx *ctx, const mcdc_store *store, const void *data, const uint8_t *d, size_t n,
                            bool host_in, std::vector<mcdc_blob> sext, const std::vector<uint8_t> &sids,
                            const std::vector<uint8_t> &types, void *packs_out, size_t packs_out_cap,
                            size_t *packs_bytes, mcdc_pack *packs, size_t packs_cap, size_t *npacks) {
  const size_t m = sext.size();
  const uint8_t *src = (const uint8_t *)data;
  size_t src_n = n;
  if (!host_in && m) {
    // device input: the new blobs gathered in HBM (one kernel), then one D2H
    // into the context's pinned staging (the zstd stage runs on the host).
    // One copy per blob cost ~15 us each: 1.1 s of the kernel-tree
    // stand-in's 72 167 blobs.
    std::vector<uint64_t> gx(3 * m);
    size_t tot = 0;
    for (size_t k = 0; k < m; ++k) {
      tot += ((uintptr_t)d + sext[k].offset - tot) & 15;  // (congruent to the source modulo 16; HBM buffers 256-aligned)
      gx[3 * k] = sext[k].offset;
      gx[3 * k + 1] = tot;
      gx[3 * k + 2] = sext[k].length;
      sext[k].offset = tot;
      tot += sext[k].length;
    }
    int rc0 = MCDC_OK;
    if ((rc0 = ensure(ctx, ctx->sv_comp, std::max<size_t>(tot, 1))) ||
        (rc0 = stage_arg(ctx, ctx->sv_ext, gx.data(), gx.size() * 8)) || (rc0 = ensure_hsave(ctx, tot)))
      return rc0;
    launch_gather(d, (const uint64_t *)ctx->sv_ext.p, m, (uint8_t *)ctx->sv_comp.p, ctx->stream);
    HIP_TRY(hipGetLastError());
    if (tot) HIP_TRY(hipMemcpyAsync(ctx->h_save, ctx->sv_comp.p, tot, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    src = (const uint8_t *)ctx->h_save;
    src_n = tot;
  }
  size_t ecap = 0;
  for (auto &e : sext) ecap += e.length + e.length / 64 + 64;
  // (the encoded blobs in a buffer the context keeps: a fresh multi-GB vector
  // per call was zero-filled and page-faulted)
  auto enc_buf = [&](size_t bytes) -> uint8_t * {  // (pinned: the sealed blobs' D2H runs at the DMA rate)
    return ensure_pinned(ctx, ctx->h_encb, ctx->h_encb_cap, bytes) == MCDC_OK ? (uint8_t *)ctx->h_encb : nullptr;
  };
  uint8_t *enc = enc_buf(std::max<size_t>(ecap, 1));
  if (!enc) return fail(MCDC_E_NOMEM, "host allocation of %zu bytes failed", ecap);
  std::vector<uint64_t> eo(m + 1, 0);
  int rc = MCDC_OK;
  if (m) {
    rc = mcdc_encode_blobs(ctx, store->key, src, src_n, sext.data(), m, store->nonces, enc, ecap, eo.data());
    if (rc == MCDC_E_CAPACITY) {
      ecap = std::max<uint64_t>(eo[m], 1);
      if (!(enc = enc_buf(ecap))) return fail(MCDC_E_NOMEM, "host allocation of %zu bytes failed", ecap);
      rc = mcdc_encode_blobs(ctx, store->key, src, src_n, sext.data(), m, store->nonces, enc, ecap, eo.data());
    }
    if (rc) return rc;
  }
  std::vector<mcdc_blob> eext(m);
  for (size_t k = 0; k < m; ++k) eext[k] = mcdc_blob{eo[k], eo[k + 1] - eo[k]};
  size_t pb = 0;
  rc = mcdc_pack_blobs(ctx, store->key, enc, eo[m], eext.data(), sids.data(), types.data(), m,
                       store->max_pack_size, store->header_nonces, store->nheader_nonces, store->padding,
                       store->npadding, packs_out, packs_out_cap, &pb, packs, packs_cap, npacks);
  if (packs_bytes) *packs_bytes = pb;
  return rc;
}

int mcdc_save_files(mcdc_ctx *ctx, const mcdc_params *params, mcdc_index *ix, const mcdc_store *store,
                    const void *data, size_t n, const mcdc_blob *files, size_t nfiles, uint64_t *file_blobs,
                    uint8_t *ids, uint8_t *is_new, size_t blobs_cap, size_t *nblobs, void *packs_out,
                    size_t packs_out_cap, size_t *packs_bytes, mcdc_pack *packs, size_t packs_cap, size_t *npacks) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!params || !ix || !store || (!data && n) || (nfiles && (!files || !file_blobs)) || !nblobs || !npacks)
    return fail(MCDC_E_INVALID, "NULL argument");
  if ((rc = mcdc_params_check(params, nullptr, nullptr))) return rc;
  if (ix->device != ctx->device) return fail(MCDC_E_INVALID, "the index lives on device %d", ix->device);
  if ((rc = check_extents(files, nfiles, n))) return rc;
  if ((ids && is_device_ptr(ids)) || (is_new && is_device_ptr(is_new)) || (packs_out && is_device_ptr(packs_out)))
    return fail(MCDC_E_INVALID, "ids / is_new / packs_out must be host memory");
  *nblobs = 0;
  *npacks = 0;
  if (packs_bytes) *packs_bytes = 0;
  const double t0 = now_ms();
  t_trace0 = t0;
  const bool host_in = data && !is_device_ptr(data);
  // the bytes in HBM (one copy of a host input)
  const uint8_t *d = (const uint8_t *)data;
  if (host_in && n) {
    if ((rc = ensure(ctx, ctx->sv_in, n))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->sv_in.p, data, n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    d = (const uint8_t *)ctx->sv_in.p;
  }
  // processor::save_file: a file smaller than MIN_CHUNK_SIZE is one blob
  // (:144-153; the constant, whatever the chunker's own min); the others go
  // through the chunker (:160-205)
  const uint64_t gate = store->gate_bytes ? store->gate_bytes : kMinChunkSize;
  std::vector<uint64_t> boff, blen;
  std::vector<size_t> big;
  size_t cap = 0;
  for (size_t f = 0; f < nfiles; ++f)
    if (files[f].length >= gate) {
      big.push_back(f);
      boff.push_back(files[f].offset);
      blen.push_back(files[f].length);
      cap += files[f].length / (params->min_size - 1) + 2;
    }
  std::vector<mcdc_chunk> bch(std::max<size_t>(cap, 1));
  std::vector<size_t> bcnt(std::max<size_t>(big.size(), 1));
  if (!big.empty()) {
    size_t got = 0;
    if ((rc = mcdc_chunk_batch_device(ctx, params, d, boff.data(), blen.data(), big.size(), bch.data(), cap,
                                      bcnt.data(), &got)))
      return rc;
  }
  SAVE_T("chunked");
  // every blob in processing order (file order, chunk order), offsets into d,
  // in the context's pinned list (the IDs' kernels read it by one DMA)
  if ((rc = ensure_pinned(ctx, ctx->h_list, ctx->h_list_cap, (nfiles + cap + 1) * sizeof(mcdc_chunk)))) return rc;
  mcdc_chunk *const list = (mcdc_chunk *)ctx->h_list;
  size_t bi = 0, at = 0, nb = 0;
  for (size_t f = 0; f < nfiles; ++f) {
    file_blobs[f] = nb;
    if (bi < big.size() && big[bi] == f) {
      for (size_t j = 0; j < bcnt[bi]; ++j, ++at)
        list[nb++] = mcdc_chunk{files[f].offset + bch[at].offset, bch[at].length, bch[at].hash};
      ++bi;
    } else {
      list[nb++] = mcdc_chunk{files[f].offset, files[f].length, 0};
    }
  }
  if (nfiles) file_blobs[nfiles] = nb;
  *nblobs = nb;
  if (nb > blobs_cap || (nb && !ids)) return fail(MCDC_E_CAPACITY, "%zu blobs, capacity %zu", nb, blobs_cap);
  SAVE_T("list");
  // ID::from_content of every blob (CalculateID of a small file is the same
  // hash), into HBM: the index reads them there, the caller's array gets one
  // copy (queued before the index's kernels, complete when they are)
  if (nb) {
    if ((rc = ensure(ctx, ctx->sv_ids, nb * 32)) || (rc = mcdc_chunk_ids_device(ctx, d, n, list, nb,
                                                                                  (uint8_t *)ctx->sv_ids.p)))
      return rc;
    HIP_TRY(hipMemcpyAsync(ids, ctx->sv_ids.p, nb * 32, hipMemcpyDeviceToHost, ctx->stream));
  }
  SAVE_T("ids");
  // save_blob's dedup check (:173-180) -- the index changes here.  From here
  // on every failure, whatever returns it (capacity, nonces, a HIP call),
  // leaves through the one rollback below: the previous index buffer is
  // intact until the next add, so the index is exactly as before the call.
  std::vector<uint8_t> nw(std::max<size_t>(nb, 1));
  size_t m = 0;
  if (nb && (rc = mcdc_index_add(ctx, ix, (const uint8_t *)ctx->sv_ids.p, nb, nw.data(), nullptr, nullptr, &m)))
    return rc;
  SAVE_T("index");
  auto rest = [&]() -> int {
    if (store->key && m > store->nnonces)
      return fail(MCDC_E_INVALID, "%zu new blobs need %zu nonces (%zu given)", m, m, store->nnonces);
    std::vector<mcdc_blob> sext(m);
    std::vector<uint8_t> sids(32 * m);
    for (size_t i = 0, k = 0; i < nb; ++i)
      if (nw[i]) {
        sext[k] = mcdc_blob{list[i].offset, list[i].length};
        std::memcpy(sids.data() + 32 * k++, ids + 32 * i, 32);
      }
    const std::vector<uint8_t> types(std::max<size_t>(m, 1), 0);  // BlobType::Data (processor.rs:191)
    SAVE_T("new list");
    if (store->gpu_compress && m)
      return save_encode_gpu(ctx, store, d, n, sext, sids, types, packs_out, packs_out_cap, packs_bytes, packs,
                             packs_cap, npacks);
    return save_encode_host(ctx, store, data, d, n, host_in, std::move(sext), sids, types, packs_out, packs_out_cap,
                            packs_bytes, packs, packs_cap, npacks);
  };
  rc = rest();
  if (rc == MCDC_OK && ctx->knobs.test_fail_after_index)  // test hook (tests/test_gpu_save.py)
    rc = fail(MCDC_E_DEVICE, "injected failure after the index add (option test_fail_after_index)");
  if (rc) {
    if (nb) {  // rollback: the index as before the call
      ix->cur ^= 1;
      ix->size -= m;
    }
    return rc;
  }
  if (is_new) std::memcpy(is_new, nw.data(), nb);
  ctx->timing = mcdc_timing{};
  ctx->timing.bytes = n;
  ctx->timing.chunks = nb;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

// ---------------------------------------------------- zstd compression --
// SecureStorage::compress (storage.rs:74-84) of every chunk on the GPU
// (mcdc_zcomp.hip): one zstd frame per chunk, frames back to back.
int mcdc_zstd_compress_device(mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks, size_t nchunks,
                              void *d_out, size_t out_cap, size_t *out_bytes, mcdc_blob *frames) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!d_data && n) || (nchunks && (!chunks || !frames))) return fail(MCDC_E_INVALID, "NULL argument");
  if ((d_data && !is_device_ptr(d_data)) || (d_out && !is_device_ptr(d_out)))
    return fail(MCDC_E_INVALID, "d_data / d_out must be device pointers");
  if (out_bytes) *out_bytes = 0;
  if (nchunks == 0) return MCDC_OK;
  if (nchunks >= (1ull << 31)) return fail(MCDC_E_TOOBIG, "too many chunks (%zu)", nchunks);
  const double t0 = now_ms();
  hipStream_t st = ctx->stream;
  size_t tmpb = zc_tmp_bytes(nchunks);
  if ((rc = stage_arg(ctx, ctx->b3_chunks, chunks, nchunks * sizeof(mcdc_chunk))) ||
      (rc = ensure(ctx, ctx->zc_cnt, (nchunks + 1) * 8)) || (rc = ensure(ctx, ctx->zc_first, (nchunks + 1) * 8)) ||
      (rc = ensure(ctx, ctx->zc_misc, 32)) || (rc = ensure(ctx, ctx->zc_tmp, tmpb)) ||
      (rc = ensure(ctx, ctx->zc_cls, nchunks + 1)) || (rc = ensure(ctx, ctx->zc_wcnt, (nchunks + 1) * 8)) ||
      (rc = ensure(ctx, ctx->zc_wfirst, (nchunks + 1) * 8)))
    return rc;
  uint64_t *misc = (uint64_t *)ctx->zc_misc.p;  // [0] err, [1] raw bound, [2] output base
  HIP_TRY(hipMemsetAsync(misc, 0, 32, st));
  HIP_TRY(hipEventRecord(ctx->ev_start, st));
  const DevChunk *dch = (const DevChunk *)ctx->b3_chunks.p;
  uint64_t *first = (uint64_t *)ctx->zc_first.p, *wfirst = (uint64_t *)ctx->zc_wfirst.p;
  launch_zc_nblocks(dch, nchunks, n, (uint64_t *)ctx->zc_cnt.p, first, (uint64_t *)ctx->zc_wcnt.p, wfirst,
                    (uint32_t *)misc, misc + 1, (uint8_t *)ctx->zc_cls.p, ctx->zc_tmp.p, tmpb, st);
  HIP_TRY(hipGetLastError());
  std::vector<uint64_t> hfirst(nchunks + 1), hwfirst(nchunks + 1);
  std::vector<uint8_t> hcls(nchunks);  // (the k_zc_small class of each chunk: the list may be device memory)
  uint64_t hm[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(hm, misc, 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hfirst.data(), first, (nchunks + 1) * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hwfirst.data(), wfirst, (nchunks + 1) * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hcls.data(), ctx->zc_cls.p, nchunks, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hm[0]) return fail(MCDC_E_INVALID, "a chunk lies outside the %zu-byte buffer or is 2 GiB or longer", n);
  if (out_bytes) *out_bytes = hm[1];  // the capacity that always suffices (raw frames of 32 KiB blocks)
  if (hm[1] > out_cap || !d_out)
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %llu bytes", out_cap, (unsigned long long)hm[1]);
  uint64_t *ext = (uint64_t *)direct_out(ctx, frames);
  if (!ext && is_device_ptr(frames)) return fail(MCDC_E_INVALID, "frames is a device pointer of another device");
  if (!ext) {
    if ((rc = ensure(ctx, ctx->zf_ext, nchunks * 16))) return rc;
    ext = (uint64_t *)ctx->zf_ext.p;
  }
  const ZcBatches zbt = zc_batches(hfirst.data(), hwfirst.data(), nchunks, ctx->knobs);
  if ((rc = zc_ensure_sets(ctx, zbt.mw, zbt.mb, zbt.two, tmpb)) ||
      (rc = zc_enqueue(ctx, (const uint8_t *)d_data, n, dch, first, wfirst, hfirst.data(), hwfirst.data(), hcls.data(),
                       zbt, (uint8_t *)d_out, ext, misc)))
    return rc;
  HIP_TRY(hipEventRecord(ctx->ev_end, st));
  uint64_t total = 0;
  HIP_TRY(hipMemcpyAsync(&total, misc + 2, 8, hipMemcpyDeviceToHost, st));
  if (ext == ctx->zf_ext.p) HIP_TRY(hipMemcpyAsync(frames, ext, nchunks * 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (out_bytes) *out_bytes = total;
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_end));
  ctx->timing = mcdc_timing{};
  ctx->timing.device_ms = ms;
  ctx->timing.bytes = n;
  ctx->timing.chunks = nchunks;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

int mcdc_zstd_compress_scratch(mcdc_ctx *ctx, const mcdc_chunk *chunks, size_t nchunks, size_t *bytes) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!bytes || (nchunks && !chunks)) return fail(MCDC_E_INVALID, "NULL argument");
  if (is_device_ptr(chunks)) return fail(MCDC_E_INVALID, "chunks must be host memory");
  *bytes = 0;
  if (nchunks == 0) return MCDC_OK;
  std::vector<uint64_t> first(nchunks + 1, 0), wfirst(nchunks + 1, 0);
  for (size_t i = 0; i < nchunks; ++i) {
    const uint64_t len = chunks[i].length, nb = len ? (len + kZcBlock - 1) / kZcBlock : 1;
    first[i + 1] = first[i] + nb;
    wfirst[i + 1] = wfirst[i] + zc_span(len);
  }
  // as mcdc_zstd_compress_device sizes its batch sets
  const ZcBatches zbt = zc_batches(first.data(), wfirst.data(), nchunks, ctx->knobs);
  const bool two = zbt.two;
  const uint64_t mw = zbt.mw, mb = zbt.mb;
  // (every buffer as ensure() allocates it, headroom included; the call's
  // own buffers as mcdc_zstd_compress_device requests them)
  const uint64_t tmpb = std::max(zc_tmp_bytes(nchunks), zc_tmp_bytes(mb));
  const uint64_t set = ensure_bytes(tmpb) + ensure_bytes(mb * sizeof(ZcBlock)) +
                       ensure_bytes(zc_set_stage_bytes(mw, mb)) + 2 * ensure_bytes((mb + 1) * 8) +
                       ensure_bytes(zc_set_words_bytes(mw)) + ensure_bytes(mb * kZcExtra);
  const uint64_t call = ensure_bytes(nchunks * sizeof(mcdc_chunk)) + 4 * ensure_bytes((nchunks + 1) * 8) +
                        ensure_bytes(nchunks + 1) +
                        ensure_bytes(32) + ensure_bytes(nchunks * 16);
  *bytes = (size_t)(set * (two ? 2 : 1) + call);
  return MCDC_OK;
}

// ------------------------------------------------------- zstd raw frames --
int mcdc_zstd_frames_device(mcdc_ctx *ctx, const void *d_data, size_t n, const mcdc_chunk *chunks, size_t nchunks,
                            void *d_out, size_t out_cap, size_t *out_bytes, mcdc_blob *frames) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!d_data && n) || (nchunks && (!chunks || !frames))) return fail(MCDC_E_INVALID, "NULL argument");
  if ((d_data && !is_device_ptr(d_data)) || (d_out && !is_device_ptr(d_out)))
    return fail(MCDC_E_INVALID, "d_data / d_out must be device pointers");
  // k_zframe_write stores whole 16-byte quads at d_out + off[i]
  if ((uintptr_t)d_out & 15) return fail(MCDC_E_INVALID, "d_out must be 16-byte aligned");
  if (out_bytes) *out_bytes = 0;
  if (nchunks == 0) return MCDC_OK;
  if (nchunks >= (1ull << 31)) return fail(MCDC_E_TOOBIG, "too many chunks (%zu)", nchunks);
  const double t0 = now_ms();
  hipStream_t st = ctx->stream;
  const size_t tmpb = zframe_tmp_bytes(nchunks);
  if ((rc = stage_arg(ctx, ctx->b3_chunks, chunks, nchunks * sizeof(mcdc_chunk))) ||
      (rc = ensure(ctx, ctx->zf_sz, (nchunks + 1) * 8)) || (rc = ensure(ctx, ctx->zf_off, (nchunks + 1) * 8)) ||
      (rc = ensure(ctx, ctx->zf_tmp, tmpb)) || (rc = ensure(ctx, ctx->err, 32)))
    return rc;
  uint32_t *err = (uint32_t *)ctx->err.p + 6;
  HIP_TRY(hipMemsetAsync(err, 0, 4, st));
  HIP_TRY(hipEventRecord(ctx->ev_start, st));
  launch_zframe_sizes((const DevChunk *)ctx->b3_chunks.p, nchunks, n, (uint64_t *)ctx->zf_sz.p,
                      (uint64_t *)ctx->zf_off.p, err, ctx->zf_tmp.p, tmpb, st);
  HIP_TRY(hipGetLastError());
  uint32_t herr = 0;
  uint64_t total = 0;
  HIP_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&total, (uint64_t *)ctx->zf_off.p + nchunks, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (herr) return fail(MCDC_E_INVALID, "a chunk lies outside the %zu-byte buffer", n);
  if (out_bytes) *out_bytes = total;
  if (total > out_cap || !d_out) return fail(MCDC_E_CAPACITY, "output capacity %zu < %llu bytes", out_cap,
                                             (unsigned long long)total);
  uint64_t *ext = (uint64_t *)direct_out(ctx, frames);
  if (!ext && is_device_ptr(frames)) return fail(MCDC_E_INVALID, "frames is a device pointer of another device");
  if (!ext) {
    if ((rc = ensure(ctx, ctx->zf_ext, nchunks * 16))) return rc;
    ext = (uint64_t *)ctx->zf_ext.p;
  }
  launch_zframe_write((const uint8_t *)d_data, (const DevChunk *)ctx->b3_chunks.p, nchunks,
                      (const uint64_t *)ctx->zf_off.p, (uint8_t *)d_out, ext, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev_end, st));
  if (ext == ctx->zf_ext.p) HIP_TRY(hipMemcpyAsync(frames, ext, nchunks * 16, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_end));
  ctx->timing = mcdc_timing{};
  ctx->timing.device_ms = ms;
  ctx->timing.bytes = n;
  ctx->timing.chunks = nchunks;
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

// --------------------------------------------------------------- packer --
// Packer::add_blob / flush for a run of encoded blobs in host memory
// (plan_packs), packs assembled on the host, pack IDs (BLAKE3 of each pack)
// by mcdc_chunk_ids_device.
int mcdc_pack_blobs(mcdc_ctx *ctx, const uint8_t key[32], const void *h_blobs, size_t n_in, const mcdc_blob *blobs,
                    const uint8_t *ids, const uint8_t *types, size_t nblobs, uint64_t max_pack_size,
                    const uint8_t *header_nonces, size_t nnonces, const uint8_t *padding, size_t npadding,
                    void *h_out, size_t out_cap, size_t *out_bytes, mcdc_pack *packs, size_t packs_cap,
                    size_t *npacks) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((!h_blobs && n_in) || (nblobs && (!blobs || !ids || !types)) || !npacks)
    return fail(MCDC_E_INVALID, "NULL argument");
  if ((h_blobs && is_device_ptr(h_blobs)) || (h_out && is_device_ptr(h_out)))
    return fail(MCDC_E_INVALID, "h_blobs / h_out must be host memory");
  if ((rc = check_extents(blobs, nblobs, n_in))) return rc;
  *npacks = 0;
  if (out_bytes) *out_bytes = 0;
  const double t0 = now_ms();
  std::vector<uint64_t> lens(nblobs);
  for (size_t i = 0; i < nblobs; ++i) lens[i] = blobs[i].length;
  PackPlan P;
  if ((rc = plan_packs(ctx, key, lens.data(), ids, types, nblobs, max_pack_size, header_nonces, nnonces, padding,
                       npadding, P)))
    return rc;
  const size_t np = P.np();
  *npacks = np;
  if (out_bytes) *out_bytes = P.total;
  if (np > packs_cap || (packs_cap && !packs)) return fail(MCDC_E_CAPACITY, "%zu packs, capacity %zu", np, packs_cap);
  if (P.total > out_cap || (P.total && !h_out))
    return fail(MCDC_E_CAPACITY, "output capacity %zu < %zu bytes", out_cap, P.total);
  uint8_t *o = (uint8_t *)h_out;
  mcdc::host::parallel_items(np, zstd_threads(), [&](size_t k, int) {
    uint8_t *d = o + P.pk[k].offset;
    for (size_t i = P.first[k]; i < P.first[k + 1]; ++i) {
      std::memcpy(d, (const uint8_t *)h_blobs + blobs[i].offset, blobs[i].length);
      d += blobs[i].length;
    }
    std::memcpy(d, P.meta.data() + P.moff[k], P.moff[k + 1] - P.moff[k]);
  });
  // pack IDs: BLAKE3 of each pack (flush: utils::calculate_hash(&data)), on the GPU
  std::vector<uint8_t> pid(32 * std::max<size_t>(np, 1));
  if (np) {
    if ((rc = ensure(ctx, ctx->enc_in, P.total))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->enc_in.p, h_out, P.total, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = mcdc_chunk_ids_device(ctx, ctx->enc_in.p, P.total, P.pk.data(), np, pid.data()))) return rc;
  }
  fill_pack_records(P, pid.data(), packs);
  ctx->timing.total_ms = now_ms() - t0;
  return MCDC_OK;
}

// ------------------------------------------------------------ batcher --
// C ABI of the cross-worker batching front-end (mapache_amd/host/batcher.hpp)
// over this library's mcdc_chunk_batch on a context of its own.
}  // extern "C"

struct mcdc_batcher {
  mcdc_ctx *ctx = nullptr;
  mcdc_params params{};
  std::unique_ptr<mcdc::host::Batcher> core;
};

extern "C" {

int mcdc_batcher_create(int device, const mcdc_params *params, size_t max_batch_bytes, size_t max_batch_files,
                        uint32_t gather_us, mcdc_batcher **out) {
  if (!out) return fail(MCDC_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_params(params, nullptr, nullptr);
  if (rc) return rc;
  if (max_batch_bytes == 0 || max_batch_files == 0) return fail(MCDC_E_INVALID, "empty batch limits");
  mcdc_batcher *b = new (std::nothrow) mcdc_batcher();
  if (!b) return fail(MCDC_E_NOMEM, "host allocation failed");
  if ((rc = mcdc_ctx_create(device, max_batch_bytes, &b->ctx))) {
    delete b;
    return rc;
  }
  b->params = *params;
  mcdc_ctx *ctx = b->ctx;
  const mcdc_params P = *params;
  auto fn = [ctx, P](const uint8_t *const *bufs, const size_t *lens, size_t k, mcdc_chunk *o, size_t cap,
                     size_t *counts, size_t *n_out, std::string *msg) {
    const int r = mcdc_chunk_batch(ctx, &P, bufs, lens, k, o, cap, counts, n_out);
    if (r && msg) *msg = mcdc_last_error();
    return r;
  };
  const uint32_t mn = params->min_size;
  b->core.reset(new (std::nothrow) mcdc::host::Batcher(fn, [mn](size_t len) { return len / (mn - 1) + 2; },
                                                       max_batch_bytes, max_batch_files, gather_us));
  if (!b->core) {
    mcdc_ctx_destroy(b->ctx);
    delete b;
    return fail(MCDC_E_NOMEM, "host allocation failed");
  }
  *out = b;
  return MCDC_OK;
}

void mcdc_batcher_destroy(mcdc_batcher *b) {
  if (!b) return;
  b->core.reset();
  mcdc_ctx_destroy(b->ctx);
  delete b;
}

int mcdc_batcher_chunk(mcdc_batcher *b, const void *data, size_t n, mcdc_chunk *out, size_t cap, size_t *n_out) {
  if (!b) return fail(MCDC_E_INVALID, "batcher is NULL");
  std::string msg;
  const int rc = b->core->chunk((const uint8_t *)data, n, out, cap, n_out, &msg);
  if (rc) return fail(rc, "%s", msg.c_str());
  return MCDC_OK;
}

int mcdc_batcher_stats(const mcdc_batcher *b, mcdc_batcher_counters *out) {
  if (!b || !out) return fail(MCDC_E_INVALID, "NULL argument");
  const mcdc::host::BatcherStats s = b->core->stats();
  out->batches = s.batches;
  out->files = s.files;
  out->bytes = s.bytes;
  out->max_batch_files = s.max_batch_files;
  return MCDC_OK;
}

int mcdc_memcpy_d2h(mcdc_ctx *ctx, void *h_dst, const void *d_src, size_t bytes) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MCDC_OK;
}

int mcdc_fill_random_device(mcdc_ctx *ctx, void *d_dst, uint64_t pos, size_t n, uint64_t seed) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!d_dst && n) return fail(MCDC_E_INVALID, "d_dst is NULL");
  launch_fill_random(d_dst, pos, n, seed, ctx->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return MCDC_OK;
}

static uint64_t mix64h(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

uint64_t mcdc_digest(const mcdc_chunk *chunks, size_t n) {
  uint64_t d = 0;
  for (size_t i = 0; i < n; ++i) {
    d = mix64h(d ^ (chunks[i].offset + 0x9e3779b97f4a7c15ull + (d << 6) + (d >> 2)));
    d = mix64h(d ^ (chunks[i].length + 0x9e3779b97f4a7c15ull + (d << 6) + (d >> 2)));
  }
  return d;
}

}  // extern "C"
