// mcdc_internal.h — device data layout shared by the HIP kernels
// (mcdc_kernels.hip) and the C-ABI host code (mcdc_api.hip).
//
// Pipeline:
//   k_scan_q    streaming, HBM-bound: per-position windowed Gear hash, exact
//               S/L flags for every position whose 48-byte window passes the
//               prefilter -> per-run candidate lists and summaries (run = kRun
//               bytes)
//   k_spec_lane one lane per segment (default when max <= 64 runs):
//               speculative cut chain from the segment start (lane_next =
//               exact fastcdc cut_gear semantics); a segment it cannot walk
//               goes to k_spec_list (the group walk below)
//   k_spec6     one 16-lane group (a DPP row) per segment: the same chain
//               (group_next), for large max and the staged pipeline
//   k_link_lane / k_link
//               per segment: continue past the segment end until the chain
//               merges with a later segment's speculative chain (the group
//               walk takes forced stretches whole: forced_run)
//   clean path  k_incr_scan (or k_incr_count + scan + k_add_base) + k_emit
//   general     k_fallback (one wave per file whose continuation never
//               merged: serial walk), k_walk_fast / k_irr_flags / k_walk_jumps
//               (segments on the true chain, one jump per irregular link),
//               k_count + hipcub scan, k_emit, k_emit_long
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcdc {

// VGPR slack: on gfx950 a kernel whose descriptor allocates
// exactly the registers its code uses (next_free_vgpr a multiple of the
// 8-register granule) loses values of whole waves: k_emit at 184/184 gave
// ~19 K wrong hashes per 64 GiB call, and the byte-identical code with only
// the descriptor's allocation raised to 192 gave none (tools/dbg/kd_patch.py).
// MCDC_VGPR_PAD(n), n = the kernel's own count, makes the allocation reach
// past every register the kernel uses; mapache_amd/build.py audits every
// kernel of the library and rejects a build in which one outside its
// documented list fills its allocation exactly.
#define MCDC_VGPR_PAD_STR(x) #x
#define MCDC_VGPR_PAD(n) asm volatile("v_mov_b32 v" MCDC_VGPR_PAD_STR(n) ", 0" ::: "v" MCDC_VGPR_PAD_STR(n))

#ifndef MCDC_KRUN
#define MCDC_KRUN 4096  // (compile-time A/B knob)
#endif
constexpr int kRun = MCDC_KRUN;       // bytes hashed per lane per scan run
constexpr int kWin = 48;              // bits 0..47 of the Gear hash = last 48 bytes
constexpr int kContMax = 64;          // continuation steps before serial fallback
constexpr int kGroup = 16;            // lanes per chain in k_spec / k_link / k_emit
constexpr uint64_t kRepMax = 1u << 30; // nodes per continuation entry (forced stretch)
constexpr uint64_t kEmitInline = 256;  // longer continuations are emitted by k_emit_long
constexpr uint8_t kRunOverflow = 255; // run_cnt marker: candidates exceed cap
constexpr uint32_t kSegNone = 0xffffffffu;
constexpr uint32_t kSegFail = 0xfffffffeu;

// per-segment flags
constexpr uint32_t kSegFirst = 1u, kSegLast = 2u;
// per-file flags (set with atomicOr by k_link)
constexpr uint32_t kFileSkip = 1u, kFileFail = 2u, kFileFallbackDone = 4u;
// error word bits
constexpr uint32_t kErrNodeCap = 1u, kErrOutCap = 2u;

// Run summary (written by the scan beside run_cnt): bits 0-13 = 1 + offset of
// the run's first S candidate (0: none), bits 14-27 = 1 + offset of its first
// L candidate, bits 28-31 = min(candidate count, 15).  Exact also for runs whose
// entry list overflowed.  A chain step decides most runs from it alone.
static_assert(kRun <= 16383, "run offsets must fit the 14-bit summary fields");
__host__ __device__ inline uint32_t run_summary(uint32_t cnt, uint32_t first_s, uint32_t first_l) {
  return (cnt > 15u ? 15u : cnt) << 28 | (first_l == 0xffffffffu ? 0u : first_l + 1u) << 14 |
         (first_s == 0xffffffffu ? 0u : first_s + 1u);
}

// Tiles of k_incr_lookback (1024 segments each), one status word per tile.
__host__ __device__ inline uint64_t lb_tiles(uint32_t nsegs) { return (uint64_t)nsegs / 1024 + 1; }

struct Seg {
  uint64_t start, end;  // arena positions [start, end)
  uint32_t file, flags;
};

struct File {
  uint64_t start, end;  // arena positions
  uint32_t first_seg, nsegs;
};

struct DevChunk {       // == mcdc_chunk
  uint64_t offset, length, hash;
};

struct DevParams {
  uint32_t min, avg, max, cap;  // cap = candidate slots per run
  uint64_t ms, ml;              // mask_s, mask_l
  uint64_t ms16, ml16;          // masks << 16 (scan keeps h << 16)
  uint32_t pf_hi;               // prefilter on the high dword of h << 16
  uint32_t pad;
};

struct Work {
  const uint8_t *base;   // 16-byte aligned arena base
  uint64_t n_al;         // arena length (multiple of 16)
  uint64_t nruns;        // ceil(n_al / kRun)
  const uint64_t *gear;  // GEAR[256]
  const uint64_t *gear16;// GEAR[256] << 16
  uint8_t *run_cnt;      // [nruns]
  uint32_t *run_sum;     // [nruns] run summary: first S / first L candidate (see run_summary)
  uint32_t *run_ent;     // [nruns * cap]: off | S<<31 | L<<30
  uint64_t *run_bits;    // [2 * (nruns / 64 + 2)]: word pair w = runs [64w, 64w + 64): [2w] bit i = run
                         // 64w + i has an S candidate, [2w + 1] an L candidate (the lane walk's index)
  uint64_t *tile_ctr;    // scan tile counter (dynamic tile order) or nullptr (static)
  uint32_t first_static; // dynamic order: each wave's first tile is its static one, the counter hands out the rest

  const Seg *segs;
  uint32_t nsegs, nfiles;
  const File *files;
  uint64_t zseg;         // segment length (bytes)

  uint64_t *nodes;       // speculative chain nodes, per segment at node_off[s]
  const uint64_t *node_off;
  uint32_t *node_cnt;
  uint64_t *seg_exit;    // first chain position >= segment end
  uint64_t *cont;        // [nsegs * kContMax] continuation entries: first node
  uint32_t *cont_rep;    // [nsegs * kContMax] nodes in the entry (cont + i*max)
  uint32_t *cont_cnt;    // continuation nodes (expanded)
  uint32_t *cont_ent;    // continuation entries
  uint32_t *link_seg;    // segment the continuation merged into (or None/Fail)
  uint32_t *link_idx;    // index of the merge node in that segment's list
  uint64_t *link_pos;    // merge position (= next true chunk start) or file end
  uint32_t *file_flags;
  uint8_t *seg_true;
  uint32_t *entry_idx;
  uint64_t *seg_count;   // chunks emitted per segment
  uint64_t *seg_off;     // exclusive prefix of seg_count
  DevChunk *out;
  uint64_t out_cap;
  uint32_t *err;         // [0] error bits, [1] files resolved by k_fallback, [2] dirty, [3] long_n
  uint32_t *long_list;   // segments whose continuation exceeds kEmitInline nodes
  uint32_t *long_n;      // (= err + 3)
  uint8_t *irr_flag;     // general path: segment's link is not to the next segment
  uint32_t *irr_list;    // sorted irregular segment indices, count in *irr_n
  uint32_t *irr_n;
  uint32_t *punt_spec;   // lane walk: segments handed to the group walk (k_spec_list), count err[4]
  uint32_t *punt_link;   // (k_link_list), count err[5]
  uint32_t ncu;          // compute units (persistent grids)
  uint64_t *lb_status;   // k_incr_lookback tile status words (lane walk: zeroed per call), ticket err[6]
  const uint32_t *run_list;  // list-mode scan (or nullptr): the full runs a chunk window can reach, ascending
  uint64_t list_n;           // (k_run_list builds it; k_scan_q<.., LIST> scans only those)
};

// Tuning switches of a context, read from the environment once, when the
// context is created (mcdc_ctx_create), never per call.  The first group
// selects tested alternative paths (the staged pipeline, lane pieces, warm /
// cold pieces, pinned-output mode); the second only exists in A/B builds
// (-DMCDC_AB_KNOBS, `python -m mapache_amd.build --ab`), the product build
// ignores those variables.
struct Knobs {
  int parts = 1;          // MCDC_PARTS: scan parts of the staged pipeline (1..4)
  int tail_rounds = 2;    // MCDC_TAIL_ROUNDS: rounds of the last part
  int part_tiles = 0;     // MCDC_PART_TILES: tiles per round (0: the scan's wave count)
  int min_rounds = 8;     // MCDC_MIN_ROUNDS: smallest call that is staged, in rounds
  int scan_pieces = 0;    // MCDC_SCAN_PIECES: lane pieces per run (0: by size, scan_pieces())
  int scan_cold = 1;      // MCDC_SCAN_COLD: cold-started lane pieces
  int pinned_direct = 1;  // MCDC_PINNED_DIRECT: k_emit writes pinned host output directly
  int lane_walk = 1;      // MCDC_LANE_WALK: 0 group walk only, 1 lane walk when max <= 64 runs, 2 always
  int lane_seg_chunks = 4;// MCDC_LANE_SEG_CHUNKS: expected chunks per segment on the lane walk
  int run_list = 1;       // MCDC_RUN_LIST: list-mode scan of batch calls (0 off, 1 when it skips >= 20 % of
                          // the runs, 2 whenever the layout allows it: tests)
  bool zc_huf = true;      // MCDC_ZC_HUF: Huffman / RLE literals in the GPU zstd compressor
  bool zc_two = true;      // MCDC_ZC_TWO: compressor batches alternate between two streams
  uint64_t save_group_blocks = 0;  // GPU save path: blocks per compression group (0: max(zc_batch, 32768))
  bool zc_small = true;    // chunks of one block through k_zc_small (0: k_zc_probe / k_zc_find, the A/B)
  // set by mcdc_ctx_set_option only (no environment variable):
  uint64_t zc_batch = 16384;           // "zc_batch_blocks": blocks per compressor batch (two streams: half each)
  bool test_fail_after_index = false;  // "test_fail_after_index": mcdc_save_files fails after its index
                                       // add (test hook: the rollback path, tests/test_gpu_save.py)
  // A/B builds only
  int group = 16;         // MCDC_GROUP: lanes per chain group (8, 16, 32)
  int spec_occ = 6;       // MCDC_SPEC_OCC: k_spec waves-per-SIMD build (5 or 6)
  int dyn_tiles = 1;      // MCDC_DYN_TILES: scan tiles from an atomic counter
  int first_static = 1;   // MCDC_FIRST_STATIC: each wave's first tile static
  int seg_chunks = 16;    // MCDC_SEG_CHUNKS: expected chunks per segment
};
Knobs read_knobs();

// launch wrappers (mcdc_kernels.hip); all enqueue on `stream`.
void launch_fill_random(void *dst, uint64_t pos, uint64_t n, uint64_t seed, hipStream_t stream);
// scan of full tiles [tile0, tile1) (+ the partial last tile when `tail`);
// ev0 / ev1 (optional) are recorded at the launch's start and end by the
// dispatch itself (hipExtLaunchKernelGGL: no marker packets between kernels)
void launch_scan(const Work &w, const DevParams &p, int num_cus, hipStream_t stream, uint64_t tile0,
                 uint64_t tile1, bool tail, int pieces, bool cold, hipEvent_t ev0 = nullptr,
                 hipEvent_t ev1 = nullptr);
int scan_pieces(uint64_t nruns_full, int num_cus);  // lane pieces per run for a whole-call scan
uint64_t scan_waves(uint64_t ntiles, int num_cus);  // waves of a scan launch over ntiles
void launch_spec(const Work &w, const DevParams &p, const Knobs &k, uint32_t s0, uint32_t s1, hipStream_t stream);
// node_cap: expanded continuation nodes per segment (~0 when everything is scanned)
void launch_link(const Work &w, const DevParams &p, const Knobs &k, uint32_t s0, uint32_t s1, uint64_t node_cap,
                 hipStream_t stream);
void launch_emit_incremental(const Work &w, const DevParams &p, uint32_t s0, uint32_t s1, uint64_t *incl,
                             void *scan_tmp, size_t scan_tmp_bytes, hipStream_t stream, int gs = 16);
// whole-call resolution with the lane walk (single part): spec, link, counts,
// offsets and boundaries of every segment, the group walk for handed-back ones
// fcnt (optional): chunks per file into pinned host memory, by the emit kernel
void launch_resolve_lane(const Work &w, const DevParams &p, uint64_t *incl, void *scan_tmp, size_t scan_tmp_bytes,
                         hipStream_t stream, uint64_t *fcnt = nullptr);
void launch_resolve_general(const Work &w, const DevParams &p, void *scan_tmp, size_t scan_tmp_bytes,
                            hipStream_t stream);
size_t scan_tmp_bytes(uint32_t nsegs);
// ev_done (optional): recorded by the dispatch; zero[0, zwords) (optional)
// cleared when the call needs no general resolution (err[2] == 0)
void launch_finish(const Work &w, uint64_t *res, hipStream_t stream, hipEvent_t ev_done = nullptr,
                   uint64_t *zero = nullptr, uint32_t zwords = 0);
void launch_file_counts(const Work &w, uint64_t *dst, hipStream_t stream);  // chunks per file -> dst
// the list-mode scan's run list from nent {first run, list index} entries
// (each <= 64 runs, the last ending at list_n), the candidate-bitmap words and
// the tile counter zeroed (words [0, nwords)); ev0: recorded at its start
// the segment plan of n files (fse: their starts, then their ends) on the
// GPU: files[n], segs, node_off (as run_pipeline's host plan); bsum: 2 words
// per 256 files
void launch_plan(const uint64_t *fse, uint64_t n, uint64_t Z, uint64_t ms1, uint64_t *bsum, File *files, Seg *segs,
                 uint64_t *node_off, hipStream_t stream);
void launch_run_list(const uint32_t *ent, uint64_t nent, uint64_t list_n, uint32_t *list, uint64_t *words,
                     uint64_t nwords, hipStream_t stream, hipEvent_t ev0 = nullptr);

}  // namespace mcdc
