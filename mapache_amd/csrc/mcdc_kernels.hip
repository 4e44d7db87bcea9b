// mcdc_kernels.hip — CDNA4 (gfx950) kernels of the FastCDC v2020 chunker.
//
// Semantics: exactly fastcdc 3.2.1 `v2020::cut_gear` applied chunk after chunk
// from the start of every file (the crate's StreamCDC == FastCDC over the
// whole slice), as called by mapache at
// /root/reference/src/archiver/processor.rs:173-202.
//
// Algorithm:
//  * Every mask bit of every MASKS entry lies in bits 0..47, so for a chunk
//    whose hashing restarted at t, the cut test at p >= t+47 depends only on
//    W_p = sum_{k<48} GEAR[x_{p-k}] << k (mod 2^48).  k_scan evaluates W_p at
//    every byte in parallel (one lane = one contiguous 2 KiB run) and records
//    the sparse positions where S(p) = (W_p & mask_s)==0 or L(p) = ... mask_l.
//  * The first 47 positions after each restart use the exact restarted hash,
//    computed on the fly (wave prefix-shift-scan) while walking chains.
//  * Chains are resolved per segment speculatively and stitched where they
//    merge (k_spec / k_link / k_walk); a file whose chains never merge falls
//    back to one serial wave (k_fallback).  No CPU in the loop.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "mcdc_internal.h"


namespace mcdc {

// ======================================================== wave helpers ====
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, unsigned d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d);
  const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// ============================================================ fill =======
// Synthetic stream shared with oracle/ (oc_fill_random) and bench.py.
__global__ void k_fill_random(uint8_t *__restrict__ dst, uint64_t pos, uint64_t n, uint64_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t head = (8 - (pos & 7)) & 7;  // bytes until the first word boundary
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid < head && tid < n) {
    const uint64_t p = pos + tid;
    dst[tid] = (uint8_t)(mix64(seed + ((p >> 3) + 1) * 0x9e3779b97f4a7c15ull) >> (8 * (p & 7)));
  }
  if (n <= head) return;
  const uint64_t words = (n - head) / 8;
  uint8_t *d = dst + head;
  const uint64_t w0 = (pos + head) >> 3;
  const bool aligned = (((uintptr_t)d) & 7) == 0;
  for (uint64_t i = tid; i < words; i += stride) {
    const uint64_t w = mix64(seed + (w0 + i + 1) * 0x9e3779b97f4a7c15ull);
    if (aligned) {
      reinterpret_cast<uint64_t *>(d)[i] = w;
    } else {
      for (int b = 0; b < 8; ++b) d[8 * i + b] = (uint8_t)(w >> (8 * b));
    }
  }
  const uint64_t tail0 = head + words * 8;
  if (tid < n - tail0) {
    const uint64_t p = pos + tail0 + tid;
    dst[tail0 + tid] = (uint8_t)(mix64(seed + ((p >> 3) + 1) * 0x9e3779b97f4a7c15ull) >> (8 * (p & 7)));
  }
}

void launch_fill_random(void *dst, uint64_t pos, uint64_t n, uint64_t seed, hipStream_t stream) {
  if (n == 0) return;
  const uint64_t words = n / 8 + 2;
  uint64_t blocks = (words + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(k_fill_random, dim3((unsigned)blocks), dim3(256), 0, stream, (uint8_t *)dst, pos,
                     n, seed);
}

// ============================================================ scan =======
// LDS holds GEAR<<16 replicated 32x: entry x, copy c at byte (x << 8) | (c << 3).
// ds_read_b64 is serviced in two 32-lane halves with bank = (addr/4) % 64;
// lane l reads copy (l & 31) -> banks 2(l&31), 2(l&31)+1: conflict-free for
// any input bytes.  The address is one v_perm_b32: byte 0 = lane offset,
// byte 1 = the data byte, bytes 2-3 = 0.
//
// The hash is kept as h' = h << 16 (mod 2^64): bits 0..47 of h live in bits
// 16..63 of h', so the bits that depend on bytes older than the 48-byte window
// fall off the top by themselves, and one v_lshl_add_u64 updates it.

__device__ __forceinline__ uint64_t lds_gear(const uint64_t *tab, uint32_t byteaddr) {
  return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(tab) + byteaddr);
}

template <int K>
__device__ __forceinline__ uint32_t gaddr(uint32_t w, uint32_t laneoff) {
  return __builtin_amdgcn_perm(w, laneoff, 0x0c0c0000u | ((4u + K) << 8));
}

#define MCDC_STEP_NC(W, K) h = (h << 1) + lds_gear(tab, gaddr<K>(W, lo));
#define MCDC_STEP_PF(W, K)                                    \
  h = (h << 1) + lds_gear(tab, gaddr<K>(W, lo));              \
  acc = min(acc, (uint32_t)(h >> 32) & pf);
#define MCDC_STEP_EX(W, K, I)                                                         \
  {                                                                                   \
    x = (x << 1) + lds_gear(tab, gaddr<K>(W, lo));                                    \
    const uint32_t s_ = (x & ms16) == 0, l_ = (x & ml16) == 0;                        \
    if (s_ | l_) {                                                                    \
      if (cnt < cap) ent[cnt] = (off + (I)) | (s_ << 31) | (l_ << 30);                \
      ++cnt;                                                                          \
    }                                                                                 \
  }

__device__ __forceinline__ void hash16(const uint64_t *tab, uint32_t lo, const uint4 d, uint64_t &h) {
  MCDC_STEP_NC(d.x, 0) MCDC_STEP_NC(d.x, 1) MCDC_STEP_NC(d.x, 2) MCDC_STEP_NC(d.x, 3)
  MCDC_STEP_NC(d.y, 0) MCDC_STEP_NC(d.y, 1) MCDC_STEP_NC(d.y, 2) MCDC_STEP_NC(d.y, 3)
  MCDC_STEP_NC(d.z, 0) MCDC_STEP_NC(d.z, 1) MCDC_STEP_NC(d.z, 2) MCDC_STEP_NC(d.z, 3)
  MCDC_STEP_NC(d.w, 0) MCDC_STEP_NC(d.w, 1) MCDC_STEP_NC(d.w, 2) MCDC_STEP_NC(d.w, 3)
}

// 16 positions: prefilter every byte; on a (rare, wave-uniform) hit re-walk
// the 16 bytes exactly and append S/L candidates.
__device__ __forceinline__ void scan16(const uint64_t *tab, uint32_t lo, const uint4 d, uint64_t &h,
                                       uint32_t pf, uint64_t ms16, uint64_t ml16, uint32_t off,
                                       uint32_t &cnt, uint32_t *ent, uint32_t cap) {
  const uint64_t h0 = h;
  uint32_t acc = 0xffffffffu;
  MCDC_STEP_PF(d.x, 0) MCDC_STEP_PF(d.x, 1) MCDC_STEP_PF(d.x, 2) MCDC_STEP_PF(d.x, 3)
  MCDC_STEP_PF(d.y, 0) MCDC_STEP_PF(d.y, 1) MCDC_STEP_PF(d.y, 2) MCDC_STEP_PF(d.y, 3)
  MCDC_STEP_PF(d.z, 0) MCDC_STEP_PF(d.z, 1) MCDC_STEP_PF(d.z, 2) MCDC_STEP_PF(d.z, 3)
  MCDC_STEP_PF(d.w, 0) MCDC_STEP_PF(d.w, 1) MCDC_STEP_PF(d.w, 2) MCDC_STEP_PF(d.w, 3)
  if (__builtin_expect(__any(acc == 0), 0)) {
    if (acc == 0) {
      uint64_t x = h0;
      MCDC_STEP_EX(d.x, 0, 0) MCDC_STEP_EX(d.x, 1, 1) MCDC_STEP_EX(d.x, 2, 2) MCDC_STEP_EX(d.x, 3, 3)
      MCDC_STEP_EX(d.y, 0, 4) MCDC_STEP_EX(d.y, 1, 5) MCDC_STEP_EX(d.y, 2, 6) MCDC_STEP_EX(d.y, 3, 7)
      MCDC_STEP_EX(d.z, 0, 8) MCDC_STEP_EX(d.z, 1, 9) MCDC_STEP_EX(d.z, 2, 10) MCDC_STEP_EX(d.z, 3, 11)
      MCDC_STEP_EX(d.w, 0, 12) MCDC_STEP_EX(d.w, 1, 13) MCDC_STEP_EX(d.w, 2, 14) MCDC_STEP_EX(d.w, 3, 15)
    }
  }
}

// Summary of a run whose entries were appended in position order (the
// lane-strided paths): exact when the list holds them all; an overflowed list
// may miss the first candidate of a kind, so it reads "unknown" (count set,
// both offsets 0) and chain steps consult the bytes.
__device__ __forceinline__ uint32_t summary_from_entries(const uint32_t *ent, uint32_t cnt, uint32_t cap) {
  if (cnt > cap) return 15u << 28;
  uint32_t fs = 0xffffffffu, fl = 0xffffffffu;
  for (uint32_t i = cnt; i-- > 0;) {
    const uint32_t e = ent[i];
    if (e >> 31) fs = e & 0x00ffffffu;
    if ((e >> 30) & 1u) fl = e & 0x00ffffffu;
  }
  return run_summary(cnt, fs, fl);
}

// One full run of RUN bytes.  PF = 64-byte groups kept in flight ahead of the
// group being hashed (register ring of 4*PF uint4 per lane).
template <int RUN, int PF>
__device__ __forceinline__ void scan_run_full(const uint64_t *tab, uint32_t lo, const Work &W,
                                              const DevParams &P, uint64_t run, uint64_t addr_run) {
  static_assert(RUN % 64 == 0 && RUN / 64 > PF, "run too short");
  const uint4 *p = reinterpret_cast<const uint4 *>(W.base + addr_run * (uint64_t)RUN);
  uint64_t h = 0;
  if (addr_run > 0) {  // warm-up: the 48 bytes before the run complete every window
    const uint4 w0 = p[-3], w1 = p[-2], w2 = p[-1];
    hash16(tab, lo, w0, h);
    hash16(tab, lo, w1, h);
    hash16(tab, lo, w2, h);
  }
  const uint32_t pf = P.pf_hi, cap = P.cap;
  const uint64_t ms16 = P.ms16, ml16 = P.ml16;
  uint32_t *ent = W.run_ent + run * (uint64_t)cap;
  uint32_t cnt = 0;
  constexpr int G = RUN / 64;
  uint4 ring[PF + 1][4];
#pragma unroll
  for (int k = 0; k < PF; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) ring[k][j] = p[4 * k + j];
#pragma unroll 1
  for (int g = 0; g < G; g += PF + 1) {
    // PF+1 groups per iteration so that ring slots are compile-time indices
#pragma unroll
    for (int u = 0; u <= PF; ++u) {
      const int gg = g + u;
      if (gg < G) {
        {  // unconditional (clamped) prefetch keeps vmcnt waits counted
          const int src = gg + PF < G ? gg + PF : G - 1;
#pragma unroll
          for (int j = 0; j < 4; ++j) ring[(u + PF) % (PF + 1)][j] = p[4 * src + j];
        }
        const uint32_t off = 64u * gg;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          scan16(tab, lo, ring[u][j], h, pf, ms16, ml16, off + 16 * j, cnt, ent, cap);
      }
    }
  }
  W.run_cnt[run] = cnt > cap ? kRunOverflow : (uint8_t)cnt;
  W.run_sum[run] = summary_from_entries(ent, cnt, cap);
}

// Last, partial run: byte loop with exact tests (one lane in the whole grid).
template <int RUN>
__device__ void scan_run_tail(const uint64_t *tab, uint32_t lo, const Work &W, const DevParams &P,
                              uint64_t run) {
  const uint64_t start = run * (uint64_t)RUN, end = W.n_al;
  const uint64_t w0 = start >= (uint64_t)kWin ? start - kWin : 0;
  uint64_t h = 0;
  uint32_t cnt = 0, fs = 0xffffffffu, fl = 0xffffffffu;
  uint32_t *ent = W.run_ent + run * (uint64_t)P.cap;
  for (uint64_t q = w0; q < end; ++q) {
    h = (h << 1) + lds_gear(tab, ((uint32_t)W.base[q] << 8) | lo);
    if (q >= start) {
      const uint32_t s_ = (h & P.ms16) == 0, l_ = (h & P.ml16) == 0;
      if (s_ | l_) {
        if (cnt < P.cap) ent[cnt] = (uint32_t)(q - start) | (s_ << 31) | (l_ << 30);
        ++cnt;
        if (s_ && fs == 0xffffffffu) fs = (uint32_t)(q - start);
        if (l_ && fl == 0xffffffffu) fl = (uint32_t)(q - start);
      }
    }
  }
  W.run_cnt[run] = cnt > P.cap ? kRunOverflow : (uint8_t)cnt;
  W.run_sum[run] = run_summary(cnt, fs, fl);
}

template <int RUN, int WPE, int PF, int CH = 1, int BLOCK = 512>
__global__ __launch_bounds__(BLOCK, WPE) void k_scan_t(Work W, DevParams P) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = W.gear16[i >> 5];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nfull = W.n_al / RUN;
  const uint64_t nruns = (W.n_al + RUN - 1) / RUN;
  const uint64_t ntiles = (nruns + 63) / 64;
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    if (run < nfull) {
      scan_run_full<RUN, PF>(tab, lo, W, P, run, run);
    }
    else if (run < nruns) scan_run_tail<RUN>(tab, lo, W, P, run);
  }
}

// One run scanned by a whole wave (the runs of a partial last tile): lane l
// takes bytes [64 l, 64 l + 64) of the run after a 48-byte warm-up, so the
// run costs ~112 dependent hash steps instead of 4096 on one lane.  Exact
// S / L tests at every position; entries in position order (wave prefix sum
// over the lanes' counts, then a second walk that stores the first `cap`),
// count and summary as the main path writes them.
__device__ __forceinline__ uint64_t coop_walk(const uint64_t *tab, uint32_t lo, const Work &W, uint64_t a0,
                                              uint64_t s, uint64_t e, uint64_t ms16, uint64_t ml16, bool store,
                                              uint32_t *ent, uint32_t base_idx,
                                              uint32_t cap, uint64_t rs, uint32_t *fs, uint32_t *fl) {
  uint64_t h = 0;
  uint32_t k = 0;
  for (uint64_t b = a0; b < e; b += 16) {
    const uint4 d = *reinterpret_cast<const uint4 *>(W.base + b);
    const uint32_t wd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      h = (h << 1) + lds_gear(tab, ((wd[i >> 2] >> (8 * (i & 3))) & 0xffu) << 8 | lo);
      const uint64_t q = b + i;
      if (q >= s && q < e) {
        const uint32_t s_ = (h & ms16) == 0, l_ = (h & ml16) == 0;
        if (s_ | l_) {
          const uint32_t off = (uint32_t)(q - rs);
          if (store && base_idx + k < cap) ent[base_idx + k] = off | (s_ << 31) | (l_ << 30);
          if (s_ && *fs == 0xffffffffu) *fs = off;
          if (l_ && *fl == 0xffffffffu) *fl = off;
          ++k;
        }
      }
    }
  }
  return k;
}

__device__ void scan_run_coop(const uint64_t *tab, uint32_t lo, const Work &W, const DevParams &P, uint64_t run,
                              uint32_t lane) {
  const uint64_t rs = run * (uint64_t)kRun, re = min(rs + (uint64_t)kRun, W.n_al);
  const uint64_t s = rs + 64ull * lane, e = min(s + 64, re);
  const uint64_t a0 = s >= 48 ? s - 48 : 0;  // (16-aligned: rs and 64 * lane are)
  uint32_t *ent = W.run_ent + run * (uint64_t)P.cap;
  uint32_t fs = 0xffffffffu, fl = 0xffffffffu, dummy_s = 0, dummy_l = 0;
  uint32_t c = 0;
  if (s < re) c = (uint32_t)coop_walk(tab, lo, W, a0, s, e, P.ms16, P.ml16, false, ent, 0, P.cap, rs, &fs, &fl);
  uint32_t x = c;  // inclusive wave prefix of the counts
#pragma unroll
  for (unsigned d = 1; d < 64; d <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += v;
  }
  const uint32_t pre = x - c, total = (uint32_t)__shfl((int)x, 63, 64);
  if (c && pre < P.cap)  // second walk: store this lane's entries that fall among the first cap
    coop_walk(tab, lo, W, a0, s, e, P.ms16, P.ml16, true, ent, pre, P.cap, rs, &dummy_s, &dummy_l);
  uint32_t mfs = fs, mfl = fl;
#pragma unroll
  for (unsigned d = 1; d < 64; d <<= 1) {
    mfs = min(mfs, (uint32_t)__shfl_xor((int)mfs, d, 64));
    mfl = min(mfl, (uint32_t)__shfl_xor((int)mfl, d, 64));
  }
  if (lane == 0) {
    W.run_cnt[run] = total > P.cap ? kRunOverflow : (uint8_t)total;
    W.run_sum[run] = run_summary(total, mfs, mfl);
    // candidate bitmaps (their words were zeroed before the scan: tail runs
    // share words with each other and with the last full tile)
    uint32_t *b32 = reinterpret_cast<uint32_t *>(W.run_bits) + 4 * (run >> 6) + ((run >> 5) & 1);
    if (mfs != 0xffffffffu) atomicOr(b32, 1u << (run & 31));
    if (mfl != 0xffffffffu) atomicOr(b32 + 2, 1u << (run & 31));
  }
}

// ---- Product scan (k_scan_q).  One wave = one tile of 64 runs (one per
// lane).  Loads are quad-coalesced: lane quad i fetches one whole 64-byte line
// of run (4i+k) per load instruction k (16 lines per wave-instruction instead
// of 64), then the wave transposes through a private LDS pad (run stride 80 B:
// conflict-free ds_write_b128 / ds_read_b128) so each lane hashes its own
// contiguous run.  Per byte the loop issues one v_perm_b32 (LDS address), one
// ds_read_b64 (GEAR<<16), one v_lshl_add_u64 (hash), one v_and_b32 with the
// prefilter mask held in a VGPR (VOP2 with an SGPR operand issues at half rate
// on gfx950, tools/ubench2.hip) and half a v_min3_u32; the LDS lookups of the
// next dword are issued before the hash chain of the current one.
//
// Rare path, deferred: a 16-byte block whose prefilter fires (2^-14 per byte
// at 16/64/256 KiB; ~6 % of wave-steps have at least one such lane) is only
// queued — hash before the block, run lane, offset — in the 16 spare bytes of
// the pad rows.  The queue is drained by all lanes at once (one entry per
// lane) at the end of the tile or when it would overflow; candidates are
// counted per run with LDS atomics, so a run's entries are unordered (the chain
// walk takes the minimum).  Measured (tools/scanbench, 16 GiB): the deferred
// queue alone +7-13 % over re-walking the block under an exec mask.
//
// LDS = 64 KiB table + 16 waves x (5 KiB pad + 768 B run counters and
// first-candidate minima) = 156 KiB.
constexpr int kQPad = 80;                        // run stride in the transpose pad
constexpr int kQPadBytes = 64 * kQPad;           // 5 KiB
constexpr int kQWaveBytes = kQPadBytes + 64 * 12;  // + per-run candidate counters, first S, first L
constexpr int kSTab = 65536;                     // GEAR<<16 x 32 copies

// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4],
// lgkmcnt [11:8]); vmcnt/expcnt left at their maxima (no wait).
constexpr int kWaitLgkm4 = 0xC07F | (4 << 8);
constexpr int kWaitLgkm0 = 0xC07F;

__device__ __forceinline__ uint32_t to_vgpr(uint32_t s) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
  return v;
}

__device__ __forceinline__ void lookup4(const uint64_t *tab, uint32_t lo, uint32_t w, uint64_t *g) {
  g[0] = lds_gear(tab, gaddr<0>(w, lo));
  g[1] = lds_gear(tab, gaddr<1>(w, lo));
  g[2] = lds_gear(tab, gaddr<2>(w, lo));
  g[3] = lds_gear(tab, gaddr<3>(w, lo));
}

__device__ __forceinline__ void chain4(const uint64_t *g, uint64_t &h, uint32_t &acc, uint32_t pf) {
  h = (h << 1) + g[0];
  const uint32_t m0 = (uint32_t)(h >> 32) & pf;
  h = (h << 1) + g[1];
  const uint32_t m1 = (uint32_t)(h >> 32) & pf;
  h = (h << 1) + g[2];
  const uint32_t m2 = (uint32_t)(h >> 32) & pf;
  h = (h << 1) + g[3];
  const uint32_t m3 = (uint32_t)(h >> 32) & pf;
  acc = min(min(acc, m0), m1);  // -> v_min3_u32 x2
  acc = min(min(acc, m2), m3);
}

// Prefilter block: dwords per wave-uniform test (and per queued block).
#ifndef MCDC_QBLK_DW
#define MCDC_QBLK_DW 4
#endif
constexpr int kQBlkDw = MCDC_QBLK_DW;
static_assert(kQBlkDw == 4 || kQBlkDw == 8, "16- or 32-byte prefilter blocks");

// Drain the wave's queue: lane i re-walks entry i's block exactly.
// PC pieces per run: lane l hashes bytes [l*SUB, (l+1)*SUB) of the tile, part
// l % PC of run run0 + l / PC; offsets and counters are per run.
template <int RUN, int PC, bool LIST = false>
__device__ __attribute__((noinline)) void q_drain(const uint64_t *tab, uint32_t lo, const uint8_t *base,
                                                  uint32_t *run_ent, uint64_t ms16, uint64_t ml16, uint32_t cap,
                                                  const char *pad, uint32_t *lcnt, uint32_t qn, uint64_t run0,
                                                  uint32_t lane, const uint32_t *lst = nullptr, uint32_t lim = 0) {
  constexpr int SUB = RUN / PC;
  if (lane < qn) {
    const char *slot = pad + lane * kQPad + 64;
    uint64_t x = *reinterpret_cast<const uint64_t *>(slot);
    const uint32_t meta = *reinterpret_cast<const uint32_t *>(slot + 8);
    const uint32_t pl = meta >> 16, rl = pl / PC, off = (pl % PC) * SUB + (meta & 0xffffu);
    const uint64_t run = LIST ? (uint64_t)lst[min(rl, lim)] : run0 + rl;  // (list mode: the tile's rl-th listed run)
    // (list mode: lanes past the list's end re-scan its last run; only its own lanes store)
    const uint32_t kcap = LIST && rl > lim ? 0u : cap;
    uint32_t *ent = run_ent + run * (uint64_t)cap;
    uint32_t wd[kQBlkDw];
#pragma unroll
    for (int j = 0; j < kQBlkDw / 4; ++j) {
      const uint4 d = *reinterpret_cast<const uint4 *>(base + run * (uint64_t)RUN + off + 16 * j);
      wd[4 * j] = d.x; wd[4 * j + 1] = d.y; wd[4 * j + 2] = d.z; wd[4 * j + 3] = d.w;
    }
#pragma unroll
    for (int i = 0; i < 4 * kQBlkDw; ++i) {
      x = (x << 1) + lds_gear(tab, ((wd[i >> 2] >> (8 * (i & 3))) & 0xffu) << 8 | lo);
      const uint32_t s_ = (x & ms16) == 0, l_ = (x & ml16) == 0;
      if (s_ | l_) {
        const uint32_t k = atomicAdd(&lcnt[rl], 1u);
        if (k < kcap) ent[k] = (off + i) | (s_ << 31) | (l_ << 30);
        if (s_) atomicMin(&lcnt[64 + rl], off + i);   // first S / first L of the run (summary)
        if (l_) atomicMin(&lcnt[128 + rl], off + i);
      }
    }
  }
}

struct QScan {  // per-wave state of k_scan_q
  const uint64_t *tab;
  uint32_t lo, lane, pf, cap;
  uint64_t ms16, ml16;
  char *pad;
  uint32_t *lcnt;
  const uint8_t *base;
  uint32_t *run_ent;
  const uint32_t *lst;  // list mode: the tile's runs (W.run_list + RPT t), lim = valid entries - 1
  uint32_t lim;
};

// 64 bytes (16 dwords) of one run: lookups one dword ahead of the chain;
// every prefilter block (4 kQBlkDw bytes) a wave-uniform test queues the
// blocks whose prefilter fired.
// ND dwords (16: one 64-byte group; 12: the re-walked first 48 bytes of a
// cold-started piece).  skip3: the first 48 positions of a cold-started piece
// hold incomplete windows; their blocks are not tested here (see k_scan_q).
template <int RUN, int PC, int ND = 16, bool LIST = false>
__device__ __forceinline__ void scan64q(const QScan &q, const uint32_t *w, uint64_t &h, uint32_t off,
                                        uint32_t &qn, uint64_t run0, bool skip3 = false) {
  uint64_t g[2][4];
  lookup4(q.tab, q.lo, w[0], g[0]);
  uint32_t acc = 0xffffffffu;
  uint64_t hb = h;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    if (d + 1 < ND) lookup4(q.tab, q.lo, w[d + 1], g[(d + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    // one wait per dword for its 4 lookups (the next dword's 4 stay in flight)
    // instead of the compiler's one wait per lookup
    if (d + 1 < ND) __builtin_amdgcn_s_waitcnt(kWaitLgkm4);
    else __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    chain4(g[d & 1], h, acc, q.pf);
    if (d % kQBlkDw == kQBlkDw - 1) {
      const uint64_t m = (d < 12 && skip3) ? 0ull : __ballot(acc == 0);
      if (__builtin_expect(m != 0, 0)) {
        const uint32_t n = (uint32_t)__popcll(m);
        if (qn + n > 64) {
          q_drain<RUN, PC, LIST>(q.tab, q.lo, q.base, q.run_ent, q.ms16, q.ml16, q.cap, q.pad, q.lcnt, qn, run0, q.lane,
                                 q.lst, q.lim);
          qn = 0;
        }
        if (acc == 0) {
          const uint32_t slot =
              qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          char *sp = q.pad + slot * kQPad + 64;
          *reinterpret_cast<uint64_t *>(sp) = hb;
          *reinterpret_cast<uint32_t *>(sp + 8) = (q.lane << 16) | (off + 4 * (d - (kQBlkDw - 1)));
        }
        qn += n;
      }
      acc = 0xffffffffu;
      hb = h;
    }
  }
}

// A tile's RPT (16, 32 or 64; run0 a multiple of it) runs into the candidate
// bitmaps: bits [run0 % 64, + RPT) of word pair run0 / 64, by one vector store
// per plane of the matching width.
template <int RPT>
__device__ __forceinline__ void store_run_bits(uint64_t *bits, uint64_t run0, uint64_t bs, uint64_t bl) {
  const uint64_t w = run0 >> 6;
  if constexpr (RPT == 64) {
    bits[2 * w] = bs;
    bits[2 * w + 1] = bl;
  } else if constexpr (RPT == 32) {
    uint32_t *p = reinterpret_cast<uint32_t *>(bits) + 4 * w + ((run0 >> 5) & 1);
    p[0] = (uint32_t)bs;
    p[2] = (uint32_t)bl;
  } else {
    static_assert(RPT == 16, "16, 32 or 64 runs per tile");
    uint16_t *p = reinterpret_cast<uint16_t *>(bits) + 8 * w + ((run0 >> 4) & 3);
    p[0] = (uint16_t)bs;
    p[4] = (uint16_t)bl;
  }
}

// CW (cold warm-up): a piece starts from h = 0 instead of re-reading the 48
// bytes before it; its first 48 bytes stay in registers and are re-walked at
// the end of the tile from the previous lane's final hash (the state after
// the previous piece), so the previous piece's last line is fetched once.
// Lane 0 still warms up from memory (the previous tile is another wave's).
//
// LIST (run-list mode, small-file calls): tile t is the RPT runs
// W.run_list[RPT t, + RPT) instead of the contiguous runs RPT t.. -- the runs
// some chunk window can reach (a file's first min_size - 64 bytes never are:
// cut_gear starts hashing at min_size, v2020), so the bytes of every file
// below min_size and every file's head are not scanned.  Each lane warms up
// from the 48 bytes before its piece (pieces of consecutive list entries need
// not be adjacent); the runs' bitmap bits are set with atomics (words zeroed
// by k_run_list); the arena's partial last run is the tail (scan_run_coop).
template <int RUN, int PC, bool CW, bool LIST = false>
__global__ __launch_bounds__(1024, 4) void k_scan_q(Work W, DevParams P, uint64_t tile0, uint64_t tile1,
                                                   int do_tail) {
  static_assert(!LIST || (PC == 2 && !CW), "list mode: two warm pieces per run");
  // + one 8-byte slot per wave: lane 0's warm-up hash waits there for the
  // tile-end re-walk (CW) instead of holding two VGPRs across the tile
  __shared__ __attribute__((aligned(16))) uint64_t smem[(kSTab + 16 * kQWaveBytes) / 8 + 16];
  if constexpr (PC == 2 && !CW) MCDC_VGPR_PAD(112);  // 112 used: not an exact fill (MCDC_VGPR_PAD)
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) smem[i] = W.gear16[i >> 5];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR
  QScan q;
  q.lst = nullptr;
  q.lim = 0;
  q.tab = smem;
  q.lo = (lane & 31) << 3;
  q.lane = lane;
  q.pf = to_vgpr(P.pf_hi);
  q.cap = P.cap;
  q.ms16 = P.ms16;
  q.ml16 = P.ml16;
  q.pad = reinterpret_cast<char *>(smem) + kSTab + wv * kQWaveBytes;
  q.lcnt = reinterpret_cast<uint32_t *>(q.pad + kQPadBytes);
  q.base = W.base;
  q.run_ent = W.run_ent;
  q.lcnt[lane] = 0;
  q.lcnt[64 + lane] = 0xffffffffu;
  q.lcnt[128 + lane] = 0xffffffffu;
  // the call's error / dirty / hand-back words start at zero (the first part's
  // launch clears them: no memset launch on the resolution's critical path)
  if (tile0 == 0 && blockIdx.x == 0 && threadIdx.x < 8) W.err[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  // wave index, CU-major: the first gridDim.x tiles of a static round land on
  // different CUs (a launch with fewer tiles than waves then uses every CU)
  const uint64_t wid = (uint64_t)wv * gridDim.x + blockIdx.x;
  constexpr int SUB = RUN / PC, RPT = 64 / PC;  // bytes per lane piece, runs per tile
  const uint64_t nfull = W.n_al / RUN;
  const uint64_t ntiles_full = nfull / RPT;
  if (!LIST && tile1 > ntiles_full) tile1 = ntiles_full;
  constexpr int G = SUB / 64;
  static_assert(G % 2 == 0, "even group count");
  const uint32_t qi = lane >> 2, qj = lane & 3;
  // load k: lane (4i+j) fetches piece j of run 4i+k; it lands in the pad at run*80 + 16j
  char *wr = q.pad + 4 * qi * kQPad + 16 * qj;
  const char *rd = q.pad + lane * kQPad;
  const uint32_t o0 = 4 * qi * SUB + 16 * qj;  // lane's byte offset in the tile for load 0, group 0
  // Tiles are handed out either statically (wave w: tiles w, w + nwaves, ...)
  // or, with W.tile_ctr, in request order from one atomic counter: waves that
  // run fast take more tiles, so the launch ends without a ragged last round.
  // The next index is requested when a tile starts, so its latency is hidden.
  // (static when every wave gets at most one tile: nothing to balance)
  // With first_static the first tile of every wave is its static one and the
  // counter hands out tiles from tile0 + nwaves on: the launch does not start
  // with every wave queued on one atomic before its first load.
  const bool dyn = W.tile_ctr != nullptr && tile1 - tile0 > nwaves;
  const uint64_t dyn0 = tile0 + (W.first_static ? nwaves : 0);
  auto grab = [&]() -> uint64_t {
    uint64_t v = 0;
    if (lane == 0) v = atomicAdd(reinterpret_cast<unsigned long long *>(W.tile_ctr), 1ull);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return dyn0 + (((uint64_t)hi << 32) | lo);
  };
  // The runs of the partial last tile (< 64) are taken first, one per wave
  // (scan_run_coop), so they overlap the full tiles instead of trailing them
  // (a 1.3 GB call: scan 0.80 -> ~0.4 ms).
  if (do_tail) {  // one wave per run, the last waves first (in a static round they have the fewest tiles)
    const uint64_t nruns = (W.n_al + RUN - 1) / RUN;
    for (uint64_t run = (LIST ? nfull : ntiles_full * RPT) + (nwaves - 1 - wid); run < nruns; run += nwaves)
      scan_run_coop(q.tab, q.lo, W, P, run, lane);
  }
  uint64_t t = dyn && !W.first_static ? grab() : tile0 + wid;
  while (t < tile1) {
    const uint64_t t_next = dyn ? grab() : t + nwaves;
    const uint64_t run0 = t * RPT;
    uint64_t piece = t * 64 + lane;
    uint64_t ra = 0, rb = 0;  // list mode: this lane quad's two runs (pieces 4 qi .. 4 qi + 3), byte offsets
    if constexpr (LIST) {
      q.lst = W.run_list + run0;
      q.lim = (uint32_t)min<uint64_t>(RPT, W.list_n - run0) - 1;
      piece = (uint64_t)q.lst[min(lane / PC, q.lim)] * PC + lane % PC;
      ra = (uint64_t)q.lst[min(2 * qi, q.lim)] * RUN + 16 * qj;
      rb = (uint64_t)q.lst[min(2 * qi + 1, q.lim)] * RUN + 16 * qj;
    }
    uint64_t h = 0, hw = 0;
    if (piece > 0 && (!CW || lane == 0)) {  // warm-up: the 48 bytes before the piece complete every window
      const uint4 *p = reinterpret_cast<const uint4 *>(W.base + piece * (uint64_t)SUB);
      const uint4 w0 = p[-3], w1 = p[-2], w2 = p[-1];
      hash16(q.tab, q.lo, w0, hw);
      hash16(q.tab, q.lo, w1, hw);
      hash16(q.tab, q.lo, w2, hw);
    }
    if (!CW) h = hw;
    else if (lane == 0) smem[(kSTab + 16 * kQWaveBytes) / 8 + wv] = hw;
    uint4 f0, f1, f2;  // CW: the piece's first 48 bytes
    uint32_t qn = 0;  // wave-uniform queue length
    const uint8_t *tb = W.base + run0 * (uint64_t)RUN;  // wave-uniform tile base (SGPR)
#define MCDC_LDQ(k, gg)                                                                                     \
  (LIST ? *reinterpret_cast<const uint4 *>(W.base + ((k) < 2 ? ra : rb) + ((k) & 1) * SUB + 64 * (gg))       \
        : *reinterpret_cast<const uint4 *>(tb + (uint64_t)(uint32_t)(o0 + (k) * SUB + 64 * (gg))))
    uint4 a0 = MCDC_LDQ(0, 0), a1 = MCDC_LDQ(1, 0), a2 = MCDC_LDQ(2, 0), a3 = MCDC_LDQ(3, 0);
    uint4 b0 = MCDC_LDQ(0, 1), b1 = MCDC_LDQ(1, 1), b2 = MCDC_LDQ(2, 1), b3 = MCDC_LDQ(3, 1);
#pragma unroll 1
    for (int g = 0; g < G; g += 2) {
      {
        *reinterpret_cast<uint4 *>(wr) = a0;
        *reinterpret_cast<uint4 *>(wr + kQPad) = a1;
        *reinterpret_cast<uint4 *>(wr + 2 * kQPad) = a2;
        *reinterpret_cast<uint4 *>(wr + 3 * kQPad) = a3;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(rd);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(rd + 16);
        const uint4 c2 = *reinterpret_cast<const uint4 *>(rd + 32);
        const uint4 c3 = *reinterpret_cast<const uint4 *>(rd + 48);
        const uint32_t w[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                                c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
        if (CW && g == 0) { f0 = c0; f1 = c1; f2 = c2; }
        scan64q<RUN, PC, 16, LIST>(q, w, h, 64u * g, qn, run0, CW && g == 0);
      }
      {
        *reinterpret_cast<uint4 *>(wr) = b0;
        *reinterpret_cast<uint4 *>(wr + kQPad) = b1;
        *reinterpret_cast<uint4 *>(wr + 2 * kQPad) = b2;
        *reinterpret_cast<uint4 *>(wr + 3 * kQPad) = b3;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(rd);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(rd + 16);
        const uint4 c2 = *reinterpret_cast<const uint4 *>(rd + 32);
        const uint4 c3 = *reinterpret_cast<const uint4 *>(rd + 48);
        // both 64-byte halves of the next 128-byte lines are requested back
        // to back (groups g+2, g+3): requesting them a step apart let L2 evict
        // the line in between (+12 % fabric reads, FETCH_SIZE calibrated
        // against the bare load pattern in tools/scanbench quadread)
        const int ga = g + 2 < G ? g + 2 : G - 1, gb = g + 3 < G ? g + 3 : G - 1;  // clamped
        a0 = MCDC_LDQ(0, ga); b0 = MCDC_LDQ(0, gb); a1 = MCDC_LDQ(1, ga); b1 = MCDC_LDQ(1, gb);
        a2 = MCDC_LDQ(2, ga); b2 = MCDC_LDQ(2, gb); a3 = MCDC_LDQ(3, ga); b3 = MCDC_LDQ(3, gb);
        const uint32_t w[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                                c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
        scan64q<RUN, PC, 16, LIST>(q, w, h, 64u * (g + 1), qn, run0);
      }
    }
#undef MCDC_LDQ
    if (CW) {  // re-walk the first 48 positions from the state after the previous piece
      const uint32_t plo = __shfl_up((uint32_t)h, 1u), phi = __shfl_up((uint32_t)(h >> 32), 1u);
      uint64_t hp = lane == 0 ? smem[(kSTab + 16 * kQWaveBytes) / 8 + wv] : (((uint64_t)phi << 32) | plo);
      const uint32_t w[12] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w, f2.x, f2.y, f2.z, f2.w};
      scan64q<RUN, PC, 12>(q, w, hp, 0u, qn, run0);
    }
    if (qn)
      q_drain<RUN, PC, LIST>(q.tab, q.lo, q.base, q.run_ent, q.ms16, q.ml16, q.cap, q.pad, q.lcnt, qn, run0, lane,
                             q.lst, q.lim);
    const uint32_t cnt = q.lcnt[lane], fs = q.lcnt[64 + lane], fl = q.lcnt[128 + lane];
    q.lcnt[lane] = 0;
    q.lcnt[64 + lane] = 0xffffffffu;
    q.lcnt[128 + lane] = 0xffffffffu;
    if constexpr (LIST) {  // (entries past the list's end repeat its last run: written once, by its own lane)
      if (lane <= q.lim) {
        const uint64_t run = q.lst[lane];
        W.run_cnt[run] = cnt > q.cap ? kRunOverflow : (uint8_t)cnt;
        W.run_sum[run] = run_summary(cnt, fs, fl);
        uint32_t *b32 = reinterpret_cast<uint32_t *>(W.run_bits) + 4 * (run >> 6) + ((run >> 5) & 1);
        if (fs != 0xffffffffu) atomicOr(b32, 1u << (run & 31));
        if (fl != 0xffffffffu) atomicOr(b32 + 2, 1u << (run & 31));
      }
      t = t_next;
      continue;
    }
    const bool mine = PC == 1 || lane < RPT;
    if (mine) {
      const uint64_t run = run0 + lane;
      W.run_cnt[run] = cnt > q.cap ? kRunOverflow : (uint8_t)cnt;
      W.run_sum[run] = run_summary(cnt, fs, fl);
    }
    {  // the tile's runs in the candidate bitmaps: RPT bits per plane, one store each
      const uint64_t bs = __ballot(mine && fs != 0xffffffffu), bl = __ballot(mine && fl != 0xffffffffu);
      if (lane == 0) store_run_bits<RPT>(W.run_bits, run0, bs, bl);
    }
    t = t_next;
  }
}

// The list-mode scan's run list: entry i = {first run, list index} of up to 64
// consecutive runs (the host merges and splits the files' ranges), written
// one thread per entry; the same grid zeroes the candidate-bitmap words and
// the tile counter after them (the scan sets the listed runs' bits with atomics).
__global__ void k_run_list(const uint2 *ent, uint64_t nent, uint64_t list_n, uint32_t *list, uint64_t *words,
                           uint64_t nwords) {
  MCDC_VGPR_PAD(16);  // (not an exact fill)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nent) {  // (nent = 0: the zeroing only)
    const uint2 e = ent[i];
    const uint64_t p1 = i + 1 < nent ? ent[i + 1].y : list_n;
    for (uint64_t j = e.y; j < p1; ++j) list[j] = e.x + (uint32_t)(j - e.y);
  }
  for (uint64_t k = i; k < nwords; k += (uint64_t)gridDim.x * blockDim.x) words[k] = 0;
}

void launch_run_list(const uint32_t *ent, uint64_t nent, uint64_t list_n, uint32_t *list, uint64_t *words,
                     uint64_t nwords, hipStream_t stream, hipEvent_t ev0) {
  const uint64_t n = std::max<uint64_t>(std::max(nent, std::min<uint64_t>(nwords, 65536)), 1);
  hipExtLaunchKernelGGL(k_run_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ev0, nullptr, 0,
                        reinterpret_cast<const uint2 *>(ent), nent, list_n, list, words, nwords);
}

// The segment plan of a batch on the GPU (run_pipeline, a new layout of many
// files): from the files' arena extents fs[i], fe[i], per file nseg =
// ceil(len / Z) segments of Z bytes (the last shorter), each with room for
// len / (min_size - 1) + 2 chain nodes, as the host plan builds them.  Two
// kernels: per-block sums of the segment and node counts, then per file its
// prefix (the sums of the blocks before its own, then a block scan) and its
// File, Seg and node_off records (node_off[first + nseg] too: the next file's
// first entry, or node_off[nsegs]).
__device__ __forceinline__ void plan_counts(uint64_t len, uint64_t Z, uint64_t ms1, uint64_t &nseg, uint64_t &nodes) {
  nseg = (len + Z - 1) / Z;
  nodes = nseg ? (nseg - 1) * (Z / ms1 + 2) + (len - (nseg - 1) * Z) / ms1 + 2 : 0;
}

__device__ __forceinline__ void block_sum2(uint64_t &a, uint64_t &b, uint64_t *sh) {  // (256 threads; a, b -> totals)
  const uint32_t t = threadIdx.x;
  sh[t] = a;
  sh[256 + t] = b;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (t < o) {
      sh[t] += sh[t + o];
      sh[256 + t] += sh[256 + t + o];
    }
    __syncthreads();
  }
  a = sh[0];
  b = sh[256];
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_plan_count(const uint64_t *fs, const uint64_t *fe, uint64_t n, uint64_t Z,
                                                     uint64_t ms1, uint64_t *bsum) {
  __shared__ uint64_t sh[512];
  MCDC_VGPR_PAD(16);  // (not an exact fill)
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t ns = 0, nd = 0;
  if (i < n) plan_counts(fe[i] - fs[i], Z, ms1, ns, nd);
  block_sum2(ns, nd, sh);
  if (threadIdx.x == 0) {
    bsum[2 * blockIdx.x] = ns;
    bsum[2 * blockIdx.x + 1] = nd;
  }
}

__global__ __launch_bounds__(256) void k_plan_write(const uint64_t *fs, const uint64_t *fe, uint64_t n, uint64_t Z,
                                                     uint64_t ms1, const uint64_t *bsum, File *files, Seg *segs,
                                                     uint64_t *node_off) {
  __shared__ uint64_t sh[512];
  MCDC_VGPR_PAD(24);  // (not an exact fill)
  const uint32_t t = threadIdx.x;
  // the blocks before this one
  uint64_t bs = 0, bn = 0;
  for (uint32_t b = t; b < blockIdx.x; b += 256) {
    bs += bsum[2 * b];
    bn += bsum[2 * b + 1];
  }
  block_sum2(bs, bn, sh);
  const uint64_t i = (uint64_t)blockIdx.x * 256 + t;
  uint64_t ns = 0, nd = 0, a = 0, e = 0;
  if (i < n) {
    a = fs[i];
    e = fe[i];
    plan_counts(e - a, Z, ms1, ns, nd);
  }
  // inclusive block scan of (ns, nd), Hillis-Steele
  sh[t] = ns;
  sh[256 + t] = nd;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    const uint64_t xs = t >= o ? sh[t - o] : 0, xn = t >= o ? sh[256 + t - o] : 0;
    __syncthreads();
    sh[t] += xs;
    sh[256 + t] += xn;
    __syncthreads();
  }
  if (i >= n) return;
  const uint64_t first = bs + sh[t] - ns, node0 = bn + sh[256 + t] - nd;
  files[i] = File{a, e, (uint32_t)first, (uint32_t)ns};
  const uint64_t full = Z / ms1 + 2;
  for (uint64_t k = 0; k < ns; ++k) {
    Seg S;
    S.start = a + k * Z;
    S.end = k + 1 < ns ? S.start + Z : e;
    S.file = (uint32_t)i;
    S.flags = (k == 0 ? kSegFirst : 0u) | (k + 1 == ns ? kSegLast : 0u);
    segs[first + k] = S;
    node_off[first + k] = node0 + k * full;
  }
  node_off[first + ns] = node0 + nd;
}

void launch_plan(const uint64_t *fse, uint64_t n, uint64_t Z, uint64_t ms1, uint64_t *bsum, File *files, Seg *segs,
                 uint64_t *node_off, hipStream_t stream) {
  if (n == 0) return;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_plan_count, dim3(blocks), dim3(256), 0, stream, fse, fse + n, n, Z, ms1, bsum);
  hipLaunchKernelGGL(k_plan_write, dim3(blocks), dim3(256), 0, stream, fse, fse + n, n, Z, ms1, bsum, files, segs,
                     node_off);
}

// Product configuration: quad-coalesced scan, 16 waves (one 1024-thread
// block) per CU; tools/scanbench.hip keeps the lane-strided k_scan_t variants
// for comparison.
// Tiles are in units of 64 / pieces runs (pieces = lane pieces per run).
void launch_scan(const Work &w, const DevParams &p, int num_cus, hipStream_t stream, uint64_t tile0,
                 uint64_t tile1, bool tail, int pieces, bool cold, hipEvent_t ev0, hipEvent_t ev1) {
  const uint64_t rpt = 64 / (uint64_t)pieces;
  const uint64_t ntiles = tail ? (w.nruns + rpt - 1) / rpt - tile0 : tile1 - tile0;
  uint64_t blocks = ntiles;  // one block per CU up to the CU count (156 KiB LDS -> 1 block/CU)
  const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256);
  if (blocks > cap) blocks = cap;
  if (blocks == 0) {  // (no launch: the events still mark this point of the stream)
    if (ev0) (void)hipEventRecord(ev0, stream);
    if (ev1) (void)hipEventRecord(ev1, stream);
    return;
  }
  const int t = tail ? 1 : 0;
  const dim3 gr((unsigned)blocks), bl(1024);
  if (w.run_list) {  // list mode (tile1: the list's tiles of 32 runs; tail: the partial last run)
    hipExtLaunchKernelGGL((k_scan_q<kRun, 2, false, true>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
  } else if (cold && pieces != 1) {  // (one piece: the saved bytes would spill, 128 VGPRs)
    if (pieces == 4) hipExtLaunchKernelGGL((k_scan_q<kRun, 4, true>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
    else hipExtLaunchKernelGGL((k_scan_q<kRun, 2, true>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
  } else {
    if (pieces == 4) hipExtLaunchKernelGGL((k_scan_q<kRun, 4, false>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
    else if (pieces == 2) hipExtLaunchKernelGGL((k_scan_q<kRun, 2, false>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
    else hipExtLaunchKernelGGL((k_scan_q<kRun, 1, false>), gr, bl, 0, stream, ev0, ev1, 0, w, p, tile0, tile1, t);
  }
}

// Lane pieces per run for a whole-call scan of nruns_full full runs.  A tile
// (64 lane pieces) is 256 KiB at one piece per run, 128 KiB at two.  Measured
// (tools/pieces_big.py, device time, first tiles static): two pieces are
// faster at every size from 0.25 to 64 GiB (64 GiB 12.48 -> 12.37 ms; 80 000
// small files 0.57 -> 0.52 ms; 2 GiB -9 %) except a call of more than half
// and at most one round of one-piece tiles (1 GiB: 0.24 vs 0.28 ms); four
// pieces (48-byte warm-up per KiB) never won.
int scan_pieces(uint64_t nruns_full, int num_cus) {
  const uint64_t waves = 16ull * (uint64_t)(num_cus > 0 ? num_cus : 256);
  const uint64_t tiles1 = nruns_full / 64;  // tiles at one piece per run
  return (tiles1 * 2 > waves && tiles1 <= waves) ? 1 : 2;
}

uint64_t scan_waves(uint64_t ntiles, int num_cus) {
  uint64_t blocks = ntiles;
  const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256);
  return 16 * (blocks > cap ? cap : blocks);
}

// ===================================================== chain walking =====
// First candidate of run r in [lo, hi) recomputed from bytes (overflowed run).
__device__ uint64_t run_first_hit(const Work &W, const DevParams &P, const uint64_t *gt, uint64_t r,
                                  uint64_t lo, uint64_t hi, uint64_t cce) {
  const uint64_t rs = r * (uint64_t)kRun, rend = rs + kRun;
  const uint64_t s = rs > lo ? rs : lo, e = rend < hi ? rend : hi;
  if (s >= e) return ~0ull;
  uint64_t h = 0;
  for (uint64_t q = s - (kWin - 1); q < e; ++q) {  // s >= lo = t + 47
    h = (h << 1) + gt[W.base[q]];
    if (q >= s) {
      const uint64_t m = q < cce ? P.ms : P.ml;
      if ((h & m) == 0) return q;
    }
  }
  return ~0ull;
}

// First candidate of one run in [lo, hi) from its (up to 8, cap == 8) entries;
// entries are not position-sorted, so take the minimum.  ~0 if none.
__device__ __forceinline__ uint32_t rel_clamp(uint64_t x, uint64_t rb) {
  return x <= rb ? 0u : (x - rb >= (uint64_t)kRun ? (uint32_t)kRun : (uint32_t)(x - rb));
}

// In run-relative 32-bit coordinates: entries 0-3 preloaded, 4-7 loaded here
// only when the run has more than 4 (rare on real data).
__device__ __forceinline__ uint64_t run_first_entry(uint64_t r, uint32_t cnt, const uint4 ea,
                                                    const uint4 *eb_ptr, uint64_t lo, uint64_t hi,
                                                    uint64_t cce) {
  const uint64_t rb = r * (uint64_t)kRun;
  const uint32_t l = rel_clamp(lo, rb), h = rel_clamp(hi, rb), m = rel_clamp(cce, rb);
  uint32_t best = 0xffffffffu;
  auto take = [&](uint32_t i, uint32_t e) {
    const uint32_t off = e & 0x00ffffffu;
    const uint32_t kind = off < m ? (e >> 31) : (e >> 30) & 1u;
    if (i < cnt && off >= l && off < h && kind) best = min(best, off);
  };
  take(0, ea.x); take(1, ea.y); take(2, ea.z); take(3, ea.w);
  if (cnt > 4) {
    const uint4 eb = *eb_ptr;
    take(4, eb.x); take(5, eb.y); take(6, eb.z); take(7, eb.w);
  }
  return best == 0xffffffffu ? ~0ull : rb + best;
}

// First candidate of run r in [lo, hi) whatever the run's state: recomputed
// from bytes when it overflowed, from the preloaded entries when cap == 8,
// else from its entry list.
__device__ __forceinline__ uint64_t run_first(const Work &W, const DevParams &P, const uint64_t *gt, uint64_t r,
                                              uint32_t cnt, const uint4 ea, uint64_t lo, uint64_t hi,
                                              uint64_t cce) {
  if (cnt == 0) return ~0ull;
  if (cnt > P.cap) return run_first_hit(W, P, gt, r, lo, hi, cce);
  if (P.cap == 8)
    return run_first_entry(r, cnt, ea, reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull) + 1, lo, hi, cce);
  uint64_t found = ~0ull;
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint32_t e = W.run_ent[r * (uint64_t)P.cap + i];
    const uint64_t pos = r * (uint64_t)kRun + (e & 0x00ffffffu);
    if (pos >= lo && pos < hi && pos < found) {
      const bool ok = pos < cce ? (e >> 31) & 1 : (e >> 30) & 1;
      if (ok) found = pos;
    }
  }
  return found;
}

// A group of GS lanes (64: the whole wave; 16: a DPP row, four chains per
// wave) walks one chain.  All control flow below is group-uniform.
template <int GS>
struct Group {
  uint32_t gl, gb;  // lane within the group, first lane of the group
  __device__ __forceinline__ Group() {
    const uint32_t l = lane_id();
    gl = l & (GS - 1);
    gb = l & ~(uint32_t)(GS - 1);
  }
  __device__ __forceinline__ uint64_t ballot(bool p) const {
    const uint64_t m = __ballot(p);
    if constexpr (GS == 64) return m;
    else return (m >> gb) & ((1ull << GS) - 1);
  }
  __device__ __forceinline__ uint64_t bcast(uint64_t v, uint32_t src) const { return shfl64(v, (int)(gb + src)); }
  __device__ __forceinline__ uint64_t up(uint64_t v, unsigned d) const {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, GS);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, GS);
    return ((uint64_t)hi << 32) | lo;
  }
  // GS == 16 (a DPP row): v of lane gl - D, 0 for gl < D — DPP row_shr (a VALU
  // move, no LDS crossbar round trip like ds_bpermute)
  template <int D>
  __device__ __forceinline__ uint64_t up0(uint64_t v) const {
    static_assert(GS == 16 && D >= 1 && D <= 15, "row shift");
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x110 | D, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x110 | D, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
  }
  // GS == 16: minimum over the row, in every lane (DPP row_ror butterfly)
  __device__ __forceinline__ uint32_t row_min_u32(uint32_t v) const {
    static_assert(GS == 16, "row reduction");
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // row_ror:8
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false));  // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false));  // row_ror:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false));  // row_ror:1
    return v;
  }
};

// Candidate search of one run in chunk-relative int32 coordinates (positions
// minus c; every window lies within max <= 16 MiB of c): the first entry in
// [lo_r, hi_r) that is an S candidate before cce_r or an L candidate after it.
// Entries 0-3 preloaded, 4-7 loaded only for a run holding more than four.
__device__ __forceinline__ int32_t run_first_rel(uint32_t cnt, const uint4 ea, const uint4 *eb_ptr, int32_t rbase,
                                                 int32_t lo_r, int32_t hi_r, int32_t cce_r) {
  int32_t best = INT32_MAX;
  auto take = [&](uint32_t i, uint32_t e) {
    const int32_t p = rbase + (int32_t)(e & 0x00ffffffu);
    const uint32_t kind = p < cce_r ? (e >> 31) : ((e >> 30) & 1u);
    if (i < cnt && p >= lo_r && p < hi_r && kind) best = min(best, p);
  };
  take(0, ea.x); take(1, ea.y); take(2, ea.z); take(3, ea.w);
  if (cnt > 4) {
    const uint4 eb = *eb_ptr;
    take(4, eb.x); take(5, eb.y); take(6, eb.z); take(7, eb.w);
  }
  return best;
}

// next(c): the chunk starting at arena position c (file ends at fend) ends
// where fastcdc's cut_gear(&file[c..], min, avg, max, masks) says.  Called by
// a whole group with group-uniform c, fend; returns the next chunk start.
// Lane gl owns restart positions [PPL*gl, PPL*gl + PPL) and, per 64-run batch,
// runs [RPL*gl, RPL*gl + RPL).  Latency shape: two dependent global levels per
// step — {restart-window bytes, the first 64 runs' candidate counts}, then
// {entries of the non-empty runs}; GEAR comes from the block's LDS copy `gt`.
// Window arithmetic is 32-bit relative to c; only overflowed runs and the
// general entry lists (cap != 8) use absolute 64-bit positions.
template <int GS>
__device__ uint64_t group_next(const Group<GS> &G, const Work &W, const DevParams &P, const uint64_t *gt,
                               uint64_t c, uint64_t fend) {
  constexpr int PPL = (kWin - 1 + GS - 1) / GS;  // 1 (GS 64), 2 (32), 3 (16)
  constexpr int RPL = 64 / GS;
  const uint64_t rem = fend - c;
  if (rem <= P.min) return fend;                  // remaining <= min_size: whole tail
  // crate: center = avg, remaining = rem; rem > max -> remaining = max, else rem < avg -> center = rem
  const uint32_t remaining = rem > P.max ? P.max : (uint32_t)rem;
  const uint32_t center = (rem <= P.max && rem < P.avg) ? (uint32_t)rem : P.avg;
  const uint32_t t0 = P.min / 2 * 2, ce = center / 2 * 2, re = remaining / 2 * 2;
  if (re <= t0) return c + remaining;             // loop never runs: forced
  const uint64_t t = c + t0;
  const uint32_t wlen = min(re - t0, (uint32_t)(kWin - 1));
  const int32_t lo_r = (int32_t)(t0 + kWin - 1), hi_r = (int32_t)re, cce_r = (int32_t)ce;
  const bool cand = lo_r < hi_r;
  const uint64_t r0 = (c + (uint64_t)lo_r) / kRun, r1 = cand ? (c + (uint64_t)hi_r - 1) / kRun : 0;
  const int32_t base0 = (int32_t)((int64_t)(r0 * (uint64_t)kRun) - (int64_t)c);  // run r0's start - c
  // level 1: each lane's runs' summaries (first S / first L candidate); the
  // entry lists are read only for a run that a window boundary splits
  uint32_t sm[RPL];
  auto load_batch = [&](uint64_t rb) {
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const uint64_t r = rb + RPL * G.gl + k;
      sm[k] = (cand && r <= r1) ? W.run_sum[r] : 0u;
    }
  };
  // ---- level-1 loads, all independent
  uint32_t by[PPL];
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const uint32_t idx = PPL * G.gl + k;
    by[k] = idx < wlen ? W.base[t + idx] : 0;
  }
  load_batch(r0);
  // ---- (1) exact restarted hash for the first <= 47 tested positions
  uint64_t loc[PPL], acc = 0;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const uint32_t idx = PPL * G.gl + k;
    acc = (acc << 1) + (idx < wlen ? gt[by[k]] : 0);
    loc[k] = acc;
  }
  uint64_t x = acc;  // hash at this lane's last position: shift-scan over the group
  uint64_t excl;     // hash at the previous lane's last position
  if constexpr (GS == 16) {
    x += G.template up0<1>(x) << PPL;
    x += G.template up0<2>(x) << (2 * PPL);
    x += G.template up0<4>(x) << (4 * PPL);
    x += G.template up0<8>(x) << (8 * PPL);
    excl = G.template up0<1>(x);
  } else {
#pragma unroll
    for (unsigned d = 1; d < (unsigned)GS; d <<= 1) {
      const uint64_t v = G.up(x, d);
      if (G.gl >= d) x += v << (PPL * d);
    }
    excl = G.up(x, 1);
    if (G.gl == 0) excl = 0;
  }
  uint32_t first = 0xffffffffu;
#pragma unroll
  for (int k = PPL - 1; k >= 0; --k) {
    const uint32_t idx = PPL * G.gl + k;
    const uint64_t h = (excl << (k + 1)) + loc[k];
    if (idx < wlen && (h & ((t0 + idx < ce) ? P.ms : P.ml)) == 0) first = idx;
  }
  if constexpr (GS == 16) {  // lanes own increasing positions: the first hit is the row minimum
    const uint32_t m = G.row_min_u32(first);
    if (m != 0xffffffffu) return t + m;
  } else {
    const uint64_t b = G.ballot(first != 0xffffffffu);
    if (b) return t + G.bcast(first, (uint32_t)(__ffsll((unsigned long long)b) - 1));
  }
  if (!cand) return c + remaining;
  // ---- (2) windowed candidates for [t + 47, c + re), 64 runs per batch
  const int32_t s_end = min(cce_r, hi_r), l_beg = max(lo_r, cce_r);  // S tested before cce, L from it
  for (uint64_t rb = r0; rb <= r1; rb += 64) {
    if (rb != r0) load_batch(rb);
    int32_t found = INT32_MAX;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const uint32_t u = sm[k];
      if (found != INT32_MAX || u == 0) continue;
      const uint64_t r = rb + RPL * G.gl + k;
      const int32_t rbase = base0 + (int32_t)((r - r0) * (uint64_t)kRun);
      const uint32_t nc = u >> 28, fs1 = u & 0x3fffu, fl1 = (u >> 14) & 0x3fffu;
      // The run's first S candidate is the first in [lo, s_end) unless it lies
      // before lo and others follow; likewise its first L for [l_beg, hi).
      int32_t res = INT32_MAX;
      bool split = (fs1 | fl1) == 0;  // "unknown" (an overflowed lane-strided run)
      if (fs1) {
        const int32_t p = rbase + (int32_t)fs1 - 1;
        if (p >= lo_r && p < s_end) res = p;
        else split = p < lo_r && nc >= 2 && lo_r < s_end;
      }
      if (res == INT32_MAX && !split && fl1) {
        const int32_t p = rbase + (int32_t)fl1 - 1;
        if (p >= l_beg && p < hi_r) res = p;
        else split = p < l_beg && nc >= 2 && l_beg < hi_r;
      }
      if (split) {  // rare: the entry list (or, overflowed, the bytes) decides
        const uint32_t cnt = W.run_cnt[r];
        if (cnt <= P.cap && P.cap == 8) {
          const uint4 ea = *reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull);
          res = run_first_rel(cnt, ea, reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull) + 1, rbase, lo_r,
                              hi_r, cce_r);
        } else {
          const uint64_t f = run_first(W, P, gt, r, cnt, make_uint4(0, 0, 0, 0), c + (uint64_t)lo_r,
                                       c + (uint64_t)hi_r, c + (uint64_t)cce_r);
          if (f != ~0ull) res = (int32_t)(f - c);
        }
      }
      found = res;
    }
    if constexpr (GS == 16) {  // (found >= 0 or INT32_MAX: unsigned order = signed order)
      const uint32_t m = G.row_min_u32((uint32_t)found);
      if (m != (uint32_t)INT32_MAX) return c + (uint64_t)m;
    } else {
      const uint64_t fb = G.ballot(found != INT32_MAX);
      if (fb) return c + (uint64_t)G.bcast((uint64_t)(uint32_t)found, (uint32_t)(__ffsll((unsigned long long)fb) - 1));
    }
  }
  return c + remaining;  // forced cut (e.g. all zeros)
}

// Nonzero bytes of x, as bit 7 of each byte.
__device__ __forceinline__ uint32_t nz_bytes(uint32_t x) { return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; }

// Forced stretch.  On data without candidates (zero-filled extents, long runs
// of one byte) every step is a forced cut at max, and chains that entered the
// stretch at different phases never meet; walking it one group_next per chunk
// is what made such inputs slow.  From a chain node c1, count the steps that
// are plain forced cuts: step i (from c_i = c1 + i*max) is one when the file
// continues past c_i + max, no candidate of either kind lies in its window
// [c_i + t0 + 47, c_i + re) and its restart window [c_i + t0, c_i + t0 + 47)
// has no hit.  Candidate-freedom is read at run granularity from run_cnt (a
// non-empty run ends the stretch conservatively), at most kRounds * GS * 64
// runs ahead.  Returns K <= kmax: next(c1 + i*max) == c1 + (i+1)*max, i < K.
template <int GS>
__device__ uint64_t forced_run(const Group<GS> &G, const Work &W, const DevParams &P, const uint64_t *gt,
                               uint64_t c1, uint64_t fend, uint64_t kmax) {
  constexpr int NL = 4;           // 16-run loads per lane per round: GS * 64 runs per round
  constexpr uint32_t kRounds = 4;
  const uint64_t mx = P.max;
  const uint32_t t0 = P.min / 2 * 2, re = P.max / 2 * 2, ce = P.avg / 2 * 2;
  if (kmax == 0 || fend <= c1 + mx || re <= t0 + kWin - 1) return 0;
  uint64_t K = min(kmax, (fend - c1 - mx - 1) / mx + 1);  // steps whose remaining length exceeds max
  // (1) first non-empty run at or after the first window, within the runs the
  // K windows touch
  const uint64_t rA = (c1 + t0 + kWin - 1) / kRun;
  const uint64_t rEnd = min(W.nruns, (c1 + (K - 1) * mx + re + kRun - 1) / kRun);
  uint64_t q = rEnd, rb = rA & ~15ull;
  for (uint32_t round = 0; round < kRounds && rb < rEnd; ++round, rb += (uint64_t)GS * NL * 16) {
    const uint64_t lb = rb + (uint64_t)G.gl * NL * 16;  // this lane: runs [lb, lb + 64)
    uint4 v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k)  // (run_cnt is allocated to a multiple of 16 past nruns)
      v[k] = lb + 16 * k < rEnd ? *reinterpret_cast<const uint4 *>(W.run_cnt + lb + 16 * k) : make_uint4(0, 0, 0, 0);
    uint32_t first = 0xffffffffu;
#pragma unroll
    for (int d = 4 * NL - 1; d >= 0; --d) {  // descending: the lowest non-empty run wins
      const uint4 u = v[d / 4];
      const uint32_t x = (d % 4) == 0 ? u.x : (d % 4) == 1 ? u.y : (d % 4) == 2 ? u.z : u.w;
      const uint64_t r = lb + 4 * d;
      uint32_t m = nz_bytes(x);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (r + b < rA || r + b >= rEnd) m &= ~(0x80u << (8 * b));
      if (m) first = 4 * d + (__builtin_ctz(m) >> 3);
    }
    const uint64_t fb = G.ballot(first != 0xffffffffu);
    if (fb) {
      const uint32_t src = (uint32_t)(__ffsll((unsigned long long)fb) - 1);
      q = rb + (uint64_t)src * NL * 16 + G.bcast(first, src);
      break;
    }
    if (round + 1 == kRounds) q = min(rEnd, rb + (uint64_t)GS * NL * 16);  // horizon: unscanned counts as non-empty
  }
  const uint64_t Q = q * (uint64_t)kRun;  // no candidate in [c1 + t0 + 47, Q)
  if (Q < c1 + re) return 0;
  K = min(K, (Q - c1 - re) / mx + 1);
  // (2) restart windows, GS steps per batch: the first step with a hit ends the stretch
  for (uint64_t i0 = 0; i0 < K; i0 += GS) {
    const uint64_t i = i0 + G.gl;
    bool hit = false;
    if (i < K) {
      const uint64_t t = c1 + i * mx + t0;
      const uint64_t A = t & ~15ull;
      const uint32_t lo = (uint32_t)(t - A);
      uint64_t h = 0;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; ++k) {  // (a rolled outer loop keeps k_link's register count)
        const uint4 u = A + 16 * k < W.n_al ? *reinterpret_cast<const uint4 *>(W.base + A + 16 * k)
                                            : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int bb = 0; bb < 16; ++bb) {
          const uint32_t b = 16 * k + bb;
          const uint32_t w = bb < 4 ? u.x : bb < 8 ? u.y : bb < 12 ? u.z : u.w;
          const uint32_t x = (w >> (8 * (bb % 4))) & 0xffu;
          const bool act = b >= lo && b < lo + (kWin - 1);
          const uint64_t hn = (h << 1) + gt[x];
          h = act ? hn : h;
          const uint64_t m = (t0 + (b - lo) < ce) ? P.ms : P.ml;
          hit |= act && (h & m) == 0;
        }
      }
    }
    const uint64_t hb = G.ballot(hit);
    if (hb) return i0 + (uint64_t)(__ffsll((unsigned long long)hb) - 1);
  }
  return K;
}

// ============================================================ spec =======
__device__ __forceinline__ void load_gear_lds(uint64_t *gt, const Work &W) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) gt[i] = W.gear[i];
  __syncthreads();
}


// One group per segment: the speculative chain of segment s.
template <int GS>
__device__ __forceinline__ void spec_chain(const Group<GS> &G, const Work &W, const DevParams &P, const uint64_t *gt,
                                           uint32_t s) {
  const Seg S = W.segs[s];
  const uint64_t fend = W.files[S.file].end;
  uint64_t *out = W.nodes + W.node_off[s];
  const uint64_t cap = W.node_off[s + 1] - W.node_off[s];
  uint64_t c = S.start, k = 0, exitp = fend;
  for (;;) {
    if (k >= cap) { if (G.gl == 0) atomicOr(W.err, kErrNodeCap); break; }
    if (G.gl == 0) out[k] = c;
    ++k;
    const uint64_t nc = group_next<GS>(G, W, P, gt, c, fend);
    if (nc >= S.end) { exitp = nc; break; }
    c = nc;
  }
  if (G.gl == 0) {
    W.node_cnt[s] = (uint32_t)k;
    W.seg_exit[s] = exitp;
  }
}

template <int GS>
__device__ __forceinline__ void spec_body(Work &W, const DevParams &P, uint32_t s0, uint32_t s1) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const Group<GS> G;
  const uint32_t s = s0 + (blockIdx.x * blockDim.x + threadIdx.x) / GS;
  if (s >= s1) return;
  spec_chain<GS>(G, W, P, gt, s);
}

template <int GS>
__global__ __launch_bounds__(256) void k_spec(Work W, DevParams P, uint32_t s0, uint32_t s1) {
  spec_body<GS>(W, P, s0, s1);
}

// Same, compiled for 6 waves per SIMD (<= 80 VGPRs instead of 82: 5 -> 6
// resident waves per SIMD for a latency-bound chain walk).  The default at
// 16-lane groups; same-box ABAB at 64 GiB: resolution 0.425 -> 0.407 ms.
template <int GS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_spec6(Work W, DevParams P,
                                                                                         uint32_t s0, uint32_t s1) {
  MCDC_VGPR_PAD(80);  // 80 used: not an exact fill (MCDC_VGPR_PAD)
  spec_body<GS>(W, P, s0, s1);
}

// The segments the lane walk handed back (list, *count of them): the group
// walk, grid-stride over the list.
template <int GS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_spec_list(
    Work W, DevParams P, const uint32_t *list, const uint32_t *count) {
  MCDC_VGPR_PAD(80);
  if (*count == 0) return;  // (the common case: nothing handed back)
  __builtin_amdgcn_s_setprio(3);
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const Group<GS> G;
  const uint32_t n = *count, ng = gridDim.x * blockDim.x / GS;
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / GS; i < n; i += ng) spec_chain<GS>(G, W, P, gt, list[i]);
}

// index of c in nodes(j) (sorted), or -1; group-cooperative
template <int GS>
__device__ int find_node(const Group<GS> &G, const Work &W, uint32_t j, uint64_t c) {
  const uint64_t *nd = W.nodes + W.node_off[j];
  const uint32_t n = W.node_cnt[j];
  for (uint32_t b = 0; b < n; b += GS) {
    const uint32_t i = b + G.gl;
    const uint64_t v = i < n ? nd[i] : ~0ull;
    const uint64_t eq = G.ballot(v == c);
    if (eq) return (int)(b + __ffsll((unsigned long long)eq) - 1);
    if (G.ballot(v > c)) return -1;
  }
  return -1;
}

// ============================================================ link =======
// Continuation entries are (first node, repeat count): entry e stands for the
// nodes cont[e] + i*max, i < cont_rep[e] (a forced stretch, forced_run), so a
// continuation crosses a candidate-free extent of any length in a few entries.
// cont_cnt = expanded node count, cont_ent = entries.  `node_cap` bounds the
// expanded count (the staged pipeline's look-ahead assumes <= kContMax steps).
template <int GS>
__device__ __forceinline__ void link_chain(const Group<GS> &G, const Work &W, const DevParams &P, const uint64_t *gt,
                                           uint32_t s, uint64_t node_cap) {
  const Seg S = W.segs[s];
  const File F = W.files[S.file];
  if (S.flags & kSegLast) {
    if (G.gl == 0) {
      W.link_seg[s] = kSegNone; W.link_idx[s] = 0; W.link_pos[s] = F.end; W.cont_cnt[s] = 0; W.cont_ent[s] = 0;
    }
    return;
  }
  uint64_t c = W.seg_exit[s], total = 0;
  uint32_t ents = 0, ls = kSegFail, li = 0;
  uint64_t lp = F.end;
  for (;;) {
    if (c >= F.end) { ls = kSegNone; lp = F.end; break; }
    const uint32_t j = F.first_seg + (uint32_t)((c - F.start) / W.zseg);
    const int idx = find_node<GS>(G, W, j, c);
    if (idx >= 0) { ls = j; li = (uint32_t)idx; lp = c; break; }
    if (ents == (uint32_t)kContMax || total >= node_cap) break;  // give up: serial fallback
    uint64_t nc = group_next<GS>(G, W, P, gt, c, F.end), reps = 1;
    if (nc == c + P.max && nc < F.end) {  // forced cut: extend over the forced stretch behind it
      const uint64_t k = forced_run<GS>(G, W, P, gt, nc, F.end, min(node_cap - total - 1, kRepMax - 1));
      reps += k;
      nc += k * P.max;
    }
    if (G.gl == 0) {
      W.cont[(uint64_t)s * kContMax + ents] = c;
      W.cont_rep[(uint64_t)s * kContMax + ents] = (uint32_t)reps;
    }
    ++ents;
    total += reps;
    c = nc;
  }
  if (G.gl == 0) {
    W.link_seg[s] = ls; W.link_idx[s] = li; W.link_pos[s] = lp;
    W.cont_cnt[s] = (uint32_t)total; W.cont_ent[s] = ents;
    if (ls == kSegFail) atomicOr(&W.file_flags[S.file], kFileFail);
    else if (ls != s + 1) atomicOr(&W.file_flags[S.file], kFileSkip);
    // a long stretch is emitted by k_emit_long (general path only)
    if (ls != kSegFail && total > kEmitInline) {
      W.long_list[atomicAdd(W.long_n, 1u)] = s;
      atomicOr(W.err + 2, 1u);
    }
  }
}

template <int GS>
__global__ __launch_bounds__(256) void k_link(Work W, DevParams P, uint32_t s0, uint32_t s1, uint64_t node_cap) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const Group<GS> G;
  const uint32_t s = s0 + (blockIdx.x * blockDim.x + threadIdx.x) / GS;
  if (s >= s1) return;
  link_chain<GS>(G, W, P, gt, s, node_cap);
}

// The segments whose continuation the lane walk handed back (list, *count).
template <int GS>
__global__ __launch_bounds__(256) void k_link_list(Work W, DevParams P, const uint32_t *list, const uint32_t *count) {
  if (*count == 0) return;  // (the common case: nothing handed back)
  __builtin_amdgcn_s_setprio(3);
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const Group<GS> G;
  const uint32_t n = *count, ng = gridDim.x * blockDim.x / GS;
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / GS; i < n; i += ng)
    link_chain<GS>(G, W, P, gt, list[i], ~0ull);
}

// ======================================================= lane walk =======
// The chain walk with ONE LANE per chain: 64 chains per wave.  The group walk
// above computes every chain-uniform quantity of a step in 16 lanes and the
// four chains of a wave diverge in SALU/exec control: ~90 VALU + ~50 SALU per
// chain step, issue-bound (PMC of k_spec6: 12 % of wave cycles waiting,
// 251 us of a 64 GiB call).  Here a step is ~15 VALU per chain:
//  * the (up to) 47 restart positions: the window's bytes are realigned in
//    registers (v_cndmask + v_alignbyte) and hashed by one unrolled recurrence,
//    GEAR from a 32x replicated LDS copy (one v_perm_b32 per address,
//    conflict-free, as in the scan); the mask test is exact only for a lane
//    whose accumulated test fired (rare) or whose window is irregular;
//  * the windowed candidates from run summaries, 16 runs (4 x uint4) per
//    batch per lane, the next batch loaded while one is evaluated; a run the
//    window starts inside (the S window's first run, the L window's first
//    run) is decided from its entry list when the summary cannot tell.
// A step the lane walk does not take -- a run whose entry list overflowed, a
// continuation of kContMax steps -- hands the whole segment to the group walk
// (k_spec_list / k_link_list), which recomputes it from scratch.

__device__ __forceinline__ void load_gear_rep(uint64_t *tab, const Work &W) {
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = W.gear[i >> 5];
  __syncthreads();
}

// Per-lane select of a or b as one v_perm_b32 (sel from lane_sel): written as
// a ?: on array elements the compiler turns the register realignments below
// into dynamically indexed private arrays (scratch).
__device__ __forceinline__ uint32_t lane_sel(bool take_b) { return take_b ? 0x07060504u : 0x03020100u; }
__device__ __forceinline__ uint32_t sel32(uint32_t a, uint32_t b, uint32_t sel) { return __builtin_amdgcn_perm(b, a, sel); }

// GEAR[byte k of w] from the replicated table (copy lo8 / 8)
#define MCDC_GR(w, k, lo8) lds_gear(tab, __builtin_amdgcn_perm((w), (lo8), 0x0c0c0000u | ((4u + (k)) << 8)))

// The recurrence h = (h << 1) + GEAR[byte i] over N realigned bytes (byte i =
// byte i % 4 of e[i / 4]): step(i, GEAR[byte i]) in order, the LDS lookups
// issued 8 positions ahead of the chain.  Left to itself the compiler issued
// four lookups and waited for them before the next four: 12-16 exposed LDS
// latencies per call; the scheduling barriers keep the issue order.
template <int N, class Step>
__device__ __forceinline__ void gear_chain(const uint64_t *tab, uint32_t lo8, const uint32_t *e, Step &&step) {
  constexpr int D = 8;
  uint64_t g[N];
#pragma unroll
  for (int i = 0; i < D && i < N; ++i) g[i] = MCDC_GR(e[i >> 2], i & 3, lo8);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i + D < N) g[i + D] = MCDC_GR(e[(i + D) >> 2], (i + D) & 3, lo8);
    __builtin_amdgcn_sched_barrier(0);
    step(i, g[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// First candidate of run r in [lo_r, hi_r) (chunk-relative) from its entry
// list, for a run a window edge splits; punt when the list overflowed.
__device__ __forceinline__ int32_t lane_run_split(const Work &W, const DevParams &P, uint64_t r, uint32_t cnt,
                                                  int32_t rbase, int32_t lo_r, int32_t hi_r, int32_t cce_r, bool &punt) {
  if (cnt > P.cap) { punt = true; return INT32_MAX; }
  if (P.cap == 8) {
    const uint4 ea = *reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull);
    return run_first_rel(cnt, ea, reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull) + 1, rbase, lo_r, hi_r,
                         cce_r);
  }
  int32_t best = INT32_MAX;
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint32_t e = W.run_ent[r * (uint64_t)P.cap + i];
    const int32_t p = rbase + (int32_t)(e & 0x00ffffffu);
    const uint32_t kind = p < cce_r ? (e >> 31) : ((e >> 30) & 1u);
    if (p >= lo_r && p < hi_r && kind) best = min(best, p);
  }
  return best;
}

__device__ __forceinline__ uint64_t bits_upto(uint32_t i) { return i == 63 ? ~0ull : ((2ull << i) - 1); }

// First run in [a, b] whose bit is set in plane pl (0: S, 1: L) of the
// candidate bitmaps, ~0 if none.  pw = the word pairs wB and wB + 1, already
// loaded ({S, L} of wB in .x.y / .z.w of p0, of wB + 1 in p1); other words
// (windows past them: max > 252 KiB) are loaded here.
__device__ __forceinline__ uint64_t bit_word(const uint64_t *bits, int pl, uint64_t w, uint64_t wB, const uint4 &p0,
                                             const uint4 &p1) {
  if (w == wB) return pl ? ((uint64_t)p0.w << 32) | p0.z : ((uint64_t)p0.y << 32) | p0.x;
  if (w == wB + 1) return pl ? ((uint64_t)p1.w << 32) | p1.z : ((uint64_t)p1.y << 32) | p1.x;
  return bits[2 * w + pl];
}
__device__ __forceinline__ uint64_t first_bit_run(const uint64_t *bits, int pl, uint64_t a, uint64_t b, uint64_t wB,
                                                  const uint4 &p0, const uint4 &p1) {
  if (a > b) return ~0ull;
  const uint64_t wa = a >> 6, wb = b >> 6;
  for (uint64_t w = wa; w <= wb; ++w) {
    uint64_t m = bit_word(bits, pl, w, wB, p0, p1);
    if (w == wa) m &= ~0ull << (a & 63);
    if (w == wb) m &= bits_upto((uint32_t)(b & 63));
    if (m) return (w << 6) + (uint64_t)__builtin_ctzll(m);
  }
  return ~0ull;
}

// next(c) by one lane: group_next's semantics (the crate's cut_gear from c,
// file end fend).  Sets punt (result void) for a step it does not take.
// Two dependent memory levels per step:
//  1. the restart window's 64 bytes; the summaries of the runs holding the S
//     and the L window's first position (rS0, rL0); the S / L bitmap words
//     after them;
//  2. the summaries of the first run after rS0 with an S candidate and after
//     rL0 with an L candidate (bitmap search), and, when a window edge splits
//     rS0 or rL0 (first candidate before the edge, more in the run), its entry
//     list.
// The first qualifying S is the answer if there is one, else the first L:
// every source below yields a qualifying candidate or nothing, and the first
// qualifying one comes from one of them, so the minimum is exact.
__device__ __forceinline__ uint64_t lane_next(const Work &W, const DevParams &P, const uint64_t *tab, uint32_t lo8,
                                              uint64_t c, uint64_t fend, bool &punt) {
  const uint64_t rem = fend - c;
  if (rem <= P.min) return fend;  // remaining <= min_size: whole tail
  const uint32_t remaining = rem > P.max ? P.max : (uint32_t)rem;
  const uint32_t center = (rem <= P.max && rem < P.avg) ? (uint32_t)rem : P.avg;
  const uint32_t t0 = P.min / 2 * 2, ce = center / 2 * 2, re = remaining / 2 * 2;
  if (re <= t0) return c + remaining;  // loop never runs: forced
  const uint64_t t = c + t0;
  const uint32_t wlen = min(re - t0, (uint32_t)(kWin - 1));
  const int32_t lo_r = (int32_t)(t0 + kWin - 1), hi_r = (int32_t)re, cce_r = (int32_t)ce;
  const bool cand = lo_r < hi_r;
  const int32_t s_end = min(cce_r, hi_r), l_beg = max(lo_r, cce_r);
  const bool hasS = cand && lo_r < s_end, hasL = cand && l_beg < hi_r;
  // ---- level 1 (addresses clamped into the arrays: no branches around loads)
  const uint64_t A = t & ~15ull;
  uint32_t dw[16];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t ad = min(A + 16 * k, W.n_al - 16);  // (bytes past the arena are never used)
    const uint4 v = *reinterpret_cast<const uint4 *>(W.base + ad);
    dw[4 * k] = v.x; dw[4 * k + 1] = v.y; dw[4 * k + 2] = v.z; dw[4 * k + 3] = v.w;
  }
  const uint64_t rlast = W.nruns - 1;
  const uint64_t rS0 = min((c + (uint64_t)lo_r) / kRun, rlast);
  const uint64_t rL0 = min((c + (uint64_t)l_beg) / kRun, rlast);
  const uint64_t rS1 = hasS ? (c + (uint64_t)s_end - 1) / kRun : 0, rL1 = hasL ? (c + (uint64_t)hi_r - 1) / kRun : 0;
  const uint32_t uS0 = W.run_sum[rS0], uL0 = W.run_sum[rL0];
  // bitmap word pairs wB, wB + 1 (runs [64 wB, 64 wB + 128) hold both windows
  // after rS0 at max <= 256 KiB; + read-ahead words are allocated)
  const uint64_t wB = (rS0 + 1) >> 6;
  const uint4 bp0 = *reinterpret_cast<const uint4 *>(W.run_bits + 2 * wB);
  const uint4 bp1 = *reinterpret_cast<const uint4 *>(W.run_bits + 2 * wB + 2);

  // ---- (2) windowed candidates: S in [lo, s_end), L in [l_beg, hi) (chunk-relative).
  // Decided before the restart window's hash so that the level-2 loads are in
  // flight while it runs; the restart window's hit, if any, takes precedence.
  auto rel = [&](uint64_t r) { return (int32_t)((int64_t)(r * (uint64_t)kRun) - (int64_t)c); };
  int32_t best = INT32_MAX;
  // the runs holding each window's first position: their summaries decide,
  // unless the first candidate of the kind lies before the edge and more follow
  bool splitS = false, splitL = false;
  if (hasS) {
    const uint32_t fs1 = uS0 & 0x3fffu;
    const int32_t p = rel(rS0) + (int32_t)fs1 - 1;
    if (fs1 && p >= lo_r && p < s_end) best = p;
    else splitS = fs1 && p < lo_r && (uS0 >> 28) >= 2;
  }
  if (hasL) {
    const uint32_t fl1 = (uL0 >> 14) & 0x3fffu;
    const int32_t p = rel(rL0) + (int32_t)fl1 - 1;
    if (fl1 && p >= l_beg && p < hi_r) best = min(best, p);
    else splitL = fl1 && p < l_beg && (uL0 >> 28) >= 2;
  }
  // the first later run with a candidate of the kind (bitmap search)
  const uint64_t rS = hasS ? first_bit_run(W.run_bits, 0, rS0 + 1, rS1, wB, bp0, bp1) : ~0ull;
  const uint64_t rL = hasL ? first_bit_run(W.run_bits, 1, rL0 + 1, rL1, wB, bp0, bp1) : ~0ull;
  // ---- level 2
  const uint32_t uS = W.run_sum[min(rS, rlast)], uL = W.run_sum[min(rL, rlast)];
  // (a run's count: the summary's 4-bit field is exact below 15, which decides
  // "overflowed" for cap <= 14; larger caps read run_cnt)
  if (__builtin_expect(splitS, 0)) {
    const uint32_t cnt = P.cap <= 14 ? (uS0 >> 28) : W.run_cnt[rS0];
    best = min(best, lane_run_split(W, P, rS0, cnt, rel(rS0), lo_r, hi_r, cce_r, punt));
  }
  if (__builtin_expect(splitL, 0)) {
    const uint32_t cnt = P.cap <= 14 ? (uL0 >> 28) : W.run_cnt[rL0];
    best = min(best, lane_run_split(W, P, rL0, cnt, rel(rL0), lo_r, hi_r, cce_r, punt));
  }

  // ---- (1) exact restarted hash of the first <= 47 tested positions
  {
    const uint32_t q = (uint32_t)(t - A);  // window start within the 64 loaded bytes (0..15)
    uint32_t f[14], g[13], e[12];
    const uint32_t s8 = lane_sel(q & 8), s4 = lane_sel(q & 4);
#pragma unroll
    for (int i = 0; i < 14; ++i) f[i] = sel32(dw[i], dw[i + 2], s8);
#pragma unroll
    for (int i = 0; i < 13; ++i) g[i] = sel32(f[i], f[i + 1], s4);
#pragma unroll
    for (int j = 0; j < 12; ++j) e[j] = __builtin_amdgcn_alignbyte(g[j + 1], g[j], q & 3);
    const uint32_t mlo = (uint32_t)P.ms, mhi = (uint32_t)(P.ms >> 32);
    uint64_t h = 0;
    uint32_t acc = 0xffffffffu;
    gear_chain<kWin - 1>(tab, lo8, e, [&](int, uint64_t gv) {
      h = (h << 1) + gv;
      acc = min(acc, ((uint32_t)h & mlo) | ((uint32_t)(h >> 32) & mhi));
    });
    // every position tests mask_s when the window is whole and before ce
    const bool regular = wlen == (uint32_t)(kWin - 1) && ce >= t0 + (uint32_t)(kWin - 1);
    if (__builtin_expect(!regular || acc == 0, 0)) {  // exact: per-position mask, first hit
      uint32_t first = 0xffffffffu;
      h = 0;
      gear_chain<kWin - 1>(tab, lo8, e, [&](int i, uint64_t gv) {
        h = (h << 1) + gv;
        const uint64_t m = (t0 + (uint32_t)i < ce) ? P.ms : P.ml;
        if ((uint32_t)i < wlen && (h & m) == 0 && first == 0xffffffffu) first = (uint32_t)i;
      });
      if (first != 0xffffffffu) return t + first;
    }
  }
  if (!cand) return c + remaining;
  if (rS != ~0ull) {  // its first S lies past lo (later run); it qualifies before s_end
    const int32_t p = rel(rS) + (int32_t)(uS & 0x3fffu) - 1;
    if (p < s_end) best = min(best, p);
  }
  if (rL != ~0ull) {
    const int32_t p = rel(rL) + (int32_t)((uL >> 14) & 0x3fffu) - 1;
    if (p < hi_r) best = min(best, p);
  }
  return best != INT32_MAX ? c + (uint64_t)best : c + remaining;  // else forced cut
}

// One lane per segment, grid-stride: the speculative chain from the segment
// start (spec_chain's outputs).
__global__ __launch_bounds__(256) void k_spec_lane(Work W, DevParams P, uint32_t s0, uint32_t s1) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  __builtin_amdgcn_s_setprio(3);
  {  // per-call resets the later kernels rely on (link: file flags; counts: look-back words, offsets)
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
    for (uint32_t i = g; i < W.nfiles; i += gs) W.file_flags[i] = 0;
    if (W.lb_status)
      for (uint32_t i = g; i < lb_tiles(W.nsegs); i += gs) W.lb_status[i] = 0;
    if (g == 0) {
      W.seg_count[W.nsegs] = 0;
      W.seg_off[0] = 0;
    }
  }
  load_gear_rep(tab, W);
  const uint32_t lo8 = (threadIdx.x & 31) << 3;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x; s < s1; s += stride) {
    const Seg S = W.segs[s];
    const uint64_t fend = W.files[S.file].end;
    uint64_t *out = W.nodes + W.node_off[s];
    const uint64_t cap = W.node_off[s + 1] - W.node_off[s];
    uint64_t c = S.start, k = 0, exitp = fend;
    bool punt = false;
    for (;;) {
      if (k >= cap) { atomicOr(W.err, kErrNodeCap); break; }
      out[k++] = c;
      const uint64_t nc = lane_next(W, P, tab, lo8, c, fend, punt);
      if (punt) break;
      if (nc >= S.end) { exitp = nc; break; }
      c = nc;
    }
    if (punt) {
      W.punt_spec[atomicAdd(W.err + 4, 1u)] = s;
    } else {
      W.node_cnt[s] = (uint32_t)k;
      W.seg_exit[s] = exitp;
    }
  }
}

// One lane per segment: the continuation past the segment end until it meets
// a node of a later segment's speculative chain (link_chain's outputs).  A
// forced cut is an ordinary step here (continuation entries of one node); a
// continuation that reaches kContMax entries goes to the group walk, which
// takes forced stretches whole.
__global__ __launch_bounds__(256) void k_link_lane(Work W, DevParams P, uint32_t s0, uint32_t s1) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  __builtin_amdgcn_s_setprio(3);
  load_gear_rep(tab, W);
  const uint32_t lo8 = (threadIdx.x & 31) << 3;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x; s < s1; s += stride) {
    const Seg S = W.segs[s];
    const File F = W.files[S.file];
    if (S.flags & kSegLast) {
      W.link_seg[s] = kSegNone; W.link_idx[s] = 0; W.link_pos[s] = F.end; W.cont_cnt[s] = 0; W.cont_ent[s] = 0;
      continue;
    }
    uint64_t c = W.seg_exit[s];
    uint32_t ents = 0, ls = kSegNone, li = 0, j = 0xffffffffu, i = 0;
    uint64_t lp = F.end;
    bool punt = false;
    for (;;) {
      if (c >= F.end) { ls = kSegNone; lp = F.end; break; }
      const uint32_t jj = F.first_seg + (uint32_t)((c - F.start) / W.zseg);
      if (jj != j) { j = jj; i = 0; }
      const uint64_t *nd = W.nodes + W.node_off[j];
      const uint32_t n = W.node_cnt[j];
      uint64_t v = ~0ull;
      while (i < n) {  // nodes are sorted and c only grows: resume where the last step stopped
        v = nd[i];
        if (v >= c) break;
        ++i;
      }
      if (i < n && v == c) { ls = j; li = i; lp = c; break; }
      if (ents == (uint32_t)kContMax) { punt = true; break; }
      const uint64_t nc = lane_next(W, P, tab, lo8, c, F.end, punt);
      if (punt) break;
      W.cont[(uint64_t)s * kContMax + ents] = c;
      W.cont_rep[(uint64_t)s * kContMax + ents] = 1u;
      ++ents;
      c = nc;
    }
    if (punt) {
      W.punt_link[atomicAdd(W.err + 5, 1u)] = s;
      continue;
    }
    W.link_seg[s] = ls; W.link_idx[s] = li; W.link_pos[s] = lp;
    W.cont_cnt[s] = ents; W.cont_ent[s] = ents;
    if (ls != s + 1) atomicOr(&W.file_flags[S.file], kFileSkip);
  }
}

// ======================================================== fallback =======
// One wave walks a whole file serially and rewrites its segments' node lists.
__global__ __launch_bounds__(64) void k_fallback(Work W, DevParams P) {
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const uint32_t f = blockIdx.x;
  if (f >= W.nfiles) return;
  if (!(W.file_flags[f] & kFileFail)) return;
  const uint32_t lane = lane_id();
  const File F = W.files[f];
  if (F.nsegs == 0) return;
  const Group<64> G;
  uint32_t j = F.first_seg;
  uint64_t k = 0, c = F.start;
  bool ok = true;
  // append chain node x (uniform): close the segments before x's, then store it
  auto put = [&](uint64_t x) {
    const uint32_t jj = F.first_seg + (uint32_t)((x - F.start) / W.zseg);
    while (j < jj) {
      if (lane == 0) {
        W.node_cnt[j] = (uint32_t)k; W.link_pos[j] = x; W.cont_cnt[j] = 0; W.cont_ent[j] = 0;
        W.link_seg[j] = j + 1;
      }
      k = 0; ++j;
    }
    const uint64_t cap = W.node_off[j + 1] - W.node_off[j];
    if (k >= cap) { if (lane == 0) atomicOr(W.err, kErrNodeCap); ok = false; return; }
    if (lane == 0) W.nodes[W.node_off[j] + k] = x;
    ++k;
  };
  for (;;) {
    put(c);
    if (!ok) break;
    uint64_t nc = group_next<64>(G, W, P, gt, c, F.end);
    if (nc >= F.end) break;
    if (nc == c + P.max) {  // forced cut: take the forced stretch behind it in one go
      const uint64_t kk = forced_run<64>(G, W, P, gt, nc, F.end, kRepMax);
      for (uint64_t i = 0; i < kk && ok; ++i) put(nc + i * P.max);
      if (!ok) break;
      nc += kk * P.max;
    }
    c = nc;
  }
  const uint32_t last = F.first_seg + F.nsegs - 1;
  while (j <= last) {
    if (lane == 0) {
      W.node_cnt[j] = (uint32_t)k; W.link_pos[j] = F.end; W.cont_cnt[j] = 0; W.cont_ent[j] = 0;
      W.link_seg[j] = kSegNone;
    }
    k = 0; ++j;
  }
  if (lane == 0) {
    W.file_flags[f] = kFileFallbackDone;
    atomicAdd(W.err + 1, 1u);  // fallback file count (reported in mcdc_timing)
  }
}

// ============================================================ walk =======
// Default for every segment: on the true chain, entered at the merge index
// handed over by the previous segment (0 for a file's first segment and for
// files the serial fallback rewrote).  One thread per segment.
__global__ void k_walk_fast(Work W) {
  MCDC_VGPR_PAD(8);  // 8 used: not an exact fill (MCDC_VGPR_PAD)
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= W.nsegs) return;
  const Seg S = W.segs[s];
  const uint32_t fl = W.file_flags[S.file];
  W.seg_true[s] = 1;
  W.entry_idx[s] = ((S.flags & kSegFirst) || (fl & kFileFallbackDone)) ? 0 : W.link_idx[s - 1];
}

// Irregular segments: a continuation that did not merge into the next one.
__global__ void k_irr_flags(Work W) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= W.nsegs) return;
  W.irr_flag[s] = (!(W.segs[s].flags & kSegLast) && W.link_seg[s] != s + 1) ? 1 : 0;
}

// Files whose chain skipped segments: the path runs through consecutive
// segments between irregular ones, so only the irregular segments on it are
// visited (sorted list from DeviceSelect, binary search per jump): mark the
// skipped segments off the chain and hand the merge index to each jump target.
// One thread per file; serial steps = skips on the path, not segments.
__global__ void k_walk_jumps(Work W) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= W.nfiles) return;
  const uint32_t fl = W.file_flags[f];
  if (!(fl & kFileSkip) || (fl & kFileFallbackDone)) return;
  const File F = W.files[f];
  if (F.nsegs == 0) return;
  const uint32_t last = F.first_seg + F.nsegs - 1, n = *W.irr_n;
  uint32_t p = F.first_seg;
  for (;;) {
    uint32_t lo = 0, hi = n;  // first irregular segment >= p
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      if (W.irr_list[mid] < p) lo = mid + 1;
      else hi = mid;
    }
    if (lo == n) break;
    const uint32_t i = W.irr_list[lo];
    if (i > last) break;
    const uint32_t j = W.link_seg[i];
    const bool end = j == kSegNone || j == kSegFail || j > last;
    const uint32_t stop = end ? last + 1 : j;
    for (uint32_t t = i + 1; t < stop; ++t) W.seg_true[t] = 0;
    if (end) break;
    W.entry_idx[j] = W.link_idx[i];
    p = j;
  }
}

// =========================================================== emit ========
__global__ void k_count(Work W) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= W.nsegs) return;
  uint64_t n = 0;
  if (W.seg_true[s]) n = (uint64_t)(W.node_cnt[s] - W.entry_idx[s]) + W.cont_cnt[s];
  W.seg_count[s] = n;
}

// ChunkData.hash as fastcdc returns it: the 2-byte loop's state at the cut.
// ChunkData.hash of the chunk [c, c + len) (file ends at fend): the 2-byte
// loop's state at its return.  A hit at even index i returns (h << 2) +
// GEAR_LS = 2 * (the 1-byte state), at odd index the 1-byte state; a forced
// cut returns the state after position re - 1; a tail <= min returns 0.  The
// state is sum_{j=from..q} GEAR[x_j] << (q - j) mod 2^64 with from = max(q-63,
// restart): k_emit evaluates it as a 64-lane wave sum (lane k holds x_{q-k}).
struct ChunkQ {
  uint64_t q, from;  // last byte, first byte of the window (q < from: hash 0)
  bool dbl;
};

__device__ __forceinline__ ChunkQ chunk_q(const DevParams &P, uint64_t c, uint64_t len, uint64_t fend) {
  ChunkQ r{0, 1, false};
  const uint64_t rem = fend - c;
  if (rem <= P.min) return r;
  const uint64_t remaining = rem > P.max ? (uint64_t)P.max : rem;
  const uint64_t t0 = (uint64_t)(P.min / 2) * 2, re = (remaining / 2) * 2;
  if (len < remaining) {  // cut by a mask hit at position c + len
    r.q = c + len;
    r.dbl = (len & 1) == 0;  // even index: state is (h << 2) + GEAR_LS
  } else {                   // forced cut: state after position re - 1
    if (re <= t0) return r;
    r.q = c + re - 1;
  }
  const uint64_t t = c + t0;
  r.from = r.q >= t + 63 ? r.q - 63 : t;
  return r;
}

// ChunkData.hash of one chunk, computed by one lane: the 64 bytes ending at q
// arrive as five aligned 16-byte loads (blocks past q are not read, so no
// load leaves the arena), are realigned in registers so that byte i is
// position q - 63 + i, and run through the 2-byte loop's recurrence
// h = (h << 1) + GEAR[x] (the same sum: a term k bytes before q is shifted k
// times).  Positions before `from` (a chunk that restarted < 63 bytes before
// its cut) add nothing.  GEAR from the replicated LDS table (k_emit).
// (Round 2 summed 80 independent lookups each with its own variable shift
// and window select: ~10 VALU per byte; this is 2 VALU + 1 LDS per byte.)
__device__ __forceinline__ uint64_t chunk_hash(const Work &W, const uint64_t *tab, uint32_t lo8, const ChunkQ &cq) {
  if (cq.q < cq.from) return 0;
  const uint64_t s0 = cq.q - 63;  // q >= t0 >= 64 (min_size >= 64)
  const uint64_t B = s0 & ~15ull;
  const uint32_t off = (uint32_t)(s0 - B);
  uint32_t dw[20];
#pragma unroll
  for (int k = 0; k < 5; ++k) {  // (clamped, not skipped: bytes past q are never used; no branch per load)
    const uint4 b = *reinterpret_cast<const uint4 *>(W.base + min(B + 16 * k, W.n_al - 16));
    dw[4 * k] = b.x; dw[4 * k + 1] = b.y; dw[4 * k + 2] = b.z; dw[4 * k + 3] = b.w;
  }
  uint32_t f[18], g[17], e[16];
  const uint32_t s8 = lane_sel(off & 8), s4 = lane_sel(off & 4);
#pragma unroll
  for (int i = 0; i < 18; ++i) f[i] = sel32(dw[i], dw[i + 2], s8);
#pragma unroll
  for (int i = 0; i < 17; ++i) g[i] = sel32(f[i], f[i + 1], s4);
#pragma unroll
  for (int j = 0; j < 16; ++j) e[j] = __builtin_amdgcn_alignbyte(g[j + 1], g[j], off & 3);
  const uint32_t nex = (uint32_t)(cq.from - s0);  // leading positions outside the window
  uint64_t h = 0;
  if (__builtin_expect(__any(nex != 0), 0))
    gear_chain<64>(tab, lo8, e, [&](int i, uint64_t gv) { h = (h << 1) + ((uint32_t)i < nex ? 0ull : gv); });
  else
    gear_chain<64>(tab, lo8, e, [&](int, uint64_t gv) { h = (h << 1) + gv; });
  return cq.dbl ? h << 1 : h;
}

// Node ii of a continuation list whose entries repeat (see k_link).
__device__ __forceinline__ uint64_t cont_node(const uint64_t *ct, const uint32_t *cr, uint64_t ii, uint32_t mx) {
  uint32_t e = 0;
  uint64_t before = 0;
  for (;;) {
    const uint64_t r = cr[e];
    if (ii < before + r) break;
    before += r;
    ++e;
  }
  return ct[e] + (ii - before) * mx;
}

// One output record: the chunk [pos, nxt) of file F at output index o.
__device__ __forceinline__ void emit_one(const Work &W, const DevParams &P, const uint64_t *tab, uint32_t lo8,
                                         const File &F, uint64_t o, uint64_t pos, uint64_t nxt) {
  const ChunkQ cq = chunk_q(P, pos, nxt - pos, F.end);
  const uint64_t hash = chunk_hash(W, tab, lo8, cq);
  if (o < W.out_cap) {
    DevChunk ch;
    ch.offset = pos - F.start;
    ch.length = nxt - pos;
    ch.hash = hash;
    W.out[o] = ch;
  } else {
    atomicOr(W.err, kErrOutCap);
  }
}

// One group of GS lanes per segment (grid-stride over segments: the 64 KiB
// table is loaded once per 1024-thread block, 16 waves per CU share it: the
// emit is latency-bound and needs the waves), lane i owns chunk i (of each batch of GS)
// and computes its hash itself.  GS = 8 on the lane walk (segments of ~6
// chunks), 16 on the group walk (~16).
//
// VGPR allocations are audited at build time: filling one
// exactly lost the memory returns of whole waves (k_emit at 184/184 in round
// 2), and a wrong ChunkData.hash is the one output no later stage re-checks.
// fcnt (optional): chunks per file into pinned host memory (k_file_counts'
// work, done by the threads whose segments are emitted: it overlaps the
// emit's latency instead of following it, ~14 us for 80 000 files)
template <int GS>
__global__ __launch_bounds__(1024) void k_emit(Work W, DevParams P, uint32_t s0, uint32_t s1, uint64_t *fcnt) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  __builtin_amdgcn_s_setprio(3);
  load_gear_rep(tab, W);
  const uint32_t lo8 = (threadIdx.x & 31) << 3;
  const uint32_t lane = lane_id() & (GS - 1);
  const uint32_t ng = gridDim.x * blockDim.x / GS;
  for (uint32_t s = s0 + (blockIdx.x * blockDim.x + threadIdx.x) / GS; s < s1; s += ng) {
    // the segment's metadata in one round of loads (nothing behind the n == 0 test)
    const uint64_t n = W.seg_count[s];
    const uint32_t fi = W.segs[s].file, e = W.entry_idx[s], ncnt = W.node_cnt[s], cent = W.cont_ent[s];
    const uint64_t noff = W.node_off[s], after = W.link_pos[s], base_out = W.seg_off[s];
    const File F = W.files[fi];
    if (n == 0) continue;
    const uint64_t nn = ncnt - e;
    const uint64_t *nd = W.nodes + noff + e;
    const uint64_t *ct = W.cont + (uint64_t)s * kContMax;
    const uint32_t *cr = W.cont_rep + (uint64_t)s * kContMax;
    const uint64_t ncont = n - nn;                    // continuation nodes, expanded
    const bool plain = ncont == cent;                 // every entry a single node
    const uint64_t n_here = ncont > kEmitInline ? nn : n;  // a long stretch: k_emit_long
    auto node = [&](uint64_t i) -> uint64_t {
      if (i < nn) return nd[i];
      return plain ? ct[i - nn] : cont_node(ct, cr, i - nn, P.max);
    };
    for (uint64_t i0 = 0; i0 < n_here; i0 += GS) {
      const uint64_t i = i0 + lane;
      if (i < n_here) {
        const uint64_t pos = node(i);
        const uint64_t nxt = i + 1 < n ? node(i + 1) : after;
        emit_one(W, P, tab, lo8, F, base_out + i, pos, nxt);
      }
    }
  }
  if (fcnt)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W.nfiles; i += gridDim.x * blockDim.x) {
      const File F = W.files[i];
      fcnt[i] = F.nsegs ? W.seg_off[F.first_seg + F.nsegs] - W.seg_off[F.first_seg] : 0;
    }
}

// Continuation stretches longer than kEmitInline nodes (k_link appended their
// segments to long_list): the whole grid strides over each one's nodes.
__global__ __launch_bounds__(256) void k_emit_long(Work W, DevParams P) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[256 * 32];
  load_gear_rep(tab, W);
  const uint32_t lo8 = (threadIdx.x & 31) << 3;
  const uint32_t nl = *W.long_n;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint32_t li = 0; li < nl; ++li) {
    const uint32_t s = W.long_list[li];
    const uint64_t n = W.seg_count[s];
    if (n == 0) continue;  // off the true chain
    const uint64_t nn = W.node_cnt[s] - W.entry_idx[s], ncont = n - nn;
    if (ncont <= kEmitInline) continue;  // rewritten by k_fallback, or emitted by k_emit
    const File F = W.files[W.segs[s].file];
    const uint64_t *ct = W.cont + (uint64_t)s * kContMax;
    const uint32_t *cr = W.cont_rep + (uint64_t)s * kContMax;
    const uint64_t after = W.link_pos[s], base_out = W.seg_off[s] + nn;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ncont; i += stride) {
      const uint64_t pos = cont_node(ct, cr, i, P.max);
      const uint64_t nxt = i + 1 < ncont ? cont_node(ct, cr, i + 1, P.max) : after;
      emit_one(W, P, tab, lo8, F, base_out + i, pos, nxt);
    }
  }
}

// Call summary for the host in one small write (pinned host memory): chunk
// total, error bits, fallback file count.
// (zero: the scan's partial-tile bitmap words and tile counter, cleared for
// the next call once every reader of them has run -- unless the call needs
// the general resolution, which reads them again)
__global__ void k_finish(Work W, uint64_t *res, uint64_t *zero, uint32_t zwords) {
  MCDC_VGPR_PAD(12);  // (not an exact fill)
  if (zero && W.err[2] == 0)
    for (uint32_t i = threadIdx.x; i < zwords; i += blockDim.x) zero[i] = 0;
  if (threadIdx.x == 0) {
    res[0] = W.nsegs ? W.seg_off[W.nsegs] : 0;
    res[1] = W.err[0];
    res[2] = W.err[1];
    res[3] = W.err[2];
    res[4] = (uint64_t)W.err[4] + W.err[5];
  }
}

void launch_finish(const Work &w, uint64_t *res, hipStream_t stream, hipEvent_t ev_done, uint64_t *zero,
                   uint32_t zwords) {
  hipExtLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, stream, nullptr, ev_done, 0, w, res, zero, zwords);
}

// Chunks per file from the final segment offsets, written straight into
// pinned host memory (no segment-offset copy and host loop per call: 80 000
// files were 640 KB of pageable D2H plus a second synchronisation).
__global__ void k_file_counts(Work W, uint64_t *dst) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W.nfiles; i += gridDim.x * blockDim.x) {
    const File F = W.files[i];
    dst[i] = F.nsegs ? W.seg_off[F.first_seg + F.nsegs] - W.seg_off[F.first_seg] : 0;
  }
}

void launch_file_counts(const Work &w, uint64_t *dst, hipStream_t stream) {
  if (w.nfiles == 0) return;
  const uint32_t blocks = std::min<uint32_t>((w.nfiles + 255) / 256, 1024);
  hipLaunchKernelGGL(k_file_counts, dim3(blocks), dim3(256), 0, stream, w, dst);
}

// ============================================= incremental resolution ====
// The resolution of a prefix of segments runs while the scan of the rest of
// the arena is still in flight (mcdc_api.hip: staged pipeline).  In the
// common case every segment's continuation merged into the next segment
// (link_seg[s] == s + 1), so the true chain enters segment s at link_idx[s-1]
// and the per-segment counts / offsets / boundaries follow locally.  A segment
// whose continuation did anything else sets err[2] ("dirty"); the host then
// re-resolves the whole call with the general path (fallback, serial walk).
// Clean-path link rule: segment s continues into s + 1; or it skips exactly
// one segment (link_seg[s] == s + 2: its continuation crossed s + 1 without
// meeting s + 1's speculative chain, which is then off the true chain); or
// its continuation ran to the end of the file (kSegNone) and s + 1 is the
// file's last segment, which is then off the chain.  Anything else (a longer
// skip, a continuation that gave up) is left to the general path.
//
// With one-segment skips a segment's state is local: s is off the chain iff
// s - 1 is on it and skips s, so on(s) is the parity of the run of
// consecutive skips that ends at s - 1 (a link never leaves its file, so the
// run stops at the file's first segment).  The on-chain predecessor of an
// on-chain s is s - 1, or s - 2 when s - 1 is off (s - 2 skipped it into s).
// (Segments of ~4 expected chunks on the lane walk: ~165 of the 131 072
// links of the 64 GiB stream skip one segment, and every call would go to
// the general path.)
__device__ __forceinline__ bool seg_skips(const Work &W, uint32_t k) { return W.link_seg[k] == k + 2; }

// Clean-path state of segment s (incr_count_one computes it, incr_store
// writes it): the loads of a thread's segments are all issued before any of
// its stores (a store to a Work array may alias a later load for the
// compiler, which then serialised eight segments' dependent loads: 48 us for
// 8192 segments in one block).
struct IncrSeg {
  uint64_t count;
  uint32_t entry;
  bool on, bad;
};

__device__ __forceinline__ IncrSeg incr_count_one(const Work &W, uint32_t s) {
  // everything a segment normally needs in one round of loads, at clamped
  // indices (a load under `first ? 0 : ...` becomes a branch with its own wait)
  const uint32_t sm1 = s > 0 ? s - 1 : 0, sm2 = s > 1 ? s - 2 : 0, sp1 = min(s + 1, W.nsegs - 1);
  const uint32_t fl = W.segs[s].flags, nfl0 = W.segs[sp1].flags;
  const uint32_t nc = W.node_cnt[s], cc = W.cont_cnt[s];
  const uint32_t lp0 = W.link_seg[sm1], lidx1 = W.link_idx[sm1], l0 = W.link_seg[s];
  const uint32_t lpp0 = W.link_seg[sm2], lidx2 = W.link_idx[sm2];
  const bool first = fl & kSegFirst, last = fl & kSegLast;
  const uint32_t lp = first ? 0u : lp0, l = last ? 0u : l0, nfl = last ? 0u : nfl0;
  const uint32_t lpp = (first || s < 2) ? kSegNone : lpp0;
  bool on = true, bad = false;
  uint32_t entry = 0;
  if (!first) {
    // on(s - 1): parity of the consecutive one-segment skips ending at s - 2
    bool prev_on = true;
    if (lpp == s) {  // s - 2 skips s - 1 (rare): walk the run back
      prev_on = false;
      for (uint32_t k = s - 2; k > 0 && seg_skips(W, k - 1); --k) prev_on = !prev_on;
    }
    if (prev_on) {
      if (lp == s) entry = lidx1;
      else if (lp == s + 1) on = false;                       // s - 1 skips s
      else if (lp == kSegNone && last) on = false;            // continuation ran to the file end
      else bad = true;
    } else {  // s - 1 is off the chain: s - 2 skipped it into s
      entry = lidx2;
    }
  }
  if (on && !last)  // s's own link must keep the next segments local
    bad |= !(l == s + 1 || l == s + 2 || (l == kSegNone && (nfl & kSegLast)));
  bad |= on && entry > nc;
  IncrSeg r;
  r.count = (bad || !on) ? 0 : (uint64_t)(nc - entry) + cc;
  r.entry = entry;
  r.on = on;
  r.bad = bad;
  return r;
}

__device__ __forceinline__ void incr_store(const Work &W, uint32_t s, const IncrSeg &r) {
  W.seg_true[s] = r.on ? 1 : 0;
  W.entry_idx[s] = r.entry;
  W.seg_count[s] = r.count;
}

__global__ void k_incr_count(Work W, uint32_t s0, uint32_t s1) {
  MCDC_VGPR_PAD(16);  // 16 used: not an exact fill (MCDC_VGPR_PAD)
  const uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= s1) return;
  const IncrSeg r = incr_count_one(W, s);
  incr_store(W, s, r);
  if (r.bad) atomicOr(W.err + 2, 1u);
}

// Counts of [s0, s1) fused with the offsets for one block:
// seg_off[s + 1] = seg_off[s0] + inclusive prefix, 1024 threads x 8 segments
// per pass (one launch instead of count + device scan + add-base).
__global__ __launch_bounds__(1024) void k_incr_scan(Work W, uint32_t s0, uint32_t s1) {
  __builtin_amdgcn_s_setprio(3);
  constexpr int IT = 8;
  __shared__ uint64_t wsum[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t carry = W.seg_off[s0];
  uint32_t dirty = 0;
  for (uint64_t base = s0; base < s1; base += 1024 * IT) {
    uint64_t c[IT], tsum = 0;
    IncrSeg r[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint64_t s = base + (uint64_t)tid * IT + k;
      if (s < s1) r[k] = incr_count_one(W, (uint32_t)s);
      else r[k] = IncrSeg{0, 0, false, false};
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint64_t s = base + (uint64_t)tid * IT + k;
      if (s < s1) incr_store(W, (uint32_t)s, r[k]);
      c[k] = r[k].count;
      dirty |= r[k].bad ? 1u : 0u;
      tsum += c[k];
    }
    uint64_t x = tsum;  // inclusive wave scan
#pragma unroll
    for (unsigned d = 1; d < 64; d <<= 1) {
      const uint64_t v = shfl_up64(x, d);
      if (lane >= d) x += v;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint64_t v = wsum[k];
      wpre += (uint32_t)k < wv ? v : 0;
      total += v;
    }
    uint64_t run = carry + wpre + x - tsum;  // exclusive prefix of this thread's first segment
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint64_t s = base + (uint64_t)tid * IT + k;
      run += c[k];
      if (s < s1) W.seg_off[s + 1] = run;
    }
    carry += total;
    __syncthreads();
  }
  if (dirty) atomicOr(W.err + 2, 1u);
}

// Counts and offsets of segments [s0, s1) in ONE launch for any count
// (k_incr_count + a rocPRIM scan + k_add_base were four launches, ~25 us per
// 64 GiB call): tiles of 1024 segments are taken in order from a ticket
// (err[6]); a tile publishes its aggregate, looks back over its predecessors
// (decoupled look-back, one wave reading 64 predecessors' words at a time) and
// then publishes its inclusive prefix.  A status word holds flag and value
// together (flag in bits 62-63), written and read as one 8-byte agent-scope
// atomic, so a reader sees both or neither on any XCD.  Predecessors were
// ticketed earlier by resident blocks and publish their aggregates without
// waiting, so the spin always ends.
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = (1ull << 62) - 1;
constexpr int kLbIt = 1;  // segments per thread: 1024 per tile (consecutive lanes, consecutive segments)

__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
  return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(1024) void k_incr_lookback(Work W, uint32_t s0, uint32_t s1, uint64_t *status) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t sh_excl;
  __shared__ uint32_t sh_tile;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) sh_tile = atomicAdd(W.err + 6, 1u);
  __syncthreads();
  const uint32_t tile = sh_tile;
  const uint64_t base = s0 + (uint64_t)tile * (1024 * kLbIt);
  uint32_t dirty = 0;
  uint64_t c[kLbIt], tsum = 0;
  IncrSeg r[kLbIt];
#pragma unroll
  for (int k = 0; k < kLbIt; ++k) {
    const uint64_t s = base + (uint64_t)tid * kLbIt + k;
    if (s < s1) r[k] = incr_count_one(W, (uint32_t)s);
    else r[k] = IncrSeg{0, 0, false, false};
  }
#pragma unroll
  for (int k = 0; k < kLbIt; ++k) {
    const uint64_t s = base + (uint64_t)tid * kLbIt + k;
    if (s < s1) incr_store(W, (uint32_t)s, r[k]);
    c[k] = r[k].count;
    dirty |= r[k].bad ? 1u : 0u;
    tsum += c[k];
  }
  uint64_t x = tsum;  // inclusive wave scan
#pragma unroll
  for (unsigned d = 1; d < 64; d <<= 1) {
    const uint64_t v = shfl_up64(x, d);
    if (lane >= d) x += v;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint64_t wpre = 0, total = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t v = wsum[k];
    wpre += (uint32_t)k < wv ? v : 0;
    total += v;
  }
  if (wv == 0) {
    uint64_t excl = 0;
    if (tile == 0) {
      excl = W.seg_off[s0];
    } else {
      if (lane == 0) lb_store(status + tile, kLbAgg | total);
      int64_t j = (int64_t)tile - 1;  // lane l looks at tile j - l
      for (;;) {
        const int64_t idx = j - (int64_t)lane;
        const uint64_t v = idx >= 0 ? lb_load(status + idx) : kLbInc;  // (tile 0 is inclusive: never past it)
        const uint64_t fl = v >> 62;
        const uint64_t incm = __ballot(fl == 2), notready = __ballot(fl == 0);
        const uint32_t f = incm ? (uint32_t)__builtin_ctzll(incm) : 64u;  // nearest inclusive predecessor
        const uint64_t need = f == 64 ? ~0ull : ((2ull << f) - 1);        // lanes 0..f
        if (notready & need) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint64_t part = lane <= f ? (v & kLbVal) : 0;  // aggregates before f, f's inclusive value
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) part += shfl64(part, (int)(lane ^ d));
        excl += part;
        if (f != 64) break;
        j -= 64;
      }
    }
    if (lane == 0) {
      lb_store(status + tile, kLbInc | (excl + total));
      sh_excl = excl;
    }
  }
  __syncthreads();
  uint64_t run = sh_excl + wpre + x - tsum;  // exclusive prefix of this thread's first segment
#pragma unroll
  for (int k = 0; k < kLbIt; ++k) {
    const uint64_t s = base + (uint64_t)tid * kLbIt + k;
    run += c[k];
    if (s < s1) W.seg_off[s + 1] = run;
  }
  if (dirty) atomicOr(W.err + 2, 1u);
}

// seg_off[s + 1] = seg_off[s0] + inclusive prefix of seg_count over [s0, s].
__global__ void k_add_base(Work W, const uint64_t *incl, uint32_t s0, uint32_t s1) {
  const uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= s1) return;
  W.seg_off[s + 1] = W.seg_off[s0] + incl[s - s0];
}

size_t scan_tmp_bytes(uint32_t nsegs) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)nsegs + 1);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)nsegs + 1);
  (void)hipcub::DeviceSelect::Flagged(nullptr, c, hipcub::CountingInputIterator<uint32_t>(0u), (uint8_t *)nullptr,
                                      (uint32_t *)nullptr, (uint32_t *)nullptr, (int)nsegs + 1);
  return std::max(a, std::max(b, c));
}

static unsigned group_blocks(uint32_t n, int gs = kGroup) { return (n + 256 / gs - 1) / (256 / gs); }

Knobs read_knobs() {
  auto env = [](const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
  };
  Knobs k;
  k.parts = std::min(std::max(env("MCDC_PARTS", k.parts), 1), 4);
  k.tail_rounds = std::max(env("MCDC_TAIL_ROUNDS", k.tail_rounds), 1);
  k.part_tiles = std::max(env("MCDC_PART_TILES", k.part_tiles), 0);
  k.min_rounds = std::max(env("MCDC_MIN_ROUNDS", k.min_rounds), 0);
  k.scan_pieces = env("MCDC_SCAN_PIECES", k.scan_pieces);
  if (k.scan_pieces != 1 && k.scan_pieces != 2 && k.scan_pieces != 4) k.scan_pieces = 0;
  k.scan_cold = env("MCDC_SCAN_COLD", k.scan_cold) != 0;
  k.pinned_direct = env("MCDC_PINNED_DIRECT", k.pinned_direct) != 0;
  k.lane_walk = std::min(std::max(env("MCDC_LANE_WALK", k.lane_walk), 0), 2);
  k.lane_seg_chunks = std::max(env("MCDC_LANE_SEG_CHUNKS", k.lane_seg_chunks), 1);
  k.run_list = std::min(std::max(env("MCDC_RUN_LIST", k.run_list), 0), 2);
  k.zc_huf = env("MCDC_ZC_HUF", k.zc_huf ? 1 : 0) != 0;
  k.zc_two = env("MCDC_ZC_TWO", k.zc_two ? 1 : 0) != 0;
#ifdef MCDC_AB_KNOBS
  k.group = env("MCDC_GROUP", k.group);
  if (k.group != 8 && k.group != 16 && k.group != 32) k.group = kGroup;
  k.spec_occ = env("MCDC_SPEC_OCC", k.spec_occ) == 5 ? 5 : 6;
  k.dyn_tiles = env("MCDC_DYN_TILES", k.dyn_tiles) != 0;
  k.first_static = env("MCDC_FIRST_STATIC", k.first_static) != 0;
  k.seg_chunks = std::max(env("MCDC_SEG_CHUNKS", k.seg_chunks), 1);
#endif
  return k;
}

void launch_spec(const Work &w, const DevParams &p, const Knobs &k, uint32_t s0, uint32_t s1, hipStream_t stream) {
  if (s1 <= s0) return;
#ifdef MCDC_AB_KNOBS
  if (k.group == 8) {
    hipLaunchKernelGGL(k_spec<8>, dim3(group_blocks(s1 - s0, 8)), dim3(256), 0, stream, w, p, s0, s1);
    return;
  }
  if (k.group == 32) {
    hipLaunchKernelGGL(k_spec<32>, dim3(group_blocks(s1 - s0, 32)), dim3(256), 0, stream, w, p, s0, s1);
    return;
  }
  if (k.spec_occ == 5) {  // the 82-VGPR build
    hipLaunchKernelGGL(k_spec<16>, dim3(group_blocks(s1 - s0, 16)), dim3(256), 0, stream, w, p, s0, s1);
    return;
  }
#else
  (void)k;
#endif
  hipLaunchKernelGGL(k_spec6<16>, dim3(group_blocks(s1 - s0, 16)), dim3(256), 0, stream, w, p, s0, s1);
}

void launch_link(const Work &w, const DevParams &p, const Knobs &k, uint32_t s0, uint32_t s1, uint64_t node_cap,
                 hipStream_t stream) {
  if (s1 <= s0) return;
#ifdef MCDC_AB_KNOBS
  if (k.group == 8) {
    hipLaunchKernelGGL(k_link<8>, dim3(group_blocks(s1 - s0, 8)), dim3(256), 0, stream, w, p, s0, s1, node_cap);
    return;
  }
  if (k.group == 32) {
    hipLaunchKernelGGL(k_link<32>, dim3(group_blocks(s1 - s0, 32)), dim3(256), 0, stream, w, p, s0, s1, node_cap);
    return;
  }
#else
  (void)k;
#endif
  hipLaunchKernelGGL(k_link<16>, dim3(group_blocks(s1 - s0, 16)), dim3(256), 0, stream, w, p, s0, s1, node_cap);
}

// Blocks of a grid-stride resolution kernel with a 64 KiB LDS table: two per
// CU (the table is loaded once per block), fewer when the work is smaller.
static unsigned lane_grid(const Work &w, uint64_t items_per_block_round, uint64_t items, uint64_t per_cu = 2) {
  const uint64_t cap = per_cu * (w.ncu ? w.ncu : 256);
  const uint64_t need = (items + items_per_block_round - 1) / items_per_block_round;
  return (unsigned)std::max<uint64_t>(1, std::min(cap, need));
}

// One group of gs lanes per segment (8 on the lane walk's ~6-chunk segments,
// 16 on the group walk's ~16): a lane per chunk.  (Measured at 64 GiB: a
// quad of lanes per chunk sharing one 80-byte load was slower, 87-110 us vs
// 62 us: the emit is bound by outstanding L1 misses, not by requests.)
static void launch_emit(const Work &w, const DevParams &p, uint32_t s0, uint32_t s1, int gs, hipStream_t stream,
                        uint64_t *fcnt = nullptr) {
  if (s1 <= s0) return;
  const unsigned n = s1 - s0;
  if (gs == 8)
    hipLaunchKernelGGL(k_emit<8>, dim3(lane_grid(w, 1024 / 8, n, 1)), dim3(1024), 0, stream, w, p, s0, s1, fcnt);
  else
    hipLaunchKernelGGL(k_emit<kGroup>, dim3(lane_grid(w, 1024 / kGroup, n, 1)), dim3(1024), 0, stream, w, p, s0, s1,
                       fcnt);
}

// counts and offsets of segments [s0, s1) assuming the clean case
static void launch_counts_incremental(const Work &w, uint32_t s0, uint32_t s1, uint64_t *incl, void *scan_tmp,
                                      size_t scan_tmp_bytes_, hipStream_t stream) {
  const uint32_t n = s1 - s0;
  if (w.lb_status) {  // one launch, decoupled look-back (status words zeroed per call)
    hipLaunchKernelGGL(k_incr_lookback, dim3((n + 1024 * kLbIt - 1) / (1024 * kLbIt)), dim3(1024), 0, stream, w, s0,
                       s1, w.lb_status);
  } else if (n <= 8192) {  // one block, one pass: a single launch for small batches
    hipLaunchKernelGGL(k_incr_scan, dim3(1), dim3(1024), 0, stream, w, s0, s1);
  } else {
    hipLaunchKernelGGL(k_incr_count, dim3((n + 255) / 256), dim3(256), 0, stream, w, s0, s1);
    size_t bytes = scan_tmp_bytes_;
    (void)hipcub::DeviceScan::InclusiveSum(scan_tmp, bytes, w.seg_count + s0, incl, (int)n, stream);
    hipLaunchKernelGGL(k_add_base, dim3((n + 255) / 256), dim3(256), 0, stream, w, (const uint64_t *)incl, s0,
                       s1);
  }
}

// counts, offsets and boundaries of segments [s0, s1) assuming the clean case
void launch_emit_incremental(const Work &w, const DevParams &p, uint32_t s0, uint32_t s1, uint64_t *incl,
                             void *scan_tmp, size_t scan_tmp_bytes_, hipStream_t stream, int gs) {
  if (s1 <= s0) return;
  launch_counts_incremental(w, s0, s1, incl, scan_tmp, scan_tmp_bytes_, stream);
  launch_emit(w, p, s0, s1, gs, stream);
}

// The whole call on the lane walk: spec of every segment (one lane each), the
// group walk over the segments it handed back, the same for the links, then
// the clean path's counts, offsets and boundaries (8-lane emit groups).  The
// list kernels read their counts on the device (no host round trip): a fixed
// grid that exits at once when nothing was handed back.
void launch_resolve_lane(const Work &w, const DevParams &p, uint64_t *incl, void *scan_tmp, size_t scan_tmp_bytes_,
                         hipStream_t stream, uint64_t *fcnt) {
  if (w.nsegs == 0) return;
  const unsigned lg = lane_grid(w, 256, w.nsegs);
  const unsigned listg = w.ncu ? w.ncu : 256;
  hipLaunchKernelGGL(k_spec_lane, dim3(lg), dim3(256), 0, stream, w, p, 0u, w.nsegs);
  // (the two list kernels leave at once when nothing was handed back; skipping
  // their launches measured no different, tools/walk_ab.py)
  hipLaunchKernelGGL(k_spec_list<kGroup>, dim3(listg), dim3(256), 0, stream, w, p, (const uint32_t *)w.punt_spec,
                     (const uint32_t *)(w.err + 4));
  hipLaunchKernelGGL(k_link_lane, dim3(lg), dim3(256), 0, stream, w, p, 0u, w.nsegs);
  hipLaunchKernelGGL(k_link_list<kGroup>, dim3(listg), dim3(256), 0, stream, w, p, (const uint32_t *)w.punt_link,
                     (const uint32_t *)(w.err + 5));
  launch_counts_incremental(w, 0u, w.nsegs, incl, scan_tmp, scan_tmp_bytes_, stream);
  launch_emit(w, p, 0u, w.nsegs, 8, stream, fcnt);
}

// General resolution after k_spec / k_link of every segment: serial fallback
// for files whose chains never merged, chain walk (parallel or serial),
// counts, offsets, boundaries.
void launch_resolve_general(const Work &w, const DevParams &p, void *scan_tmp, size_t scan_tmp_bytes_,
                            hipStream_t stream) {
  if (w.nsegs == 0) return;
  hipLaunchKernelGGL(k_fallback, dim3(w.nfiles), dim3(64), 0, stream, w, p);
  hipLaunchKernelGGL(k_walk_fast, dim3((w.nsegs + 255) / 256), dim3(256), 0, stream, w);
  hipLaunchKernelGGL(k_irr_flags, dim3((w.nsegs + 255) / 256), dim3(256), 0, stream, w);
  size_t bytes = scan_tmp_bytes_;
  (void)hipcub::DeviceSelect::Flagged(scan_tmp, bytes, hipcub::CountingInputIterator<uint32_t>(0u), w.irr_flag,
                                      w.irr_list, w.irr_n, (int)w.nsegs, stream);
  hipLaunchKernelGGL(k_walk_jumps, dim3((w.nfiles + 255) / 256), dim3(256), 0, stream, w);
  hipLaunchKernelGGL(k_count, dim3((w.nsegs + 255) / 256), dim3(256), 0, stream, w);
  bytes = scan_tmp_bytes_;
  // seg_count has nsegs + 1 entries (last = 0) so seg_off[nsegs] = total
  (void)hipcub::DeviceScan::ExclusiveSum(scan_tmp, bytes, w.seg_count, w.seg_off, (int)w.nsegs + 1, stream);
  launch_emit(w, p, 0u, w.nsegs, kGroup, stream);
  hipLaunchKernelGGL(k_emit_long, dim3(2 * (w.ncu ? w.ncu : 256)), dim3(256), 0, stream, w, p);
}

}  // namespace mcdc
