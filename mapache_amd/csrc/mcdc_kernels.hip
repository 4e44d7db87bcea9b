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
#include <hipcub/hipcub.hpp>

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
}

// Last, partial run: byte loop with exact tests (one lane in the whole grid).
template <int RUN>
__device__ void scan_run_tail(const uint64_t *tab, uint32_t lo, const Work &W, const DevParams &P,
                              uint64_t run) {
  const uint64_t start = run * (uint64_t)RUN, end = W.n_al;
  const uint64_t w0 = start >= (uint64_t)kWin ? start - kWin : 0;
  uint64_t h = 0;
  uint32_t cnt = 0;
  uint32_t *ent = W.run_ent + run * (uint64_t)P.cap;
  for (uint64_t q = w0; q < end; ++q) {
    h = (h << 1) + lds_gear(tab, ((uint32_t)W.base[q] << 8) | lo);
    if (q >= start) {
      const uint32_t s_ = (h & P.ms16) == 0, l_ = (h & P.ml16) == 0;
      if (s_ | l_) {
        if (cnt < P.cap) ent[cnt] = (uint32_t)(q - start) | (s_ << 31) | (l_ << 30);
        ++cnt;
      }
    }
  }
  W.run_cnt[run] = cnt > P.cap ? kRunOverflow : (uint8_t)cnt;
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
// LDS = 64 KiB table + 16 waves x (5 KiB pad + 256 B run counters) = 148 KiB.
constexpr int kQPad = 80;                        // run stride in the transpose pad
constexpr int kQPadBytes = 64 * kQPad;           // 5 KiB
constexpr int kQWaveBytes = kQPadBytes + 64 * 4; // + per-run candidate counters
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

// Drain the wave's queue: lane i re-walks entry i's 16 bytes exactly.
template <int RUN>
__device__ __attribute__((noinline)) void q_drain(const uint64_t *tab, uint32_t lo, const uint8_t *base,
                                                  uint32_t *run_ent, uint64_t ms16, uint64_t ml16, uint32_t cap,
                                                  const char *pad, uint32_t *lcnt, uint32_t qn, uint64_t run0,
                                                  uint32_t lane) {
  if (lane < qn) {
    const char *slot = pad + lane * kQPad + 64;
    uint64_t x = *reinterpret_cast<const uint64_t *>(slot);
    const uint32_t meta = *reinterpret_cast<const uint32_t *>(slot + 8);
    const uint32_t rl = meta >> 16, off = meta & 0xffffu;
    const uint64_t run = run0 + rl;
    const uint4 d = *reinterpret_cast<const uint4 *>(base + run * (uint64_t)RUN + off);
    uint32_t *ent = run_ent + run * (uint64_t)cap;
    const uint32_t wd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      x = (x << 1) + lds_gear(tab, ((wd[i >> 2] >> (8 * (i & 3))) & 0xffu) << 8 | lo);
      const uint32_t s_ = (x & ms16) == 0, l_ = (x & ml16) == 0;
      if (s_ | l_) {
        const uint32_t k = atomicAdd(&lcnt[rl], 1u);
        if (k < cap) ent[k] = (off + i) | (s_ << 31) | (l_ << 30);
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
};

// 64 bytes (16 dwords) of one run: lookups one dword ahead of the chain;
// every 16 bytes a wave-uniform test queues the blocks whose prefilter fired.
template <int RUN>
__device__ __forceinline__ void scan64q(const QScan &q, const uint32_t *w, uint64_t &h, uint32_t off,
                                        uint32_t &qn, uint64_t run0) {
  uint64_t g[2][4];
  lookup4(q.tab, q.lo, w[0], g[0]);
  uint32_t acc = 0xffffffffu;
  uint64_t hb = h;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    if (d + 1 < 16) lookup4(q.tab, q.lo, w[d + 1], g[(d + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    // one wait per dword for its 4 lookups (the next dword's 4 stay in flight)
    // instead of the compiler's one wait per lookup
    if (d + 1 < 16) __builtin_amdgcn_s_waitcnt(kWaitLgkm4);
    else __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    __builtin_amdgcn_sched_barrier(0);
    chain4(g[d & 1], h, acc, q.pf);
    if (d % 4 == 3) {
      const uint64_t m = __ballot(acc == 0);
      if (__builtin_expect(m != 0, 0)) {
        const uint32_t n = (uint32_t)__popcll(m);
        if (qn + n > 64) {
          q_drain<RUN>(q.tab, q.lo, q.base, q.run_ent, q.ms16, q.ml16, q.cap, q.pad, q.lcnt, qn, run0, q.lane);
          qn = 0;
        }
        if (acc == 0) {
          const uint32_t slot =
              qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          char *sp = q.pad + slot * kQPad + 64;
          *reinterpret_cast<uint64_t *>(sp) = hb;
          *reinterpret_cast<uint32_t *>(sp + 8) = (q.lane << 16) | (off + 4 * (d - 3));
        }
        qn += n;
      }
      acc = 0xffffffffu;
      hb = h;
    }
  }
}

template <int RUN>
__global__ __launch_bounds__(1024, 4) void k_scan_q(Work W, DevParams P) {
  __shared__ __attribute__((aligned(16))) uint64_t smem[(kSTab + 16 * kQWaveBytes) / 8];
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) smem[i] = W.gear16[i >> 5];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR
  QScan q;
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
  __syncthreads();
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  const uint64_t nfull = W.n_al / RUN;
  const uint64_t ntiles_full = nfull / 64;
  constexpr int G = RUN / 64;
  static_assert(G % 2 == 0, "even group count");
  const uint32_t qi = lane >> 2, qj = lane & 3;
  // load k: lane (4i+j) fetches piece j of run 4i+k; it lands in the pad at run*80 + 16j
  char *wr = q.pad + 4 * qi * kQPad + 16 * qj;
  const char *rd = q.pad + lane * kQPad;
  const uint32_t o0 = 4 * qi * RUN + 16 * qj;  // lane's byte offset in the tile for load 0, group 0
  for (uint64_t t = wid; t < ntiles_full; t += nwaves) {
    const uint64_t run0 = t * 64, run = run0 + lane;
    uint64_t h = 0;
    if (run > 0) {  // warm-up: the 48 bytes before the run complete every window
      const uint4 *p = reinterpret_cast<const uint4 *>(W.base + run * (uint64_t)RUN);
      const uint4 w0 = p[-3], w1 = p[-2], w2 = p[-1];
      hash16(q.tab, q.lo, w0, h);
      hash16(q.tab, q.lo, w1, h);
      hash16(q.tab, q.lo, w2, h);
    }
    uint32_t qn = 0;  // wave-uniform queue length
    const uint8_t *tb = W.base + run0 * (uint64_t)RUN;  // wave-uniform tile base (SGPR)
#define MCDC_LDQ(k, gg) (*reinterpret_cast<const uint4 *>(tb + (uint64_t)(uint32_t)(o0 + (k) * RUN + 64 * (gg))))
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
        scan64q<RUN>(q, w, h, 64u * g, qn, run0);
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
        scan64q<RUN>(q, w, h, 64u * (g + 1), qn, run0);
      }
    }
#undef MCDC_LDQ
    if (qn) q_drain<RUN>(q.tab, q.lo, q.base, q.run_ent, q.ms16, q.ml16, q.cap, q.pad, q.lcnt, qn, run0, lane);
    const uint32_t cnt = q.lcnt[lane];
    q.lcnt[lane] = 0;
    W.run_cnt[run] = cnt > q.cap ? kRunOverflow : (uint8_t)cnt;
  }
  // partial last tile: lane-strided runs, exact per-lane path
  const uint64_t nruns = (W.n_al + RUN - 1) / RUN;
  for (uint64_t t = ntiles_full + wid; t * 64 < nruns; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    if (run < nfull) scan_run_full<RUN, 1>(q.tab, q.lo, W, P, run, run);
    else if (run < nruns) scan_run_tail<RUN>(q.tab, q.lo, W, P, run);
  }
}

// Product configuration: quad-coalesced scan, 16 waves (one 1024-thread
// block) per CU; tools/scanbench.hip keeps the lane-strided k_scan_t variants
// for comparison.
void launch_scan(const Work &w, const DevParams &p, int num_cus, hipStream_t stream) {
  const uint64_t ntiles = (w.nruns + 63) / 64;
  uint64_t blocks = (ntiles + 15) / 16;
  const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256);  // 144 KiB LDS -> 1 block/CU
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return;
  hipLaunchKernelGGL(k_scan_q<kRun>, dim3((unsigned)blocks), dim3(1024), 0, stream, w, p);
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

// In run-relative 32-bit coordinates: entries 0-3 always, 4-7 only when some
// lane of the wave has more than 4 (wave-uniform branch, rare on real data).
__device__ __forceinline__ uint64_t run_first_entry(uint64_t r, uint32_t cnt, const uint4 ea,
                                                    const uint4 eb, uint64_t lo, uint64_t hi,
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
  if (__any(cnt > 4)) {
    take(4, eb.x); take(5, eb.y); take(6, eb.z); take(7, eb.w);
  }
  return best == 0xffffffffu ? ~0ull : rb + best;
}

// next(c): the chunk starting at arena position c (file ends at fend) ends
// where fastcdc's cut_gear(&file[c..], min, avg, max, masks) says.  Called by
// a full wave with wave-uniform c, fend; returns the next chunk start.
// Latency shape: two dependent global levels per step — {restart-window bytes,
// the first 64 runs' candidate counts}, then {entries of the non-empty runs};
// GEAR comes from the block's LDS copy `gt`.
__device__ uint64_t wave_next(const Work &W, const DevParams &P, const uint64_t *gt, uint64_t c, uint64_t fend) {
  const uint32_t lane = lane_id();
  const uint64_t rem = fend - c;
  if (rem <= P.min) return fend;                  // remaining <= min_size: whole tail
  uint64_t center = P.avg, remaining = rem;
  if (rem > P.max) remaining = P.max;
  else if (rem < center) center = rem;
  const uint64_t t0 = (uint64_t)(P.min / 2) * 2, ce = (center / 2) * 2, re = (remaining / 2) * 2;
  if (re <= t0) return c + remaining;             // loop never runs: forced
  const uint64_t t = c + t0;
  const uint32_t wlen = (uint32_t)((re - t0) < (uint64_t)(kWin - 1) ? (re - t0) : (uint64_t)(kWin - 1));
  const uint64_t lo = t + (kWin - 1), hi = c + re, cce = c + ce;
  const bool cand = lo < hi;
  const uint64_t r0 = lo / kRun, r1 = cand ? (hi - 1) / kRun : 0;
  // ---- level-1 loads, all independent
  const uint32_t byte = lane < wlen ? W.base[t + lane] : 0;
  const uint64_t r = r0 + lane;
  const bool rl = cand && r <= r1;
  const uint32_t cnt = rl ? W.run_cnt[r] : 0;
  // ---- level 2: entries of non-empty runs (~15 % of runs on random data)
  uint4 ea = make_uint4(0, 0, 0, 0), eb = make_uint4(0, 0, 0, 0);
  if (P.cap == 8 && cnt > 0 && cnt <= 8) {
    const uint4 *ep = reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull);
    ea = ep[0];
    if (cnt > 4) eb = ep[1];
  }
  // ---- (1) exact restarted hash for the first <= 47 tested positions
  uint64_t h = lane < wlen ? gt[byte] : 0;
#pragma unroll
  for (unsigned d = 1; d < 64; d <<= 1) {
    const uint64_t v = shfl_up64(h, d);
    if (lane >= d) h += v << d;
  }
  bool pass = false;
  if (lane < wlen) pass = (h & ((t0 + lane < ce) ? P.ms : P.ml)) == 0;
  const uint64_t b = __ballot(pass);
  if (b) return t + (uint64_t)(__ffsll((unsigned long long)b) - 1);
  if (!cand) return c + remaining;
  // ---- (2) windowed candidates for [t + 47, c + re), first 64 runs
  {
    uint64_t found = ~0ull;
    if (rl) {
      if (cnt > P.cap) {
        found = run_first_hit(W, P, gt, r, lo, hi, cce);
      } else if (P.cap == 8) {
        found = run_first_entry(r, cnt, ea, eb, lo, hi, cce);
      } else {
        for (uint32_t i = 0; i < cnt; ++i) {
          const uint32_t e = W.run_ent[r * (uint64_t)P.cap + i];
          const uint64_t pos = r * (uint64_t)kRun + (e & 0x00ffffffu);
          if (pos >= lo && pos < hi && pos < found) {
            const bool ok = pos < cce ? (e >> 31) & 1 : (e >> 30) & 1;
            if (ok) found = pos;
          }
        }
      }
    }
    const uint64_t fb = __ballot(found != ~0ull);
    if (fb) return shfl64(found, __ffsll((unsigned long long)fb) - 1);
  }
  // ---- later batches (only when max spans more than 64 runs)
  for (uint64_t rb = r0 + 64; rb <= r1; rb += 64) {
    const uint64_t rr = rb + lane;
    uint64_t found = ~0ull;
    if (rr <= r1) {
      const uint32_t cn = W.run_cnt[rr];
      if (cn > P.cap) {
        found = run_first_hit(W, P, gt, rr, lo, hi, cce);
      } else {
        for (uint32_t i = 0; i < cn; ++i) {
          const uint32_t e = W.run_ent[rr * (uint64_t)P.cap + i];
          const uint64_t pos = rr * (uint64_t)kRun + (e & 0x00ffffffu);
          if (pos >= lo && pos < hi && pos < found) {
            const bool ok = pos < cce ? (e >> 31) & 1 : (e >> 30) & 1;
            if (ok) found = pos;
          }
        }
      }
    }
    const uint64_t fb = __ballot(found != ~0ull);
    if (fb) return shfl64(found, __ffsll((unsigned long long)fb) - 1);
  }
  return c + remaining;  // forced cut (e.g. all zeros)
}

// ============================================================ spec =======
__device__ __forceinline__ void load_gear_lds(uint64_t *gt, const Work &W) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) gt[i] = W.gear[i];
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_spec(Work W, DevParams P) {
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const uint32_t s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (s >= W.nsegs) return;
  const uint32_t lane = lane_id();
  const Seg S = W.segs[s];
  const uint64_t fend = W.files[S.file].end;
  uint64_t *out = W.nodes + W.node_off[s];
  const uint64_t cap = W.node_off[s + 1] - W.node_off[s];
  uint64_t c = S.start, k = 0, exitp = fend;
  for (;;) {
    if (k >= cap) { if (lane == 0) atomicOr(W.err, kErrNodeCap); break; }
    if (lane == 0) out[k] = c;
    ++k;
    const uint64_t nc = wave_next(W, P, gt, c, fend);
    if (nc >= S.end) { exitp = nc; break; }
    c = nc;
  }
  if (lane == 0) {
    W.node_cnt[s] = (uint32_t)k;
    W.seg_exit[s] = exitp;
  }
}

// index of c in nodes(j) (sorted), or -1; wave-cooperative
__device__ int find_node(const Work &W, uint32_t j, uint64_t c) {
  const uint32_t lane = lane_id();
  const uint64_t *nd = W.nodes + W.node_off[j];
  const uint32_t n = W.node_cnt[j];
  for (uint32_t b = 0; b < n; b += 64) {
    const uint32_t i = b + lane;
    const uint64_t v = i < n ? nd[i] : ~0ull;
    const uint64_t eq = __ballot(v == c);
    if (eq) return (int)(b + __ffsll((unsigned long long)eq) - 1);
    if (__ballot(v > c)) return -1;
  }
  return -1;
}

// ============================================================ link =======
__global__ __launch_bounds__(256) void k_link(Work W, DevParams P) {
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const uint32_t s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (s >= W.nsegs) return;
  const uint32_t lane = lane_id();
  const Seg S = W.segs[s];
  const File F = W.files[S.file];
  if (S.flags & kSegLast) {
    if (lane == 0) {
      W.link_seg[s] = kSegNone; W.link_idx[s] = 0; W.link_pos[s] = F.end; W.cont_cnt[s] = 0;
    }
    return;
  }
  uint64_t c = W.seg_exit[s];
  uint32_t steps = 0, ls = kSegFail, li = 0;
  uint64_t lp = F.end;
  for (;;) {
    if (c >= F.end) { ls = kSegNone; lp = F.end; break; }
    const uint32_t j = F.first_seg + (uint32_t)((c - F.start) / W.zseg);
    const int idx = find_node(W, j, c);
    if (idx >= 0) { ls = j; li = (uint32_t)idx; lp = c; break; }
    if (steps == (uint32_t)kContMax) break;  // give up: serial fallback
    if (lane == 0) W.cont[(uint64_t)s * kContMax + steps] = c;
    ++steps;
    c = wave_next(W, P, gt, c, F.end);
  }
  if (lane == 0) {
    W.link_seg[s] = ls; W.link_idx[s] = li; W.link_pos[s] = lp; W.cont_cnt[s] = steps;
    if (ls == kSegFail) atomicOr(&W.file_flags[S.file], kFileFail);
    else if (ls != s + 1) atomicOr(&W.file_flags[S.file], kFileSkip);
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
  uint32_t j = F.first_seg;
  uint64_t k = 0, c = F.start;
  for (;;) {
    // c belongs to segment jj; close segments before it
    const uint32_t jj = F.first_seg + (uint32_t)((c - F.start) / W.zseg);
    while (j < jj) {
      if (lane == 0) {
        W.node_cnt[j] = (uint32_t)k; W.link_pos[j] = c; W.cont_cnt[j] = 0; W.link_seg[j] = j + 1;
      }
      k = 0; ++j;
    }
    const uint64_t cap = W.node_off[j + 1] - W.node_off[j];
    if (k >= cap) { if (lane == 0) atomicOr(W.err, kErrNodeCap); break; }
    if (lane == 0) W.nodes[W.node_off[j] + k] = c;
    ++k;
    c = wave_next(W, P, gt, c, F.end);
    if (c >= F.end) break;
  }
  const uint32_t last = F.first_seg + F.nsegs - 1;
  while (j <= last) {
    if (lane == 0) {
      W.node_cnt[j] = (uint32_t)k; W.link_pos[j] = F.end; W.cont_cnt[j] = 0; W.link_seg[j] = kSegNone;
    }
    k = 0; ++j;
  }
  if (lane == 0) {
    W.file_flags[f] = kFileFallbackDone;
    atomicAdd(W.err + 1, 1u);  // fallback file count (reported in mcdc_timing)
  }
}

// ============================================================ walk =======
// Common case (every continuation merged into the next segment, or the file
// was resolved serially): every segment is on the true chain; entry = the
// merge index handed over by the previous segment.  One thread per segment.
__global__ void k_walk_fast(Work W) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= W.nsegs) return;
  const Seg S = W.segs[s];
  const uint32_t fl = W.file_flags[S.file];
  if (fl != 0 && !(fl & kFileFallbackDone)) return;  // k_walk_seq owns this file
  W.seg_true[s] = 1;
  W.entry_idx[s] = ((S.flags & kSegFirst) || (fl & kFileFallbackDone)) ? 0 : W.link_idx[s - 1];
}

// Files whose chain skipped a segment: follow the links serially (one wave).
__global__ __launch_bounds__(64) void k_walk_seq(Work W) {
  const uint32_t f = blockIdx.x;
  if (f >= W.nfiles) return;
  const uint32_t fl = W.file_flags[f];
  if (fl == 0 || (fl & kFileFallbackDone)) return;
  const uint32_t lane = lane_id();
  const File F = W.files[f];
  for (uint32_t i = lane; i < F.nsegs; i += 64) W.seg_true[F.first_seg + i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    uint32_t s = F.first_seg, e = 0;
    const uint32_t last = F.first_seg + F.nsegs - 1;
    for (;;) {
      W.seg_true[s] = 1;
      W.entry_idx[s] = e;
      if (s == last) break;
      const uint32_t j = W.link_seg[s];
      if (j == kSegNone || j == kSegFail || j > last) break;
      e = W.link_idx[s];
      s = j;
    }
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

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// One wave per segment: lane i owns chunk i (of each batch of 64); the
// chunk hashes are computed 8 at a time by the whole wave (byte loads of all 8
// windows issued together, GEAR from LDS, one wave sum each).
__global__ __launch_bounds__(256) void k_emit(Work W, DevParams P) {
  __shared__ uint64_t gt[256];
  load_gear_lds(gt, W);
  const uint32_t s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (s >= W.nsegs) return;
  const uint64_t n = W.seg_count[s];
  if (n == 0) return;
  const uint32_t lane = lane_id();
  const Seg S = W.segs[s];
  const File F = W.files[S.file];
  const uint32_t e = W.entry_idx[s];
  const uint64_t nn = W.node_cnt[s] - e;
  const uint64_t *nd = W.nodes + W.node_off[s] + e;
  const uint64_t *ct = W.cont + (uint64_t)s * kContMax;
  const uint64_t after = W.link_pos[s];
  const uint64_t base_out = W.seg_off[s];
  for (uint64_t i0 = 0; i0 < n; i0 += 64) {
    const uint64_t i = i0 + lane;
    const bool act = i < n;
    uint64_t pos = 0, nxt = 0;
    if (act) {
      pos = i < nn ? nd[i] : ct[i - nn];
      const uint64_t j = i + 1;
      nxt = j < n ? (j < nn ? nd[j] : ct[j - nn]) : after;
    }
    const ChunkQ cq = act ? chunk_q(P, pos, nxt - pos, F.end) : ChunkQ{0, 1, false};
    uint64_t mine = 0;
    const uint32_t m = (uint32_t)(n - i0 < 64 ? n - i0 : 64);
    for (uint32_t b = 0; b < m; b += 8) {  // wave-uniform
      uint32_t by[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t src = b + k < m ? b + k : m - 1;
        const uint64_t q = readlane64(cq.q, src), fr = readlane64(cq.from, src);
        const bool in = b + k < m && q >= fr + lane;  // position q - lane in [from, q]
        by[k] = in ? (uint32_t)W.base[q - lane] : 256u;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t v = by[k] < 256u ? gt[by[k]] << lane : 0;
        const uint64_t hsum = wave_sum64(v);
        if (lane == b + k) mine = hsum;
      }
    }
    if (act) {
      const uint64_t o = base_out + i;
      if (o < W.out_cap) {
        DevChunk ch;
        ch.offset = pos - F.start;
        ch.length = nxt - pos;
        ch.hash = cq.dbl ? mine << 1 : mine;
        W.out[o] = ch;
      } else {
        atomicOr(W.err, kErrOutCap);
      }
    }
  }
}

// Call summary for the host in one small write (pinned host memory): chunk
// total, error bits, fallback file count.
__global__ void k_finish(Work W, uint64_t *res) {
  if (threadIdx.x == 0) {
    res[0] = W.nsegs ? W.seg_off[W.nsegs] : 0;
    res[1] = W.err[0];
    res[2] = W.err[1];
  }
}

void launch_finish(const Work &w, uint64_t *res, hipStream_t stream) {
  hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, stream, w, res);
}

size_t scan_tmp_bytes(uint32_t nsegs) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                   (int)nsegs + 1);
  return bytes;
}

void launch_resolve(const Work &w, const DevParams &p, void *scan_tmp, size_t scan_tmp_bytes_,
                    hipStream_t stream) {
  if (w.nsegs == 0) return;
  const unsigned wave_blocks = (w.nsegs + 3) / 4;
  hipLaunchKernelGGL(k_spec, dim3(wave_blocks), dim3(256), 0, stream, w, p);
  hipLaunchKernelGGL(k_link, dim3(wave_blocks), dim3(256), 0, stream, w, p);
  hipLaunchKernelGGL(k_fallback, dim3(w.nfiles), dim3(64), 0, stream, w, p);
  hipLaunchKernelGGL(k_walk_fast, dim3((w.nsegs + 255) / 256), dim3(256), 0, stream, w);
  hipLaunchKernelGGL(k_walk_seq, dim3(w.nfiles), dim3(64), 0, stream, w);
  hipLaunchKernelGGL(k_count, dim3((w.nsegs + 255) / 256), dim3(256), 0, stream, w);
  size_t bytes = scan_tmp_bytes_;
  // seg_count has nsegs + 1 entries (last = 0) so seg_off[nsegs] = total
  hipcub::DeviceScan::ExclusiveSum(scan_tmp, bytes, w.seg_count, w.seg_off, (int)w.nsegs + 1, stream);
  hipLaunchKernelGGL(k_emit, dim3(wave_blocks), dim3(256), 0, stream, w, p);
}

}  // namespace mcdc
