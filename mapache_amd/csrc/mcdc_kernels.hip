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

// ---- Quad-coalesced scan: lane quad i loads one whole 64-byte line of run
// (4i+k) per load instruction k (16 lines per wave-instruction instead of 64),
// then the wave transposes through a private 5 KiB LDS pad (run stride 80 B:
// conflict-free ds_write_b128 / ds_read_b128) so each lane again hashes its
// own contiguous run.  LDS = 64 KiB table + 16 waves x 5 KiB = 144 KiB.
constexpr int kQPad = 80;                 // run stride in the transpose pad
constexpr int kQWaveBytes = 64 * kQPad;   // 5 KiB
constexpr int kSTab = 65536;              // GEAR<<16 x 32 copies

template <int RUN>
__global__ __launch_bounds__(1024, 4) void k_scan_q(Work W, DevParams P) {
  __shared__ __attribute__((aligned(16))) uint64_t smem[(kSTab + 16 * kQWaveBytes) / 8];
  const uint64_t *tab = smem;
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) smem[i] = W.gear16[i >> 5];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, lo = (lane & 31) << 3;
  const uint32_t wv = threadIdx.x >> 6;
  char *pad = reinterpret_cast<char *>(smem) + kSTab + wv * kQWaveBytes;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  const uint64_t nfull = W.n_al / RUN;
  const uint64_t ntiles_full = nfull / 64;
  constexpr int G = RUN / 64;
  static_assert(G % 2 == 0, "even group count");
  const uint32_t qi = lane >> 2, qj = lane & 3;
  // load k: lane (4i+j) fetches piece j of run 4i+k; it lands in the pad at run*80 + 16j
  char *wr0 = pad + (4 * qi + 0) * kQPad + 16 * qj;
  char *wr1 = pad + (4 * qi + 1) * kQPad + 16 * qj;
  char *wr2 = pad + (4 * qi + 2) * kQPad + 16 * qj;
  char *wr3 = pad + (4 * qi + 3) * kQPad + 16 * qj;
  const char *rd = pad + lane * kQPad;
  const uint32_t pf = P.pf_hi, cap = P.cap;
  const uint64_t ms16 = P.ms16, ml16 = P.ml16;
  for (uint64_t t = wid; t < ntiles_full; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    uint64_t h = 0;
    if (run > 0) {
      const uint4 *p = reinterpret_cast<const uint4 *>(W.base + run * (uint64_t)RUN);
      const uint4 w0 = p[-3], w1 = p[-2], w2 = p[-1];
      hash16(tab, lo, w0, h);
      hash16(tab, lo, w1, h);
      hash16(tab, lo, w2, h);
    }
    uint32_t *ent = W.run_ent + run * (uint64_t)cap;
    uint32_t cnt = 0;
    // quad-coalesced sources: run (4i+k), piece j
    const uint8_t *tb = W.base + t * 64 * (uint64_t)RUN + 16 * qj;
    const uint4 *s0 = reinterpret_cast<const uint4 *>(tb + (4 * qi + 0) * (uint64_t)RUN);
    const uint4 *s1 = reinterpret_cast<const uint4 *>(tb + (4 * qi + 1) * (uint64_t)RUN);
    const uint4 *s2 = reinterpret_cast<const uint4 *>(tb + (4 * qi + 2) * (uint64_t)RUN);
    const uint4 *s3 = reinterpret_cast<const uint4 *>(tb + (4 * qi + 3) * (uint64_t)RUN);
    uint4 a0 = s0[0], a1 = s1[0], a2 = s2[0], a3 = s3[0];
    uint4 b0 = s0[4], b1 = s1[4], b2 = s2[4], b3 = s3[4];
#pragma unroll 1
    for (int g = 0; g < G; g += 2) {
      {
        *reinterpret_cast<uint4 *>(wr0) = a0; *reinterpret_cast<uint4 *>(wr1) = a1;
        *reinterpret_cast<uint4 *>(wr2) = a2; *reinterpret_cast<uint4 *>(wr3) = a3;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(rd);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(rd + 16);
        const uint4 c2 = *reinterpret_cast<const uint4 *>(rd + 32);
        const uint4 c3 = *reinterpret_cast<const uint4 *>(rd + 48);
        const int gn = g + 2 < G ? g + 2 : G - 1;  // clamped, unconditional
        a0 = s0[4 * gn]; a1 = s1[4 * gn]; a2 = s2[4 * gn]; a3 = s3[4 * gn];
        const uint32_t off = 64u * g;
        scan16(tab, lo, c0, h, pf, ms16, ml16, off, cnt, ent, cap);
        scan16(tab, lo, c1, h, pf, ms16, ml16, off + 16, cnt, ent, cap);
        scan16(tab, lo, c2, h, pf, ms16, ml16, off + 32, cnt, ent, cap);
        scan16(tab, lo, c3, h, pf, ms16, ml16, off + 48, cnt, ent, cap);
      }
      {
        *reinterpret_cast<uint4 *>(wr0) = b0; *reinterpret_cast<uint4 *>(wr1) = b1;
        *reinterpret_cast<uint4 *>(wr2) = b2; *reinterpret_cast<uint4 *>(wr3) = b3;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(rd);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(rd + 16);
        const uint4 c2 = *reinterpret_cast<const uint4 *>(rd + 32);
        const uint4 c3 = *reinterpret_cast<const uint4 *>(rd + 48);
        const int gn = g + 3 < G ? g + 3 : G - 1;
        b0 = s0[4 * gn]; b1 = s1[4 * gn]; b2 = s2[4 * gn]; b3 = s3[4 * gn];
        const uint32_t off = 64u * (g + 1);
        scan16(tab, lo, c0, h, pf, ms16, ml16, off, cnt, ent, cap);
        scan16(tab, lo, c1, h, pf, ms16, ml16, off + 16, cnt, ent, cap);
        scan16(tab, lo, c2, h, pf, ms16, ml16, off + 32, cnt, ent, cap);
        scan16(tab, lo, c3, h, pf, ms16, ml16, off + 48, cnt, ent, cap);
      }
    }
    W.run_cnt[run] = cnt > cap ? kRunOverflow : (uint8_t)cnt;
  }
  const uint64_t nruns = (W.n_al + RUN - 1) / RUN;
  for (uint64_t t = ntiles_full + wid; t * 64 < nruns; t += nwaves) {
    const uint64_t run = t * 64 + lane;
    if (run < nfull) scan_run_full<RUN, 1>(tab, lo, W, P, run, run);
    else if (run < nruns) scan_run_tail<RUN>(tab, lo, W, P, run);
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
__device__ uint64_t run_first_hit(const Work &W, const DevParams &P, uint64_t r, uint64_t lo,
                                  uint64_t hi, uint64_t cce) {
  const uint64_t rs = r * (uint64_t)kRun, rend = rs + kRun;
  const uint64_t s = rs > lo ? rs : lo, e = rend < hi ? rend : hi;
  if (s >= e) return ~0ull;
  uint64_t h = 0;
  for (uint64_t q = s - (kWin - 1); q < e; ++q) {  // s >= lo = t + 47
    h = (h << 1) + W.gear[W.base[q]];
    if (q >= s) {
      const uint64_t m = q < cce ? P.ms : P.ml;
      if ((h & m) == 0) return q;
    }
  }
  return ~0ull;
}

// First candidate of one run in [lo, hi) from its (up to 8, cap == 8) entries;
// entries are not position-sorted, so take the minimum.  ~0 if none.
__device__ __forceinline__ uint64_t run_first_entry(uint64_t r, uint32_t cnt, const uint4 ea,
                                                    const uint4 eb, uint64_t lo, uint64_t hi,
                                                    uint64_t cce) {
  uint64_t found = ~0ull;
  const uint64_t rb = r * (uint64_t)kRun;
  const uint32_t e8[8] = {ea.x, ea.y, ea.z, ea.w, eb.x, eb.y, eb.z, eb.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t e = e8[i];
    const uint64_t pos = rb + (e & 0x00ffffffu);
    if ((uint32_t)i < cnt && pos >= lo && pos < hi && pos < found) {
      const bool ok = pos < cce ? (e >> 31) & 1 : (e >> 30) & 1;
      if (ok) found = pos;
    }
  }
  return found;
}

// next(c): the chunk starting at arena position c (file ends at fend) ends
// where fastcdc's cut_gear(&file[c..], min, avg, max, masks) says.  Called by
// a full wave with wave-uniform c, fend; returns the next chunk start.
// Latency shape: the restart-window bytes, the first 64 runs' candidate counts
// and (speculatively) their first 8 entries are all requested at once.
__device__ uint64_t wave_next(const Work &W, const DevParams &P, uint64_t c, uint64_t fend) {
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
  uint32_t cnt = 0;
  uint4 ea = make_uint4(0, 0, 0, 0), eb = make_uint4(0, 0, 0, 0);
  if (rl) {
    cnt = W.run_cnt[r];
    if (P.cap == 8) {
      const uint4 *ep = reinterpret_cast<const uint4 *>(W.run_ent + r * 8ull);
      ea = ep[0];
      eb = ep[1];
    }
  }
  // ---- (1) exact restarted hash for the first <= 47 tested positions
  uint64_t h = lane < wlen ? W.gear[byte] : 0;
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
        found = run_first_hit(W, P, r, lo, hi, cce);
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
        found = run_first_hit(W, P, rr, lo, hi, cce);
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
__global__ __launch_bounds__(256) void k_spec(Work W, DevParams P) {
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
    const uint64_t nc = wave_next(W, P, c, fend);
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
    c = wave_next(W, P, c, F.end);
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
    c = wave_next(W, P, c, F.end);
    if (c >= F.end) break;
  }
  const uint32_t last = F.first_seg + F.nsegs - 1;
  while (j <= last) {
    if (lane == 0) {
      W.node_cnt[j] = (uint32_t)k; W.link_pos[j] = F.end; W.cont_cnt[j] = 0; W.link_seg[j] = kSegNone;
    }
    k = 0; ++j;
  }
  if (lane == 0) W.file_flags[f] = kFileFallbackDone;
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
__device__ uint64_t chunk_hash(const Work &W, const DevParams &P, uint64_t c, uint64_t len,
                               uint64_t fend) {
  const uint64_t rem = fend - c;
  if (rem <= P.min) return 0;
  const uint64_t remaining = rem > P.max ? (uint64_t)P.max : rem;
  const uint64_t t0 = (uint64_t)(P.min / 2) * 2, re = (remaining / 2) * 2;
  uint64_t q;
  bool dbl;
  if (len < remaining) {  // cut by a mask hit at position c + len
    q = c + len;
    dbl = (len & 1) == 0;  // even index: state is (h << 2) + GEAR_LS
  } else {                 // forced cut: state after position re - 1
    if (re <= t0) return 0;
    q = c + re - 1;
    dbl = false;
  }
  const uint64_t t = c + t0;
  const uint64_t from = q >= t + 63 ? q - 63 : t;
  uint64_t h = 0;
  for (uint64_t j = from; j <= q; ++j) h = (h << 1) + W.gear[W.base[j]];
  return dbl ? h << 1 : h;
}

__global__ __launch_bounds__(256) void k_emit(Work W, DevParams P) {
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
  for (uint64_t i = lane; i < n; i += 64) {
    const uint64_t pos = i < nn ? nd[i] : ct[i - nn];
    const uint64_t j = i + 1;
    const uint64_t nxt = j < n ? (j < nn ? nd[j] : ct[j - nn]) : after;
    const uint64_t o = base_out + i;
    if (o < W.out_cap) {
      DevChunk ch;
      ch.offset = pos - F.start;
      ch.length = nxt - pos;
      ch.hash = chunk_hash(W, P, pos, nxt - pos, F.end);
      W.out[o] = ch;
    } else if (lane == 0) {
      atomicOr(W.err, kErrOutCap);
    }
  }
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
