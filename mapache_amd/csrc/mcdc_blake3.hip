// mcdc_blake3.hip — CDNA4 (gfx950) chunk IDs: BLAKE3 of every chunk of a
// boundary list, in HBM, right after the chunker.
//
// Replaces, for mapache's Archiver, the per-chunk ID::from_content(&data)
// at /root/reference/src/archiver/processor.rs:184 (src/global/mod.rs:86-88 ->
// src/utils/mod.rs:62-68: blake3::Hasher, unkeyed, 32-byte output; crate
// blake3 1.8.2).  BLAKE3 splits its input into 1024-byte "leaves" (the
// specification's chunks) of 16 64-byte blocks, chains the blocks of a leaf
// through the compression function, and joins the leaves' chaining values in
// a binary tree whose left subtree always holds the largest power-of-two
// number of leaves; the last compression carries the ROOT flag.
//
// GPU shape:
//   k_b3_groups   groups of 16 leaves (16 KiB) per chunk -> counts (full
//                 groups | tail group), tail-length histogram
//   (hipcub)      exclusive scan -> node slots and processing order
//   k_b3_owner    item -> chunk map: full groups first, then the tail groups
//                 longest first (counting sort)
//   k_b3_leaves   one lane per group: 16 x 16 block compressions from
//                 quad-coalesced loads transposed through LDS, the group's
//                 subtree reduced on the fly (completed subtrees in registers);
//                 a chunk of <= 16 leaves finishes its ID here (ROOT)
//   k_b3_tree_wide one wave per chunk of more than 16 groups (the levels of more
//                 than 512 nodes in HBM, the rest in LDS)
//   k_b3_tree     one lane per chunk of 2-16 groups: level-by-level pairing of its
//                 group nodes (the last node of an odd level moves up
//                 unchanged — the same tree as the specification's stack rule)
// Integer VALU work (~11 32-bit ops per input byte), no MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "mcdc_blake3.h"

namespace mcdc {

namespace b3 {

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au,
                   IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;
constexpr uint32_t kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8;
constexpr int kLeaf = 1024;     // BLAKE3 chunk
constexpr int kGroupLeaves = 16;  // leaves per lane in k_b3_leaves

// message word used at position i of round r (the permutation applied r
// times), compile time so the unrolled rounds index registers statically
struct Sched {
  uint8_t v[7][16];
};
constexpr Sched kS = {{{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                       {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                       {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                       {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                       {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                       {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                       {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}}};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

#define B3_G(a, b, c, d, mx, my)  \
  a = a + b + (mx);               \
  d = rotr(d ^ a, 16);            \
  c = c + d;                      \
  b = rotr(b ^ c, 12);            \
  a = a + b + (my);               \
  d = rotr(d ^ a, 8);             \
  c = c + d;                      \
  b = rotr(b ^ c, 7);

// cv <- first 8 words of compress(cv, m, counter, block_len, flags)
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint64_t counter,
                                         uint32_t block_len, uint32_t flags) {
  uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  uint32_t s8 = IV0, s9 = IV1, s10 = IV2, s11 = IV3;
  uint32_t s12 = (uint32_t)counter, s13 = (uint32_t)(counter >> 32), s14 = block_len, s15 = flags;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    B3_G(s0, s4, s8, s12, m[kS.v[r][0]], m[kS.v[r][1]])
    B3_G(s1, s5, s9, s13, m[kS.v[r][2]], m[kS.v[r][3]])
    B3_G(s2, s6, s10, s14, m[kS.v[r][4]], m[kS.v[r][5]])
    B3_G(s3, s7, s11, s15, m[kS.v[r][6]], m[kS.v[r][7]])
    B3_G(s0, s5, s10, s15, m[kS.v[r][8]], m[kS.v[r][9]])
    B3_G(s1, s6, s11, s12, m[kS.v[r][10]], m[kS.v[r][11]])
    B3_G(s2, s7, s8, s13, m[kS.v[r][12]], m[kS.v[r][13]])
    B3_G(s3, s4, s9, s14, m[kS.v[r][14]], m[kS.v[r][15]])
  }
  cv[0] = s0 ^ s8; cv[1] = s1 ^ s9; cv[2] = s2 ^ s10; cv[3] = s3 ^ s11;
  cv[4] = s4 ^ s12; cv[5] = s5 ^ s13; cv[6] = s6 ^ s14; cv[7] = s7 ^ s15;
}

__device__ __forceinline__ void iv(uint32_t cv[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3; cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// parent node: out = compress(IV, l || r, 0, 64, PARENT | extra)
__device__ __forceinline__ void parent(const uint32_t l[8], const uint32_t r[8], uint32_t extra, uint32_t out[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { m[i] = l[i]; m[8 + i] = r[i]; }
  iv(out);
  compress(out, m, 0, 64, kParent | extra);
}

// 16 little-endian message words of the block at byte address p (any
// alignment) holding `len` valid bytes (0..64; bytes past len are zero, as
// the specification pads a final block).  Reads never leave the 16-byte line
// of the block's last valid byte.
__device__ __forceinline__ void load_block(const uint8_t *p, uint32_t len, uint32_t m[16]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  const uint32_t r = (uint32_t)(a & 3);
  uint32_t raw[17];
  if (len == 64) {
    const uint4 q0 = *reinterpret_cast<const uint4 *>(w), q1 = *reinterpret_cast<const uint4 *>(w + 4),
                q2 = *reinterpret_cast<const uint4 *>(w + 8), q3 = *reinterpret_cast<const uint4 *>(w + 12);
    raw[0] = q0.x; raw[1] = q0.y; raw[2] = q0.z; raw[3] = q0.w;
    raw[4] = q1.x; raw[5] = q1.y; raw[6] = q1.z; raw[7] = q1.w;
    raw[8] = q2.x; raw[9] = q2.y; raw[10] = q2.z; raw[11] = q2.w;
    raw[12] = q3.x; raw[13] = q3.y; raw[14] = q3.z; raw[15] = q3.w;
    raw[16] = r ? w[16] : 0u;  // the 16th dword holds bytes 64-r.. only when misaligned
  } else {
    const uint32_t nw = (r + len + 3) / 4;  // dwords that hold valid bytes
#pragma unroll
    for (int i = 0; i < 17; ++i) raw[i] = (uint32_t)i < nw ? w[i] : 0u;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], r);
  if (len < 64) {  // zero the bytes past the end of the input
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int keep = (int)len - 4 * i;
      m[i] = keep >= 4 ? m[i] : keep <= 0 ? 0u : m[i] & ((1u << (8 * keep)) - 1u);
    }
  }
}

__device__ __forceinline__ void store_id(uint8_t *dst, const uint32_t h[8]) {
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  d[0] = make_uint4(h[0], h[1], h[2], h[3]);
  d[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

__device__ __forceinline__ uint32_t leaves_of(uint64_t len) {
  return len == 0 ? 1u : (uint32_t)((len + kLeaf - 1) / kLeaf);
}

}  // namespace b3

using namespace b3;

// Work items are 16-KiB groups of leaves.  Per chunk: len / 16 KiB full groups
// (256 full blocks each) and at most one tail group (the rest, or the empty
// input's one empty block).  Group counts are packed: low 32 bits full
// groups, high 32 bits tail groups, so one scan gives both the node slots
// (their sum) and the processing order: every full group first, in chunk
// order, then the tail groups sorted by block count, longest first (a
// counting sort over 256 bins) — the lanes of a wave then run loops of equal
// length (in chunk order a wave ran as long as its longest lane: ~10 % of
// its lane-cycles idle on the 64 GiB stream).
constexpr uint32_t kGroupBytes = kGroupLeaves * kLeaf;
constexpr int kTailBins = 256;
// chunks of kTreeLaneMax < groups <= kTreeWaveMax: the wave-parallel tree
constexpr uint64_t kTreeLaneMax = 16, kTreeWaveMax = 512;

__device__ __forceinline__ uint64_t gtotal(uint64_t x) { return (x & 0xffffffffull) + (x >> 32); }

__device__ __forceinline__ uint32_t tail_bin(uint64_t len) {  // 0 = 256 blocks ... 255 = one block
  const uint32_t rem = (uint32_t)(len % kGroupBytes);
  return kTailBins - (len == 0 ? 1u : (rem + 63) / 64);
}

// A chunk outside [0, nbytes) of the buffer gets no groups and sets *err.
__global__ __launch_bounds__(256) void k_b3_groups(const DevChunk *chunks, uint64_t n, uint64_t nbytes,
                                                   uint64_t *gcnt, uint32_t *hist, uint32_t *err) {
  __shared__ uint32_t lh[kTailBins];
  lh[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const DevChunk c = chunks[i];
    const bool ok = c.offset <= nbytes && c.length <= nbytes - c.offset;
    const uint64_t full = ok ? c.length / kGroupBytes : 0;
    const bool tail = ok && (c.length % kGroupBytes != 0 || c.length == 0);
    gcnt[i] = full | ((uint64_t)tail << 32);
    if (tail) atomicAdd(&lh[tail_bin(c.length)], 1u);
    if (!ok) atomicOr(err, 1u);
  } else if (i == n) {
    gcnt[i] = 0;
  }
  __syncthreads();
  if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

// Every hashing kernel first checks the group total against the host's bound
// (b3_group_bound assumes disjoint chunks; overlapping or repeated chunks
// exceed it): over the bound nothing is written, and the host re-runs the
// hashing with the exact total it reads back (mcdc_chunk_ids_device).
// owner[item] = chunk: full groups at [0, F) in chunk order, tail groups at
// F + (start of their bin) + (arrival order within the bin).
__global__ __launch_bounds__(256) void k_b3_owner(const DevChunk *chunks, const uint64_t *goff, uint64_t n,
                                                  uint64_t bound, const uint32_t *hist, uint32_t *cur,
                                                  uint32_t *owner, uint32_t *wide, uint32_t *wide_cnt) {
  __shared__ uint32_t bs[kTailBins], lc[kTailBins];
  const uint32_t t = threadIdx.x;
  bs[t] = hist[t];
  lc[t] = 0;
  __syncthreads();
  for (uint32_t d = 1; d < kTailBins; d <<= 1) {  // inclusive scan of the bins
    const uint32_t v = t >= d ? bs[t - d] : 0u;
    __syncthreads();
    bs[t] += v;
    __syncthreads();
  }
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + t;
  const uint64_t last = goff[n];
  const bool ok = i < n && gtotal(last) <= bound;
  if (ok) {  // chunks for the wave-parallel tree
    const uint64_t m = gtotal(goff[i + 1]) - gtotal(goff[i]);
    if (m > kTreeLaneMax) wide[atomicAdd(wide_cnt, 1u)] = (uint32_t)i;
  }
  uint64_t a = 0, b = 0;
  uint32_t bin = 0, rank = 0;
  bool tl = false;
  if (ok) {
    a = goff[i];
    b = goff[i + 1];
    tl = (b >> 32) != (a >> 32);
    if (tl) {
      bin = tail_bin(chunks[i].length);
      rank = atomicAdd(&lc[bin], 1u);  // rank within the block's share of the bin
    }
  }
  __syncthreads();
  // one global reservation per bin and block (a global atomic per tail
  // serialised on 256 addresses: 0.44 ms per 64 GiB call)
  if (lc[t]) lc[t] = atomicAdd(&cur[t], lc[t]);
  __syncthreads();
  if (!ok) return;
  for (uint64_t g = a & 0xffffffffull; g < (b & 0xffffffffull); ++g) owner[g] = (uint32_t)i;
  if (tl) owner[(last & 0xffffffffull) + (bs[bin] - hist[bin]) + lc[bin] + rank] = (uint32_t)i;
}

// One lane per group (<= 16 leaves).  The group's subtree (a complete binary
// tree when it holds 16 leaves, the specification's tree of its leaves
// otherwise) is built on the fly: a finished leaf merges with the completed
// subtrees below it (one per set bit of its index) and is kept at its level
// (levels 0-1 in registers, 2-3 in LDS: 32 VGPRs would cost the fourth wave
// per SIMD).  The main loop runs over 64-byte blocks with a wave-uniform trip
// count (the wave's longest lane; shorter lanes idle under the exec mask,
// rare once the items are ordered); the one partial block a group can end
// with is hashed after it.
//
// Loads (MCDC_B3_QUAD, default): quad-coalesced, as in the scan — for block
// j, load q of lane 4k + i fetches the 16 bytes at offset 16 i of block j of
// lane 16 q + k at the block's own byte address (gfx950 reads a misaligned
// dwordx4 as the 16 bytes at that address: tools/dbg/unaligned_probe.hip), so
// a wave-instruction touches 16 runs of 64 contiguous bytes instead of 64
// scattered 16-byte pieces; the wave transposes through a private 4 KiB LDS
// pad and each lane reads its own block.  Pad layout: row r (a block) piece i
// (16 B) at slot 4 r + (i ^ ((r >> 2) & 3)) -- conflict-free for both sides:
// a ds_write_b128 8-lane group (two rows, bank (a/4) mod 32) covers the 8
// distinct 16-byte slots of a 128-byte bank row, and each ds_read_b128
// 16-lane group (bank (a/4) mod 64) reads 16 distinct slots of a 256-byte
// row (the 80-byte row stride it replaces had 2-way write conflicts).
// MCDC_B3_QUAD=0: each lane loads its own block (four 16-byte loads).  Block
// j + 1 is requested before block j is compressed.
#ifndef MCDC_B3_QUAD
#define MCDC_B3_QUAD 1
#endif
#if MCDC_B3_QUAD
constexpr int kB3Pad = 4;  // uint4 per pad row (64 B, swizzled)
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *gq;  // global (not flat) loads

__device__ __forceinline__ uint4 gload(uint64_t a) {
  const u32x4 v = *reinterpret_cast<gq>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_b3_leaves(
    const uint8_t *base, const DevChunk *chunks, const uint64_t *goff, const uint32_t *owner, uint64_t n,
    uint64_t bound, uint32_t *nodes, uint8_t *ids) {
#if MCDC_B3_QUAD
  __shared__ uint4 pad_all[4][64 * kB3Pad];
#endif
  __shared__ uint32_t up_all[4][2 * 8 * 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t last_off = goff[n];
  const uint64_t total = gtotal(last_off);
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + 64 * wv;  // the wave's first item
  if (g0 >= total || total > bound) return;  // wave-uniform; the grid is sized by the host bound
  const uint64_t p = g0 + lane;
  const bool act = p < total;
  uint32_t i = 0, nfull = 0, tail = 0, nleaves = 1;
  uint64_t l0 = 0, slot_idx = 0;
  bool has_tail = false;
  const uint8_t *gp = reinterpret_cast<const uint8_t *>(chunks);  // (a readable address for idle lanes)
  if (act) {
    i = owner[p];
    const DevChunk ch = chunks[i];
    const uint64_t a = goff[i];
    const uint64_t gi = p < (last_off & 0xffffffffull) ? p - (a & 0xffffffffull) : ch.length / kGroupBytes;
    nleaves = leaves_of(ch.length);
    l0 = gi * kGroupLeaves;
    const uint64_t grem = ch.length - gi * kGroupBytes;
    const uint32_t gbytes = (uint32_t)(grem < kGroupBytes ? grem : kGroupBytes);
    nfull = gbytes / 64;
    tail = gbytes % 64;
    has_tail = tail != 0 || gbytes == 0;  // (the empty input is one empty block)
    gp = base + ch.offset + gi * kGroupBytes;
    slot_idx = gtotal(a) + gi;
  }
  const uint32_t nblk = nfull + (has_tail ? 1u : 0u);
  const bool whole = nleaves <= kGroupLeaves;  // this group is the chunk's whole tree
  const bool root1 = nleaves == 1;             // ... and its only leaf is the root
  // the wave's longest and shortest lanes (wave-uniform)
  uint32_t nmax = nfull, nmin = nfull;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, d));
    nmin = min(nmin, (uint32_t)__shfl_xor((int)nmin, d));
  }
  nmax = __builtin_amdgcn_readfirstlane(nmax);
  nmin = __builtin_amdgcn_readfirstlane(nmin);
  const uint64_t gpa = reinterpret_cast<uint64_t>(gp);
#if MCDC_B3_QUAD
  // the four blocks this lane fetches: lane 16 q + k's block, piece i
  const uint32_t qk = lane >> 2, qi = lane & 3;
  uint64_t aq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int src = 16 * q + (int)qk;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)gpa, src), hi = (uint32_t)__shfl((int)(uint32_t)(gpa >> 32), src);
    aq[q] = (((uint64_t)hi << 32) | lo) + 16 * qi;
  }
  uint4 *pad = pad_all[wv];
  uint4 *wr = pad + kB3Pad * qk + (qi ^ ((qk >> 2) & 3));
  const uint4 *rd = pad + kB3Pad * lane;
  const uint32_t sw = (lane >> 2) & 3;  // the read side of the swizzle
  uint4 a0, a1, a2, a3;
  // block b of every source lane; past a lane's last full block (only in
  // waves of unequal lanes) the address is clamped to it, or to a readable
  // dummy when it has none (the data is not used)
  auto fetch = [&](uint32_t b) {
    if (b < nmin) {
      a0 = gload(aq[0] + 64ull * b);
      a1 = gload(aq[1] + 64ull * b);
      a2 = gload(aq[2] + 64ull * b);
      a3 = gload(aq[3] + 64ull * b);
    } else {
      auto clamped = [&](int q) {
        const uint32_t nf = (uint32_t)__shfl((int)nfull, 16 * q + (int)qk);
        return nf ? aq[q] + 64ull * min(b, nf - 1) : reinterpret_cast<uint64_t>(chunks);
      };
      a0 = gload(clamped(0));
      a1 = gload(clamped(1));
      a2 = gload(clamped(2));
      a3 = gload(clamped(3));
    }
  };
#else
  uint4 a0, a1, a2, a3;
  auto fetch = [&](uint32_t b) {
    const uint64_t x = nfull ? gpa + 64ull * min(b, nfull - 1) : reinterpret_cast<uint64_t>(chunks);
    a0 = gload(x); a1 = gload(x + 16); a2 = gload(x + 32); a3 = gload(x + 48);
  };
#endif
  // completed subtrees: levels 0-1 in registers, 2-3 in LDS ([level][word][lane])
  uint32_t s0[8], s1[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) s0[w] = s1[w] = 0;
  uint32_t *up = up_all[wv];
  auto sget = [&](uint32_t l, uint32_t out[8]) {
    if (l < 2) {
#pragma unroll
      for (int w = 0; w < 8; ++w) out[w] = l == 0 ? s0[w] : s1[w];
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) out[w] = up[((l - 2) * 8 + w) * 64 + lane];
    }
  };
  auto sput = [&](uint32_t l, const uint32_t in[8]) {
    if (l < 2) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s0[w] = l == 0 ? in[w] : s0[w];
        s1[w] = l == 1 ? in[w] : s1[w];
      }
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) up[((l - 2) * 8 + w) * 64 + lane] = in[w];
    }
  };
  uint32_t cv[8];
  iv(cv);
  if (nmax) fetch(0);
#pragma unroll 1
  for (uint32_t j = 0; j < nmax; ++j) {
#if MCDC_B3_QUAD
    wr[0] = a0;
    wr[16 * kB3Pad] = a1;
    wr[32 * kB3Pad] = a2;
    wr[48 * kB3Pad] = a3;
    const uint4 c0 = rd[0 ^ sw], c1 = rd[1 ^ sw], c2 = rd[2 ^ sw], c3 = rd[3 ^ sw];
#else
    const uint4 c0 = a0, c1 = a1, c2 = a2, c3 = a3;
#endif
    if (j + 1 < nmax) fetch(j + 1);
    if (j < nfull) {
      const uint32_t m[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                              c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
      const uint32_t b = j & 15, k = j >> 4;
      const bool last = j + 1 == nblk;
      const bool end = b == 15 || last;
      compress(cv, m, l0 + k, 64,
               (b == 0 ? kChunkStart : 0) | (end ? kChunkEnd : 0) | (root1 && last ? kRoot : 0));
      if (end && !last) {  // leaf k done and more follow: merge the completed subtrees, keep it
        uint32_t l = 0;
        while ((k >> l) & 1) {
          uint32_t left[8];
          sget(l, left);
          parent(left, cv, 0, cv);
          ++l;
        }
        sput(l, cv);
        iv(cv);
      }
    }
  }
  if (!act) return;
  if (has_tail) {  // the group's final, partial block
    const uint32_t b = nfull & 15, k = nfull >> 4;
    uint32_t m[16];
    load_block(gp + 64ull * nfull, tail, m);
    compress(cv, m, l0 + k, tail, (b == 0 ? kChunkStart : 0) | kChunkEnd | (root1 ? kRoot : 0));
  }
  // right edge: fold the kept subtrees, smallest first; the last fold is the
  // chunk's root when the group is the whole tree
  const uint32_t K = (nblk - 1) >> 4;  // leaves kept = index of the last leaf
#pragma unroll
  for (uint32_t l = 0; l < 4; ++l) {
    if ((K >> l) & 1) {
      uint32_t left[8];
      sget(l, left);
      parent(left, cv, (whole && (K >> (l + 1)) == 0) ? kRoot : 0, cv);
    }
  }
  if (whole) {
    store_id(ids + 32ull * i, cv);
  } else {
    uint4 *d = reinterpret_cast<uint4 *>(nodes + 8 * slot_idx);
    d[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    d[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
  }
}

// One lane per chunk of 2 - kTreeLaneMax groups: level-by-level pairing of its
// group nodes in place (nodes [goff[i], goff[i+1]) belong to this lane only).
// Chunks of more than kTreeLaneMax groups (over 256 KiB: mapache's own
// 512K/1M/8M chunks, up to 512 groups, and the packer's ~16 MiB packs, whose
// IDs are calculate_hash of the pack, src/utils/mod.rs:62-68) are paired by a
// whole wave (k_b3_tree_wide): per level, lanes take pairs; the levels above
// kTreeWaveMax nodes in place in HBM, the rest in LDS.  A 512-group chunk
// costs 13 wave-steps instead of 511 serial compressions on one lane (the
// tree was 11 % of a 512K/1M/8M ID pass); a 16 MiB pack ~20 instead of 1023
// (1.6-1.8 ms per kernel-tree save call on the lane path, round 5).
// k_b3_owner lists these chunks; persistent waves draw them from a counter.

// order the wave's LDS accesses (fences keep the compiler from moving a
// lane's write above another lane's read of the same node)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void k_b3_tree_wide(const uint64_t *goff, uint64_t n, uint64_t bound,
                                                     uint32_t *nodes, uint8_t *ids, const uint32_t *wide,
                                                     uint32_t *cnt) {
  __shared__ uint4 nd[2 * kTreeWaveMax];  // node j = nd[2 j], nd[2 j + 1] (16 KiB)
  const uint32_t lane = threadIdx.x;
  if (gtotal(goff[n]) > bound) return;
  const uint32_t total = cnt[0];
  // persistent waves draw chunks from the list (drawn before the loop and at
  // its end, lane 0's value read explicitly: see next_tile in mcdc_aead.hip)
  auto draw = [&]() {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(cnt + 1, 1u);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  };
  uint32_t k = draw();
  while (k < total) {
    const uint64_t i = wide[k];
    const uint64_t g0 = gtotal(goff[i]);
    uint64_t mg = gtotal(goff[i + 1]) - g0;
    uint4 *gn = reinterpret_cast<uint4 *>(nodes + 8 * g0);  // (this chunk's nodes: this wave's only)
    // levels of more than kTreeWaveMax nodes in place in HBM: batch t0 reads
    // nodes [2 t0, + 128) and writes [t0, + 64) -- each lane's store follows
    // the wave's loads of the batch (its inputs), and later batches read above
    // what earlier ones wrote; a level's stores are made visible to the next
    // level's loads by the fence (the L1 is not coherent with them)
    while (mg > kTreeWaveMax) {
      const uint64_t pairs = mg / 2;
      for (uint64_t t0 = 0; t0 < pairs; t0 += 64) {
        const uint64_t t = t0 + lane;
        uint32_t l[8], r[8], o[8];
        if (t < pairs) {
          const uint4 a = gn[4 * t], bb = gn[4 * t + 1], c = gn[4 * t + 2], d = gn[4 * t + 3];
          l[0] = a.x; l[1] = a.y; l[2] = a.z; l[3] = a.w; l[4] = bb.x; l[5] = bb.y; l[6] = bb.z; l[7] = bb.w;
          r[0] = c.x; r[1] = c.y; r[2] = c.z; r[3] = c.w; r[4] = d.x; r[5] = d.y; r[6] = d.z; r[7] = d.w;
          parent(l, r, 0, o);
        }
        __builtin_amdgcn_wave_barrier();
        if (t < pairs) {
          gn[2 * t] = make_uint4(o[0], o[1], o[2], o[3]);
          gn[2 * t + 1] = make_uint4(o[4], o[5], o[6], o[7]);
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (mg & 1) {  // the last node of an odd level moves up unchanged (it lies above every write)
        if (lane < 2) gn[2 * pairs + lane] = gn[2 * (mg - 1) + lane];
      }
      mg = pairs + (mg & 1);
      __threadfence();
    }
    uint32_t m = (uint32_t)mg;
    for (uint32_t t = lane; t < 2 * m; t += 64) nd[t] = gn[t];
    wave_lds_sync();
    while (m > 1) {
      const uint32_t pairs = m / 2;
      for (uint32_t t0 = 0; t0 < pairs; t0 += 64) {  // (batch t0 reads nodes >= 2 t0, writes nodes < t0 + 64)
        const uint32_t t = t0 + lane;
        uint32_t l[8], r[8], o[8];
        if (t < pairs) {
          const uint4 a = nd[4 * t], bb = nd[4 * t + 1], c = nd[4 * t + 2], d = nd[4 * t + 3];
          l[0] = a.x; l[1] = a.y; l[2] = a.z; l[3] = a.w; l[4] = bb.x; l[5] = bb.y; l[6] = bb.z; l[7] = bb.w;
          r[0] = c.x; r[1] = c.y; r[2] = c.z; r[3] = c.w; r[4] = d.x; r[5] = d.y; r[6] = d.z; r[7] = d.w;
          parent(l, r, m == 2 ? kRoot : 0, o);
        }
        wave_lds_sync();  // (every read of the batch before any write)
        if (t < pairs) {
          nd[2 * t] = make_uint4(o[0], o[1], o[2], o[3]);
          nd[2 * t + 1] = make_uint4(o[4], o[5], o[6], o[7]);
        }
        wave_lds_sync();
      }
      if (m & 1) {  // the last node of an odd level moves up unchanged
        if (lane < 2) nd[2 * pairs + lane] = nd[2 * (m - 1) + lane];
        wave_lds_sync();
      }
      m = pairs + (m & 1);
    }
    if (lane < 2) reinterpret_cast<uint4 *>(ids + 32ull * i)[lane] = nd[lane];
    wave_lds_sync();
    k = draw();
  }
}

__global__ void k_b3_tree(const DevChunk *chunks, const uint64_t *goff, uint64_t n, uint64_t bound, uint32_t *nodes,
                          uint8_t *ids) {
  MCDC_VGPR_PAD(48);  // 48 used: not an exact fill (MCDC_VGPR_PAD)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || gtotal(goff[n]) > bound) return;
  uint64_t m = gtotal(goff[i + 1]) - gtotal(goff[i]);
  if (m < 2) return;  // finished by k_b3_leaves
  if (m > kTreeLaneMax) return;  // k_b3_tree_wide
  uint32_t *nd = nodes + 8 * gtotal(goff[i]);
  uint32_t l[8], r[8], o[8];
  while (m > 1) {
    const uint64_t pairs = m / 2;
    for (uint64_t t = 0; t < pairs; ++t) {
#pragma unroll
      for (int w = 0; w < 8; ++w) { l[w] = nd[16 * t + w]; r[w] = nd[16 * t + 8 + w]; }
      parent(l, r, m == 2 ? kRoot : 0, o);
#pragma unroll
      for (int w = 0; w < 8; ++w) nd[8 * t + w] = o[w];
    }
    if (m & 1) {
#pragma unroll
      for (int w = 0; w < 8; ++w) nd[8 * pairs + w] = nd[8 * (m - 1) + w];
    }
    m = pairs + (m & 1);
  }
  store_id(ids + 32ull * i, o);
}

size_t b3_tmp_bytes(uint64_t nchunks) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)nchunks + 1);
  return b;
}

uint64_t b3_group_bound(uint64_t total_bytes, uint64_t nchunks) {
  return total_bytes / ((uint64_t)kGroupLeaves * kLeaf) + nchunks + 1;
}

void launch_b3_prepare(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *gcnt, uint64_t *goff,
                       uint32_t *hist, uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t stream) {
  (void)hipMemsetAsync(hist, 0, 2 * kTailBins * sizeof(uint32_t), stream);
  hipLaunchKernelGGL(k_b3_groups, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, chunks, n, nbytes,
                     gcnt, hist, err);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, gcnt, goff, (int)n + 1, stream);
}

void launch_b3_hash(const uint8_t *base, const DevChunk *chunks, uint64_t n, const uint64_t *goff,
                    uint64_t group_bound, uint32_t *hist, uint32_t *owner, uint32_t *nodes, uint8_t *ids,
                    uint64_t *gcnt, hipStream_t stream) {
  if (n == 0) return;
  // bin cursors, the wide-tree list count and draw counter
  (void)hipMemsetAsync(hist + kTailBins, 0, (kB3HistWords - kTailBins) * sizeof(uint32_t), stream);
  uint32_t *wide = reinterpret_cast<uint32_t *>(gcnt), *wcnt = hist + 2 * kTailBins;
  hipLaunchKernelGGL(k_b3_owner, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, chunks, goff, n,
                     group_bound, (const uint32_t *)hist, hist + kTailBins, owner, wide, wcnt);
  hipLaunchKernelGGL(k_b3_leaves, dim3((unsigned)((group_bound + 255) / 256)), dim3(256), 0, stream, base, chunks,
                     goff, (const uint32_t *)owner, n, group_bound, nodes, ids);
  // (at most as many waves as fit: 16 KiB of LDS each)
  hipLaunchKernelGGL(k_b3_tree_wide, dim3((unsigned)std::min<uint64_t>(n, 2048)), dim3(64), 0, stream, goff, n,
                     group_bound, nodes, ids, (const uint32_t *)wide, wcnt);
  hipLaunchKernelGGL(k_b3_tree, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, chunks, goff, n, group_bound,
                     nodes, ids);
}

uint64_t b3_groups_total(uint64_t packed) { return (packed & 0xffffffffull) + (packed >> 32); }

}  // namespace mcdc
