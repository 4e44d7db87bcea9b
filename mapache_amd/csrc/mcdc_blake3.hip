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
//   k_b3_groups   groups of 16 leaves (16 KiB) per chunk -> counts
//   (hipcub)      exclusive scan -> group offsets
//   k_b3_owner    group -> chunk map
//   k_b3_leaves   one lane per group: 16 x 16 block compressions, the group's
//                 subtree reduced on the fly (a 4-deep chaining-value stack in
//                 LDS); a chunk of <= 16 leaves finishes its ID here (ROOT)
//   k_b3_tree     one lane per larger chunk: level-by-level pairing of its
//                 group nodes (the last node of an odd level moves up
//                 unchanged — the same tree as the specification's stack rule)
// Integer VALU work (~11 32-bit ops per input byte), no MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

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

// A chunk outside [0, nbytes) of the buffer gets no groups and sets *err.
__global__ void k_b3_groups(const DevChunk *chunks, uint64_t n, uint64_t nbytes, uint64_t *gcnt, uint32_t *err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const DevChunk c = chunks[i];
    const bool ok = c.offset <= nbytes && c.length <= nbytes - c.offset;
    gcnt[i] = ok ? (leaves_of(c.length) + kGroupLeaves - 1) / kGroupLeaves : 0;
    if (!ok) atomicOr(err, 1u);
  } else if (i == n) {
    gcnt[i] = 0;
  }
}

// Every hashing kernel first checks the group total against the host's bound
// (b3_group_bound assumes disjoint chunks; overlapping or repeated chunks
// exceed it): over the bound nothing is written, and the host re-runs the
// hashing with the exact total it reads back (mcdc_chunk_ids_device).
__global__ void k_b3_owner(const uint64_t *goff, uint64_t n, uint64_t bound, uint32_t *owner) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || goff[n] > bound) return;
  for (uint64_t g = goff[i]; g < goff[i + 1]; ++g) owner[g] = (uint32_t)i;
}

// One lane per group of <= 16 leaves.  The group's subtree (a complete binary
// tree when it holds 16 leaves, the specification's tree of its leaves
// otherwise) is built with a chaining-value stack in LDS.  The main loop runs
// over the group's full 64-byte blocks only (one uniform code path for the
// whole wave); the one partial block a group can end with is hashed after it.
__global__ __launch_bounds__(256) void k_b3_leaves(const uint8_t *base, const DevChunk *chunks,
                                                   const uint64_t *goff, const uint32_t *owner, uint64_t n,
                                                   uint64_t bound, uint32_t *nodes, uint8_t *ids) {
  __shared__ uint32_t stk[256][4][8];
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = goff[n];
  if (g >= total || total > bound) return;  // the grid is sized by the host bound
  const uint32_t i = owner[g];
  const DevChunk ch = chunks[i];
  const uint32_t nleaves = leaves_of(ch.length);
  const uint64_t gi = g - goff[i];                      // group index within the chunk
  const uint64_t l0 = gi * kGroupLeaves;                // first leaf of the group
  const bool whole = nleaves <= kGroupLeaves;           // this group is the chunk's whole tree
  const bool root1 = nleaves == 1;                      // ... and its only leaf is the root
  const uint64_t grem = ch.length - l0 * kLeaf;
  const uint32_t gbytes = (uint32_t)(grem < (uint64_t)(kGroupLeaves * kLeaf) ? grem : kGroupLeaves * kLeaf);
  const uint32_t nfull = gbytes / 64, tail = gbytes % 64;
  const bool has_tail = tail != 0 || gbytes == 0;       // (the empty input is one empty block)
  const uint32_t nblk = nfull + (has_tail ? 1u : 0u);
  const uint8_t *p = base + ch.offset + l0 * kLeaf;
  const uint32_t r = (uint32_t)((uintptr_t)p & 3);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(p - r);  // (stays a global pointer)
  uint32_t (*st)[8] = stk[threadIdx.x];
  uint32_t cv[8];
  iv(cv);
  int sp = 0;
  // Block j + 1 is requested before block j is compressed: a wave waits on
  // memory only when its next block has not arrived during a whole
  // compression, which keeps enough waves ready for the VALU's dual-rate issue
  // (tools/ubench3.hip: the G mix runs at 2 cycles per instruction with 4 ready
  // waves per SIMD, 4 with 2).
  uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0, n2 = n0, n3 = n0;
  uint32_t n16 = 0;
  // (loads are unconditional — the last iteration re-reads its own block —
  // so no wait is forced at a control-flow join)
  auto fetch = [&](const uint32_t *ww) {
    n0 = *reinterpret_cast<const uint4 *>(ww);
    n1 = *reinterpret_cast<const uint4 *>(ww + 4);
    n2 = *reinterpret_cast<const uint4 *>(ww + 8);
    n3 = *reinterpret_cast<const uint4 *>(ww + 12);
    const uint32_t x = ww[r ? 16 : 15];  // dword 16 holds the block's last bytes only when misaligned
    n16 = r ? x : 0u;
  };
  if (nfull) fetch(w);
#pragma unroll 1
  for (uint32_t j = 0; j < nfull; ++j, w += 16) {
    const uint32_t b = j & 15, k = j >> 4;
    uint32_t m[16];
    {
      const uint4 q0 = n0, q1 = n1, q2 = n2, q3 = n3;
      const uint32_t x16 = n16;
      fetch(j + 1 < nfull ? w + 16 : w);
      const uint32_t raw[17] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w, x16};
#pragma unroll
      for (int t = 0; t < 16; ++t) m[t] = __builtin_amdgcn_alignbyte(raw[t + 1], raw[t], r);
    }
    const bool last = j + 1 == nblk;
    const bool end = b == 15 || last;
    compress(cv, m, l0 + k, 64,
             (b == 0 ? kChunkStart : 0) | (end ? kChunkEnd : 0) | (root1 && last ? kRoot : 0));
    if (end && !last) {  // leaf k done and more follow: push it, merging completed subtrees
      for (uint32_t t = k + 1; (t & 1) == 0; t >>= 1) {
        --sp;
        parent(st[sp], cv, 0, cv);
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) st[sp][t] = cv[t];
      ++sp;
      iv(cv);
    }
  }
  if (has_tail) {  // the group's final, partial block
    const uint32_t b = nfull & 15, k = nfull >> 4;
    uint32_t m[16];
    load_block(p + 64ull * nfull, tail, m);
    compress(cv, m, l0 + k, tail, (b == 0 ? kChunkStart : 0) | kChunkEnd | (root1 ? kRoot : 0));
  }
  while (sp > 0) {  // right edge; the top node is the chunk's root when `whole`
    --sp;
    parent(st[sp], cv, (whole && sp == 0) ? kRoot : 0, cv);
  }
  if (whole) {
    store_id(ids + 32ull * i, cv);
  } else {
    uint4 *d = reinterpret_cast<uint4 *>(nodes + 8 * g);
    d[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    d[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
  }
}

// One lane per chunk of more than one group: level-by-level pairing of its
// group nodes in place (nodes [goff[i], goff[i+1]) belong to this lane only).
__global__ void k_b3_tree(const DevChunk *chunks, const uint64_t *goff, uint64_t n, uint64_t bound, uint32_t *nodes,
                          uint8_t *ids) {
  MCDC_VGPR_PAD(48);  // 48 used: not an exact fill (MCDC_VGPR_PAD)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || goff[n] > bound) return;
  uint64_t m = goff[i + 1] - goff[i];
  if (m < 2) return;  // finished by k_b3_leaves
  uint32_t *nd = nodes + 8 * goff[i];
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
                       uint32_t *err, void *tmp, size_t tmp_bytes, hipStream_t stream) {
  hipLaunchKernelGGL(k_b3_groups, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, chunks, n, nbytes,
                     gcnt, err);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, gcnt, goff, (int)n + 1, stream);
}

void launch_b3_hash(const uint8_t *base, const DevChunk *chunks, uint64_t n, const uint64_t *goff,
                    uint64_t group_bound, uint32_t *owner, uint32_t *nodes, uint8_t *ids, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_b3_owner, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, goff, n, group_bound, owner);
  hipLaunchKernelGGL(k_b3_leaves, dim3((unsigned)((group_bound + 255) / 256)), dim3(256), 0, stream, base, chunks,
                     goff, (const uint32_t *)owner, n, group_bound, nodes, ids);
  hipLaunchKernelGGL(k_b3_tree, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, chunks, goff, n, group_bound,
                     nodes, ids);
}

}  // namespace mcdc
