// mcdc_aead.hip — CDNA4 (gfx950) SecureStorage sealing: AES-256-GCM-SIV
// (RFC 8452) of many blobs at once, in HBM.
//
// Replaces, for mapache's save path, SecureStorage::encrypt_with_key /
// decrypt_with_key (/root/reference/src/repository/storage.rs:97-118,
// 128-144; crate aes-gcm-siv 0.11.1): per blob a 12-byte nonce, no AAD, and
// the output nonce || ciphertext || tag.  Per nonce (RFC 8452 §4) the
// key-generating key encrypts six blocks le32(i) || nonce; their first halves
// give the authentication key H (blocks 0-1) and the AES-256 encryption key
// (blocks 2-5).  The tag is AES(enc, (POLYVAL_H(plaintext blocks, length block)
// ^ nonce) with bit 127 cleared); the ciphertext is AES-CTR under enc from the
// tag with bit 127 set and a little-endian 32-bit counter in bytes 0-3.
//
// GPU shape.  A blob is cut into tiles of up to 64 rows of 64
// 16-byte blocks; one wave works one tile, lane l on blocks l, l+64, ... so a
// row is one coalesced 1-KiB access.
//   k_aead_sizes   output bytes and tiles per blob; two hipcub scans
//   k_aead_prep    one lane per blob: the blob record, the tile -> blob map,
//                  the six key-derivation blocks, the AES-256 key schedule and
//                  the POLYVAL powers H^1..H^64, H^4096
//   k_aead_polyval one wave per tile: each lane runs Horner with G = H^64 over
//                  its strided blocks using a 256-entry table of y·G in LDS
//                  (16 lookups and 16 byte-steps per block), multiplies by
//                  H^(64-l), and the wave XOR-reduces to the tile's sum
//   k_aead_tag     one lane per blob: tiles combined with H^4096, length
//                  block, nonce, AES -> tag (open: compared with the stored tag)
//   k_aead_ctr     one wave per tile: one AES-256 block per lane per row
//                  (T-table, 32 replicas in LDS so that every lookup is
//                  conflict-free), the keystream shifted one lane (DPP
//                  wave_shr) to the output's 16-byte alignment, plaintext read
//                  at any alignment, aligned 16-byte stores; the nonce and tag
//                  bytes go out with the first and last quads of the blob
// Integer VALU + LDS work, no MFMA (AES and GF(2^128) have no MFMA form).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "mcdc_aead.h"
#include "mcdc_internal.h"

namespace mcdc {

namespace aead {

// ------------------------------------------------------------- tables ---
struct Tables {
  uint8_t sbox[256];
  uint32_t te0[256];  // little-endian column word of MixColumns(S[x] in row 0): (2s, s, s, 3s)
};

constexpr uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
constexpr uint8_t rot8(uint8_t x, int k) { return (uint8_t)((x << k) | (x >> (8 - k))); }

constexpr Tables make_tables() {
  Tables t{};
  uint8_t ex[256] = {}, lg[256] = {};
  uint8_t x = 1;
  for (int i = 0; i < 255; ++i) {  // powers of the generator 3
    ex[i] = x;
    lg[x] = (uint8_t)i;
    x = (uint8_t)(x ^ xt(x));
  }
  for (int i = 0; i < 256; ++i) {
    const uint8_t inv = i ? ex[(255 - lg[i]) % 255] : 0;
    const uint8_t s = (uint8_t)(inv ^ rot8(inv, 1) ^ rot8(inv, 2) ^ rot8(inv, 3) ^ rot8(inv, 4) ^ 0x63);
    t.sbox[i] = s;
    const uint8_t s2 = xt(s), s3 = (uint8_t)(s2 ^ s);
    t.te0[i] = (uint32_t)s2 | (uint32_t)s << 8 | (uint32_t)s << 16 | (uint32_t)s3 << 24;
  }
  return t;
}

constexpr Tables kHostTab = make_tables();
static_assert(kHostTab.sbox[0] == 0x63 && kHostTab.sbox[0x53] == 0xED && kHostTab.sbox[0xFF] == 0x16, "S-box");
__constant__ Tables kDevTab = make_tables();

#ifndef MCDC_CTR_WAVES
#define MCDC_CTR_WAVES 12
#endif
#ifndef MCDC_PV_NIB  // POLYVAL row step from 32 nibble tables (1) or one byte table with x^-8 steps (0)
#define MCDC_PV_NIB 1
#endif
#ifndef MCDC_AEAD_PERSIST  // bit 0: k_aead_polyval, bit 1: k_aead_ctr draw tiles from a counter (A/B: tools/dbg/build_persist_ab.sh)
#define MCDC_AEAD_PERSIST 3
#endif
#ifndef MCDC_CTR_ILP
#define MCDC_CTR_ILP 1
#endif
// k_aead_ctr: waves per block, all sharing one 64-KiB table; two blocks per
// CU.  12: 73 VGPRs -> 6 waves per SIMD (A/B over 8-16, tools/dbg/build_ctr_ab.sh:
// 12 fastest; 16 fills 64 of 64 VGPRs, see MCDC_VGPR_PAD, and is SGPR-bound at 7).
constexpr int kCtrWaves = MCDC_CTR_WAVES;
constexpr int kRep = 32;  // T-table replicas: ds_read_b32 banks are (addr/4) mod 32 per 32-lane half
constexpr int kTabWords = 256 * kRep;

__device__ __forceinline__ void fill_table(uint32_t *tt) {
  for (int k = threadIdx.x; k < kTabWords; k += blockDim.x) tt[k] = kDevTab.te0[k / kRep];
  __syncthreads();
}

// ---------------------------------------------------------------- AES ---
__device__ __forceinline__ uint32_t rl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rl24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }
// tl = table + (lane % 32): entry x of this lane's replica
__device__ __forceinline__ uint32_t te(const uint32_t *tl, uint32_t x) { return tl[x * kRep]; }
__device__ __forceinline__ uint32_t sb(const uint32_t *tl, uint32_t x) { return (te(tl, x) >> 8) & 0xffu; }

// AES-256 encryption of one block; rk: 60 words (registers or uniform memory)
__device__ __forceinline__ uint4 aes256(const uint32_t *tl, const uint32_t *rk, uint4 in) {
  uint32_t a0 = in.x ^ rk[0], a1 = in.y ^ rk[1], a2 = in.z ^ rk[2], a3 = in.w ^ rk[3];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const uint32_t b0 = te(tl, a0 & 255) ^ rl8(te(tl, (a1 >> 8) & 255)) ^ rl16(te(tl, (a2 >> 16) & 255)) ^
                        rl24(te(tl, a3 >> 24)) ^ rk[4 * r];
    const uint32_t b1 = te(tl, a1 & 255) ^ rl8(te(tl, (a2 >> 8) & 255)) ^ rl16(te(tl, (a3 >> 16) & 255)) ^
                        rl24(te(tl, a0 >> 24)) ^ rk[4 * r + 1];
    const uint32_t b2 = te(tl, a2 & 255) ^ rl8(te(tl, (a3 >> 8) & 255)) ^ rl16(te(tl, (a0 >> 16) & 255)) ^
                        rl24(te(tl, a1 >> 24)) ^ rk[4 * r + 2];
    const uint32_t b3 = te(tl, a3 & 255) ^ rl8(te(tl, (a0 >> 8) & 255)) ^ rl16(te(tl, (a1 >> 16) & 255)) ^
                        rl24(te(tl, a2 >> 24)) ^ rk[4 * r + 3];
    a0 = b0;
    a1 = b1;
    a2 = b2;
    a3 = b3;
  }
  // last round: SubBytes + ShiftRows; S[x] is byte 1 (and 2) of Te0[x]
  auto fin = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t k) {
    return (((te(tl, x0 & 255) >> 8) & 0xffu) | (te(tl, (x1 >> 8) & 255) & 0xff00u) |
            (te(tl, (x2 >> 16) & 255) & 0xff0000u) | ((te(tl, x3 >> 24) << 8) & 0xff000000u)) ^
           k;
  };
  return make_uint4(fin(a0, a1, a2, a3, rk[56]), fin(a1, a2, a3, a0, rk[57]), fin(a2, a3, a0, a1, rk[58]),
                    fin(a3, a0, a1, a2, rk[59]));
}

// The CTR kernel's AES: Te0 with 64 replicas, entry x of lane l's replica at
// byte x * 256 + 4 l (64 KiB), so one v_perm_b32 builds a lookup's LDS address
// from the state word (byte k -> bits 8-15) and 4 l (bits 0-7); ds_read_b32
// banks are (addr / 4) mod 32, so the 32 lanes of a half hit 32 banks.
// v_bitop3_b32 merges three terms per instruction.  ~500 VALU + 224 LDS reads
// per block (the 32-replica version above: ~850 VALU).
//
// MCDC_AES_2T (default): ds_read_b32 serves 32-lane groups with banks
// (a / 4) mod 32 (MI355X_MICROARCH.md, LDS table), so 32 replicas are
// conflict-free too, and the same 64 KiB hold two tables: row x = Te0[x] for
// lanes l mod 32 at 4 l, then Te2[x] = rotl16(Te0[x]) at 128 + 4 l.  A column
// T0(a) ^ rotl8 T0(b) ^ rotl16 T0(c) ^ rotl24 T0(d) ^ k is then
// [T0(a) ^ T2(c) ^ k] ^ rotl8[T0(b) ^ T2(d)]: one rotate instead of three
// (8 VALU per column with the four address perms instead of 9).
#ifndef MCDC_AES_2T
#define MCDC_AES_2T 1
#endif
constexpr int kRepP = 64;
constexpr int kTabPWords = 256 * kRepP;

__device__ __forceinline__ void fill_table_p(uint32_t *tt) {
  for (int k = threadIdx.x; k < kTabPWords; k += blockDim.x) {
    const uint32_t t = kDevTab.te0[k / kRepP];
    tt[k] = (MCDC_AES_2T && (k & 32)) ? __builtin_amdgcn_alignbit(t, t, 16) : t;
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int K>
__device__ __forceinline__ uint32_t tp(const uint8_t *tb, uint32_t w, uint32_t lane4) {
  const uint32_t a = __builtin_amdgcn_perm(w, lane4, 0x0c0c0000u | ((4u + K) << 8));  // (byte K of w) << 8 | 4 l
  return *reinterpret_cast<const uint32_t *>(tb + a);
}

// N independent blocks per call: N x 16 lookups per round in flight per lane,
// which is what hides the LDS latency (one block per lane left the LDS ~50 %
// and the VALU ~30 % busy, PMC: tools/aead_pmc.sh).
template <int N>
__device__ __forceinline__ void aes256p(const uint8_t *tb, uint32_t lane4, const uint32_t *rk, uint4 (&st)[N]) {
  uint32_t a[N][4];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    a[j][0] = st[j].x ^ rk[0];
    a[j][1] = st[j].y ^ rk[1];
    a[j][2] = st[j].z ^ rk[2];
    a[j][3] = st[j].w ^ rk[3];
  }
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    uint32_t b[N][4];
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#if MCDC_AES_2T
        const uint32_t w = tp<1>(tb, a[j][(c + 1) & 3], lane4) ^ tp<3>(tb, a[j][(c + 3) & 3], lane4 | 128u);
        b[j][c] = xor3(tp<0>(tb, a[j][c], lane4), tp<2>(tb, a[j][(c + 2) & 3], lane4 | 128u), rk[4 * r + c]) ^ rl8(w);
#else
        b[j][c] = xor3(xor3(tp<0>(tb, a[j][c], lane4), rl8(tp<1>(tb, a[j][(c + 1) & 3], lane4)),
                            rl16(tp<2>(tb, a[j][(c + 2) & 3], lane4))),
                       rl24(tp<3>(tb, a[j][(c + 3) & 3], lane4)), rk[4 * r + c]);
#endif
      }
    }
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) a[j][c] = b[j][c];
  }
  // last round: S[x] = byte 1 of Te0[x]; two perms gather the four S bytes, then (u | v) ^ k
#pragma unroll
  for (int j = 0; j < N; ++j) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t u = __builtin_amdgcn_perm(tp<1>(tb, a[j][(c + 1) & 3], lane4), tp<0>(tb, a[j][c], lane4),
                                               0x0c0c0501u);
      const uint32_t v = __builtin_amdgcn_perm(tp<3>(tb, a[j][(c + 3) & 3], lane4),
                                               tp<2>(tb, a[j][(c + 2) & 3], lane4), 0x05010c0cu);
      o[c] = __builtin_amdgcn_bitop3_b32(u, v, rk[56 + c], 0x56);  // (u | v) ^ k
    }
    st[j] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// FIPS-197 §5.2 for Nk = 8, words little-endian (RotWord = rotate right 8)
__device__ __forceinline__ void expand256(const uint32_t *tl, const uint32_t k[8], uint32_t rk[60]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) rk[i] = k[i];
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 8; i < 60; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 8 == 0) t = __builtin_amdgcn_alignbit(t, t, 8);
    if (i % 8 == 0 || i % 8 == 4)
      t = sb(tl, t & 255) | sb(tl, (t >> 8) & 255) << 8 | sb(tl, (t >> 16) & 255) << 16 | sb(tl, t >> 24) << 24;
    if (i % 8 == 0) {
      t ^= rcon;
      rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11b : 0);
    }
    rk[i] = rk[i - 8] ^ t;
  }
}

// ------------------------------------------------------------ POLYVAL ---
// Field element = 16 bytes as a little-endian 128-bit integer (bit i = x^i),
// modulus x^128 + x^127 + x^126 + x^121 + 1; dot(a, b) = a b x^-128.

// dot(a, b) bit by bit, LSB first: r = (r + b_i a) x^-1
__device__ __attribute__((noinline)) uint4 dotb(uint4 a, uint4 b) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t bk = bw[k];
#pragma unroll 8
    for (int i = 0; i < 32; ++i) {
      const uint32_t m = 0u - ((bk >> i) & 1u);
      r0 ^= a.x & m;
      r1 ^= a.y & m;
      r2 ^= a.z & m;
      r3 ^= a.w & m;
      const uint32_t odd = 0u - (r0 & 1u);
      r0 = __builtin_amdgcn_alignbit(r1, r0, 1);
      r1 = __builtin_amdgcn_alignbit(r2, r1, 1);
      r2 = __builtin_amdgcn_alignbit(r3, r2, 1);
      r3 = (r3 >> 1) ^ (odd & 0xe1000000u);  // + P, then / x: P/x = x^127 + x^126 + x^125 + x^120
    }
  }
  return make_uint4(r0, r1, r2, r3);
}

// v x mod P
__device__ __forceinline__ uint4 mulx(uint4 v) {
  const uint32_t c = 0u - (v.w >> 31);
  return make_uint4((v.x << 1) ^ (c & 1u), __builtin_amdgcn_alignbit(v.y, v.x, 31),
                    __builtin_amdgcn_alignbit(v.z, v.y, 31),
                    __builtin_amdgcn_alignbit(v.w, v.z, 31) ^ (c & 0xc2000000u));
}

// dot(y, G) with M[b] = b(x) G mod P: Z = (Z + M[y_k]) x^-8 for bytes k = 0..15.
// x^-8: the low byte z cancels against z P; z (x^128 + x^127 + x^126 + x^121)
// / x^8 lands in the top word as z << 17 ^ z << 22 ^ z << 23 ^ z << 24.
__device__ __forceinline__ uint4 m8mul(const uint4 *M, uint4 y) {
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint4 m = M[(yw[k >> 2] >> (8 * (k & 3))) & 255];
    z0 ^= m.x;
    z1 ^= m.y;
    z2 ^= m.z;
    z3 ^= m.w;
    const uint32_t lo = z0 & 255;
    z0 = __builtin_amdgcn_alignbit(z1, z0, 8);
    z1 = __builtin_amdgcn_alignbit(z2, z1, 8);
    z2 = __builtin_amdgcn_alignbit(z3, z2, 8);
    z3 = (z3 >> 8) ^ (lo << 17) ^ (lo << 22) ^ (lo << 23) ^ (lo << 24);
  }
  return make_uint4(z0, z1, z2, z3);
}

// ------------------------------------------------------------ memory ---
__device__ __forceinline__ uint4 u4xor(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

// bytes [e, e + 16) of a || b (e in 0..15)
__device__ __forceinline__ uint4 shift16(uint4 a, uint4 b, uint32_t e) {
  const uint32_t s = e & 3;
  uint32_t w0, w1, w2, w3, w4;
  switch (e >> 2) {
    case 0: w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; break;
    case 1: w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; break;
    case 2: w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; break;
    default: w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, s), __builtin_amdgcn_alignbyte(w2, w1, s),
                    __builtin_amdgcn_alignbyte(w3, w2, s), __builtin_amdgcn_alignbyte(w4, w3, s));
}

// bytes [f, t) of a 4-byte word kept, the rest zero
__device__ __forceinline__ uint32_t keep4(uint32_t w, int64_t f, int64_t t) {
  const uint32_t lo = f <= 0 ? 0xffffffffu : f >= 4 ? 0u : 0xffffffffu << (8 * f);
  const uint32_t hi = t >= 4 ? 0xffffffffu : t <= 0 ? 0u : 0xffffffffu >> (32 - 8 * t);
  return w & lo & hi;
}

// 16 bytes at address a (e = a % 16, passed wave-uniform); bytes outside
// [lo, hi) read as zero, and only 16-byte quads holding a byte of [lo, hi)
// are touched (so nothing outside the caller's buffer is read).
__device__ __forceinline__ uint4 load16(uint64_t a, uint64_t lo, uint64_t hi, uint32_t e) {
  const uint64_t q = a - e;
  uint4 l0 = make_uint4(0, 0, 0, 0), l1 = l0;
  if (q + 16 > lo && q < hi) l0 = *reinterpret_cast<const uint4 *>(q);
  if (e && q + 32 > lo && q + 16 < hi) l1 = *reinterpret_cast<const uint4 *>(q + 16);
  uint4 r = shift16(l0, l1, e);
  if (a < lo || a + 16 > hi) {
    const int64_t f = (int64_t)(lo - a), t = (int64_t)(hi - a);
    r = make_uint4(keep4(r.x, f, t), keep4(r.y, f - 4, t - 4), keep4(r.z, f - 8, t - 8), keep4(r.w, f - 12, t - 12));
  }
  return r;
}

__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t k) {
  const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
  return (w >> (8 * (k & 3))) & 0xffu;
}

// POLYVAL tiles: the last ones hold kAeadRows rows each, the first the rest;
// a first tile under half that joins the next (up to 1.5 x kAeadRows rows):
// every tile ends with one per-lane H^(64 - l) multiply (~1.5 K VALU per lane)
// and a wave reduction, which cost as much as ~11 rows' lookups.
__device__ __forceinline__ uint64_t ptiles_of(uint64_t s) {
  const uint64_t nblk = (s + 15) / 16, rows = (nblk + 63) / 64;
  const uint64_t pt = (rows + kAeadRows - 1) / kAeadRows;
  return pt > 1 && rows - kAeadRows * (pt - 1) < kAeadRows / 2 ? pt - 1 : pt;
}

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

}  // namespace aead

using namespace aead;

// ------------------------------------------------------------ kernels ---
__global__ void k_aead_sizes(int open, const uint64_t *ext, uint64_t n, uint64_t n_in, uint64_t *olen,
                             uint64_t *tcnt, uint32_t *err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t off = ext[2 * i], len = ext[2 * i + 1];
    if (!(off <= n_in && len <= n_in - off)) {
      atomicOr(err, 1u);
      olen[i] = 0;
      tcnt[i] = 0;
      return;
    }
    const bool has = !open || len >= kAeadOverhead;
    const uint64_t s = open ? (has ? len - kAeadOverhead : 0) : len;
    const uint64_t T = has ? (open ? s : s + kAeadOverhead) : 0;
    const uint64_t ct = T ? ((T - 1) / 16 + 2 + kAeadTileBlocks - 1) / kAeadTileBlocks : 0;
    const uint64_t pt = ptiles_of(s);
    olen[i] = T;
    tcnt[i] = ct > pt ? ct : pt;
  } else if (i == n) {
    olen[n] = 0;
    tcnt[n] = 0;
  }
}

// Blob extents from a boundary list (offset, length, hash records).
__global__ void k_aead_from_chunks(const uint64_t *chunks, uint64_t n, uint64_t *ext) {
  MCDC_VGPR_PAD(8);  // 8 used: not an exact fill (MCDC_VGPR_PAD)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    ext[2 * i] = chunks[3 * i];
    ext[2 * i + 1] = chunks[3 * i + 1];
  }
}

void launch_aead_from_chunks(const void *chunks, uint64_t n, uint64_t *ext, hipStream_t stream) {
  if (n)
    hipLaunchKernelGGL(k_aead_from_chunks, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                       (const uint64_t *)chunks, n, ext);
}

// One lane per blob.
__global__ __launch_bounds__(256) void k_aead_prep(int open, AeadMaster mk, const uint8_t *in, const uint64_t *ext,
                                                   const uint32_t *nonces, uint64_t n, uint8_t *out,
                                                   const uint64_t *ooff, const uint64_t *toff, AeadRec *rec,
                                                   AeadKeys *keys, uint32_t *owner) {
  __shared__ uint32_t tt[kTabWords];
  fill_table(tt);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t *tl = tt + (threadIdx.x % kRep);
  const uint64_t off = ext[2 * i], len = ext[2 * i + 1];
  AeadRec R{};
  R.tile0 = toff[i];
  for (uint64_t t = R.tile0; t < toff[i + 1]; ++t) owner[t] = (uint32_t)i;
  const uint64_t base = (uint64_t)(uintptr_t)in + off;
  if (open) {
    R.ok = len >= kAeadOverhead;
    R.len = R.ok ? len - kAeadOverhead : 0;
    R.src = base + kAeadNonce;
    R.dst = (uint64_t)(uintptr_t)out + ooff[i];
    R.ext = R.dst;
    R.pv = R.dst;
    if (R.ok) {
      const uint4 nv = load16(base, base, base + len, (uint32_t)(base & 15));
      const uint64_t ta = base + len - kAeadTag;
      const uint4 tg = load16(ta, base, base + len, (uint32_t)(ta & 15));
      R.nonce[0] = nv.x;
      R.nonce[1] = nv.y;
      R.nonce[2] = nv.z;
      R.tag[0] = tg.x;
      R.tag[1] = tg.y;
      R.tag[2] = tg.z;
      R.tag[3] = tg.w;
    }
  } else {
    R.ok = 1;
    R.len = len;
    R.src = base;
    R.ext = (uint64_t)(uintptr_t)out + ooff[i];
    R.dst = R.ext + kAeadNonce;
    R.pv = R.src;
    R.nonce[0] = nonces[3 * i];
    R.nonce[1] = nonces[3 * i + 1];
    R.nonce[2] = nonces[3 * i + 2];
  }
  R.ptiles = (uint32_t)ptiles_of(R.len);
  rec[i] = R;
  if (!R.ok) return;
  // RFC 8452 §4: AES_K(le32(j) || nonce), j = 0..5, first 8 bytes of each
  uint4 o[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) o[j] = aes256(tl, mk.rk, make_uint4((uint32_t)j, R.nonce[0], R.nonce[1], R.nonce[2]));
  const uint4 H = make_uint4(o[0].x, o[0].y, o[1].x, o[1].y);
  const uint32_t k8[8] = {o[2].x, o[2].y, o[3].x, o[3].y, o[4].x, o[4].y, o[5].x, o[5].y};
  uint32_t rk[60];
  expand256(tl, k8, rk);
  AeadKeys &K = keys[i];
#pragma unroll
  for (int j = 0; j < 60; j += 4) *reinterpret_cast<uint4 *>(&K.rk[j]) = make_uint4(rk[j], rk[j + 1], rk[j + 2], rk[j + 3]);
  *reinterpret_cast<uint4 *>(K.h) = H;
  uint4 w = H;
  *reinterpret_cast<uint4 *>(K.w[63]) = H;
  for (int j = 62; j >= 0; --j) {
    w = dotb(w, H);
    *reinterpret_cast<uint4 *>(K.w[j]) = w;
  }
#if MCDC_PV_NIB
  {  // the row step U -> dot(U, G) is linear: its images of x^j, j = 0..127
    uint4 b = dotb(w, make_uint4(1, 0, 0, 0));  // G x^-128
    *reinterpret_cast<uint4 *>(K.bas[0]) = b;
    for (int j = 1; j < 128; ++j) {
      b = mulx(b);
      *reinterpret_cast<uint4 *>(K.bas[j]) = b;
    }
  }
#endif
  for (int j = 0; j < 6; ++j) w = dotb(w, w);  // (H^64)^64
  *reinterpret_cast<uint4 *>(K.h4096) = w;
}

// Order LDS writes of a wave before its own later reads (wave-private tables).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The wave's next tile from the launch's counter (persistent waves: a wave
// that drew a short tile draws again instead of idling in its block).  Lane
// 0 draws, and lane 0's value is read explicitly (readlane, not
// readfirstlane).  Call it only in wave-uniform control flow, outside the loop
// condition: with the draw at the head of `for (;;)` the compiler lowered the
// loop exit as divergent and some waves re-drew tile 0 forever (a hang of
// every call with fewer tiles than waves, round 3).
__device__ __forceinline__ uint32_t next_tile(uint32_t *ctr) {
  uint32_t t = 0;
  if ((threadIdx.x & 63) == 0) t = atomicAdd(ctr, 1u);
  return (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
}

// dot(y, G) = XOR over the 32 nibbles k of y of T_k[nibble], T_k[e] =
// sum over the set bits i of e of bas[4 k + i] (AeadKeys::bas): 32 conflict-
// free ds_read_b128 (a table's 16 entries cover the 64 banks once; lanes
// reading one entry broadcast) and no shifts or reductions — the byte-table
// form (m8mul) spent ~385 VALU per block on its x^-8 steps and read a 4 KiB
// table at random (60 % of its LDS cycles bank conflicts).
// (nibble at bit S) << 4 | lb in two VALU ops (v_bfe_u32 + v_lshl_or_b32;
// the compiler's own form of the same expression took 2.6)
template <int S>
__device__ __forceinline__ uint32_t nib_addr(uint32_t w, uint32_t lb) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, 4\n\tv_lshl_or_b32 %0, %0, 4, %3" : "=&v"(r) : "v"(w), "i"(S), "v"(lb));
  return r;
}

typedef uint32_t pv_u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(3))) pv_u32x4 *lds_u4;
typedef const __attribute__((address_space(1))) pv_u32x4 *glb_u4;

// 16 bytes at a 16-byte aligned global address (one global_load_dwordx4)
__device__ __forceinline__ uint4 gld16(uint64_t a) {
  const pv_u32x4 v = *reinterpret_cast<glb_u4>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// two nibbles (J, J + 1) of word w, tables 8 D + J and 8 D + J + 1
template <int D, int J>
__device__ __forceinline__ void nib2(uint32_t w, uint32_t lb, uint32_t &z0, uint32_t &z1, uint32_t &z2,
                                     uint32_t &z3) {
  const uint32_t oa = nib_addr<4 * J>(w, lb), ob = nib_addr<4 * J + 4>(w, lb);
  const pv_u32x4 a = *reinterpret_cast<lds_u4>((uintptr_t)(oa + 256 * (8 * D + J)));
  const pv_u32x4 b = *reinterpret_cast<lds_u4>((uintptr_t)(ob + 256 * (8 * D + J + 1)));
  z0 = xor3(z0, a.x, b.x);
  z1 = xor3(z1, a.y, b.y);
  z2 = xor3(z2, a.z, b.z);
  z3 = xor3(z3, a.w, b.w);
}

template <int D>
__device__ __forceinline__ void nibword(uint32_t w, uint32_t lb, uint32_t &z0, uint32_t &z1, uint32_t &z2,
                                        uint32_t &z3) {
  nib2<D, 0>(w, lb, z0, z1, z2, z3);
  nib2<D, 2>(w, lb, z0, z1, z2, z3);
  nib2<D, 4>(w, lb, z0, z1, z2, z3);
  nib2<D, 6>(w, lb, z0, z1, z2, z3);
}

__device__ __forceinline__ uint4 nibmul(const uint4 *T, uint4 y) {
  // the tables' LDS address (the low 32 bits of the generic pointer) is a
  // multiple of 8 KiB, so a lookup's address is the nibble ORed into it; the
  // table number goes into the ds_read offset
  const uint32_t lb = (uint32_t)reinterpret_cast<uintptr_t>(T);
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  nibword<0>(y.x, lb, z0, z1, z2, z3);
  nibword<1>(y.y, lb, z0, z1, z2, z3);
  nibword<2>(y.z, lb, z0, z1, z2, z3);
  nibword<3>(y.w, lb, z0, z1, z2, z3);
  return make_uint4(z0, z1, z2, z3);
}

// One POLYVAL tile: its sum, exponents relative to its end.
__device__ __forceinline__ void polyval_tile(const AeadRec *__restrict__ rec, const AeadKeys *__restrict__ keys,
                                             uint4 *M, uint32_t lane, uint32_t i, uint32_t t, uint32_t tile,
                                             uint4 *__restrict__ tsum) {
#if MCDC_PV_NIB
  {  // the 32 nibble tables: lane builds entries 8 (lane & 1) .. + 8 of table lane >> 1
    const uint32_t k = lane >> 1;
    const uint4 *bs = reinterpret_cast<const uint4 *>(keys[i].bas[4 * k]);
    const uint4 b0 = bs[0], b1 = bs[1], b2 = bs[2], b3 = bs[3];
    const uint4 hi = (lane & 1) ? b3 : make_uint4(0, 0, 0, 0);
    wave_sync();  // the previous tile's reads of the tables are done
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      uint4 v = hi;
      if (e & 1) v = u4xor(v, b0);
      if (e & 2) v = u4xor(v, b1);
      if (e & 4) v = u4xor(v, b2);
      M[16 * k + 8 * (lane & 1) + e] = v;
    }
    wave_sync();
  }
#else
  {  // M[b] = b(x) G, G = H^64: lane builds entries lane + 64 q
    uint4 base[8];
    base[0] = *reinterpret_cast<const uint4 *>(keys[i].w[0]);
#pragma unroll
    for (int j = 1; j < 8; ++j) base[j] = mulx(base[j - 1]);
    wave_sync();  // the previous tile's reads of M are done
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t e = lane + 64 * q;
      uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t m = 0u - ((e >> j) & 1u);
        v = make_uint4(v.x ^ (base[j].x & m), v.y ^ (base[j].y & m), v.z ^ (base[j].z & m), v.w ^ (base[j].w & m));
      }
      M[e] = v;
    }
    wave_sync();
  }
#endif
  const AeadRec &R = rec[i];
  const uint64_t s = R.len, nblk = (s + 15) / 16, V = (nblk + 63) / 64 * 64, rows_all = V / 64;
  const uint64_t rows0 = rows_all - (uint64_t)kAeadRows * (R.ptiles - 1);
  const uint64_t vstart = t == 0 ? 0 : 64 * (rows0 + (uint64_t)kAeadRows * (t - 1));
  const uint32_t rows = (uint32_t)(t == 0 ? rows0 : kAeadRows);
  const uint64_t pad = V - nblk;
  const uint64_t lo = R.pv, hi = R.pv + s;
  const uint64_t a0 = R.pv - 16 * pad + 16 * (vstart + lane);  // (virtual block v at pv + 16 (v - pad))
  const uint32_t e = rfl((uint32_t)(R.pv & 15));  // (wave-uniform: scalar branches in load16)
  uint4 U = make_uint4(0, 0, 0, 0);
  uint4 X = load16(a0, lo, hi, e);
  // a row whose 1 KiB lies inside [lo, hi) needs no per-lane bounds (wave-uniform test)
  const uint64_t rb = ((uint64_t)rfl((uint32_t)((a0 - 16 * lane) >> 32)) << 32) | rfl((uint32_t)(a0 - 16 * lane));
  const uint64_t lo_u = ((uint64_t)rfl((uint32_t)(lo >> 32)) << 32) | rfl((uint32_t)lo);
  const uint64_t hi_u = ((uint64_t)rfl((uint32_t)(hi >> 32)) << 32) | rfl((uint32_t)hi);
#pragma unroll 1
  for (uint32_t r = 0; r < rows; ++r) {
    const uint4 Xc = X;
    if (r + 1 < rows) {
      const uint64_t ra = rb + 1024ull * (r + 1);
      if (ra >= lo_u && ra + 1024 <= hi_u) {
        const uint64_t q = a0 + 1024ull * (r + 1) - e;
        const uint4 l0 = gld16(q);
        const uint4 l1 = e ? gld16(q + 16) : make_uint4(0, 0, 0, 0);
        X = shift16(l0, l1, e);
      } else {
        X = load16(a0 + 1024ull * (r + 1), lo, hi, e);
      }
    }
#if MCDC_PV_NIB
    U = u4xor(nibmul(M, U), Xc);  // U <- U G + X
#else
    U = u4xor(m8mul(M, U), Xc);  // U <- U G + X
#endif
  }
  U = dotb(U, *reinterpret_cast<const uint4 *>(keys[i].w[lane]));  // lane l's last block sits 64 - l from the end
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    U.x ^= (uint32_t)__shfl_xor((int)U.x, o);
    U.y ^= (uint32_t)__shfl_xor((int)U.y, o);
    U.z ^= (uint32_t)__shfl_xor((int)U.z, o);
    U.w ^= (uint32_t)__shfl_xor((int)U.w, o);
  }
  if (lane == 0) tsum[tile] = U;
}

// Persistent waves over the tiles; a tile past a blob's POLYVAL tiles is skipped.
constexpr int kPvTab = MCDC_PV_NIB ? 512 : 256;  // uint4 per wave: 32 nibble tables of 16 (8 KiB) / 256 bytes
__global__ __launch_bounds__(256) void k_aead_polyval(const AeadRec *__restrict__ rec,
                                                      const AeadKeys *__restrict__ keys,
                                                      const uint32_t *__restrict__ owner, uint64_t ntiles,
                                                      uint4 *__restrict__ tsum, uint32_t *ctr) {
  __shared__ __attribute__((aligned(256))) uint4 mt[4][kPvTab];  // (nibmul ORs offsets into the base)
#if MCDC_PV_NIB
  MCDC_VGPR_PAD(104);  // 104 used: not an exact fill (MCDC_VGPR_PAD)
#endif
  const uint32_t wv = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t tile = (MCDC_AEAD_PERSIST & 1) ? next_tile(ctr) : blockIdx.x * 4 + wv;
  for (;;) {
    if (tile >= ntiles) break;
    const uint32_t i = rfl(owner[tile]);
    const uint32_t t = tile - (uint32_t)rec[i].tile0;
    if (t < rec[i].ptiles) polyval_tile(rec, keys, mt[wv], lane, i, t, tile, tsum);
    if (!(MCDC_AEAD_PERSIST & 1)) break;
    tile = next_tile(ctr);
  }
}

// One lane per blob: POLYVAL of the whole blob, the tag.
__global__ __launch_bounds__(256) void k_aead_tag(int open, AeadRec *rec, const AeadKeys *keys, const uint4 *tsum,
                                                  uint64_t n, int32_t *status) {
  __shared__ uint32_t tt[kTabWords];
  fill_table(tt);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t *tl = tt + (threadIdx.x % kRep);
  const AeadRec R = rec[i];
  if (!R.ok) {
    if (open) status[i] = -1;
    return;
  }
  const AeadKeys &K = keys[i];
  const uint4 h4096 = *reinterpret_cast<const uint4 *>(K.h4096), H = *reinterpret_cast<const uint4 *>(K.h);
  uint4 S = make_uint4(0, 0, 0, 0);
  for (uint32_t t = 0; t < R.ptiles; ++t) S = u4xor(t ? dotb(S, h4096) : S, tsum[R.tile0 + t]);
  const uint64_t bits = 8 * R.len;  // length block: le64(bitlen(AAD) = 0) || le64(bitlen(P))
  S = dotb(make_uint4(S.x, S.y, S.z ^ (uint32_t)bits, S.w ^ (uint32_t)(bits >> 32)), H);
  S = make_uint4(S.x ^ R.nonce[0], S.y ^ R.nonce[1], S.z ^ R.nonce[2], S.w & 0x7fffffffu);
  uint32_t rk[60];
#pragma unroll
  for (int j = 0; j < 60; j += 4) {
    const uint4 v = *reinterpret_cast<const uint4 *>(&K.rk[j]);
    rk[j] = v.x;
    rk[j + 1] = v.y;
    rk[j + 2] = v.z;
    rk[j + 3] = v.w;
  }
  const uint4 tag = aes256(tl, rk, S);
  if (!open) {
    *reinterpret_cast<uint4 *>(rec[i].tag) = tag;
  } else {
    status[i] = (tag.x == R.tag[0] && tag.y == R.tag[1] && tag.z == R.tag[2] && tag.w == R.tag[3]) ? 0 : -1;
  }
}

// Output byte at sealed offset b (seal: nonce | data | tag; open: data only).
__device__ __forceinline__ uint32_t edge_byte(const AeadRec &R, uint64_t addr, uint4 val, uint32_t k) {
  if (addr < R.dst) {
    const uint32_t j = (uint32_t)(addr - R.ext);  // 0..11
    const uint32_t w = j < 4 ? R.nonce[0] : j < 8 ? R.nonce[1] : R.nonce[2];
    return (w >> (8 * (j & 3))) & 0xffu;
  }
  if (addr < R.dst + R.len) return byte_of(val, k);
  const uint32_t j = (uint32_t)(addr - R.dst - R.len);  // 0..15
  const uint32_t w = j < 8 ? (j < 4 ? R.tag[0] : R.tag[1]) : (j < 12 ? R.tag[2] : R.tag[3]);
  return (w >> (8 * (j & 3))) & 0xffu;
}

// Write output quad at aligned address qa: bytes inside [R.ext, R.ext + T) only.
__device__ __forceinline__ void store_quad(const AeadRec &R, uint64_t T, uint64_t qa, uint4 val) {
  if (qa >= R.dst && qa + 16 <= R.dst + R.len) {
    *reinterpret_cast<uint4 *>(qa) = val;
    return;
  }
  uint32_t w[4] = {0, 0, 0, 0};
  bool all = true;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint64_t a = qa + k;
    const bool in = a >= R.ext && a < R.ext + T;
    all = all && in;
    if (in) w[k >> 2] |= edge_byte(R, a, val, k) << (8 * (k & 3));
  }
  if (all) {
    *reinterpret_cast<uint4 *>(qa) = make_uint4(w[0], w[1], w[2], w[3]);
    return;
  }
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint64_t a = qa + k;
    if (a >= R.ext && a < R.ext + T) *reinterpret_cast<uint8_t *>(a) = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  }
}

// One tile of output quads: CTR keystream, plaintext xor, nonce/tag.
__device__ __forceinline__ void ctr_tile(int open, const AeadRec *__restrict__ rec, const AeadKeys *__restrict__ keys,
                                         const uint32_t *__restrict__ owner, const uint8_t *tb, uint32_t lane,
                                         uint32_t lane4, uint32_t tile) {
  const uint32_t i = rfl(owner[tile]);
  const AeadRec &R = rec[i];
  const uint32_t t = tile - (uint32_t)R.tile0;
  const uint64_t T = open ? R.len : R.len + kAeadOverhead;
  if (T == 0) return;
  const uint64_t q_first = R.ext >> 4, q_last = (R.ext + T - 1) >> 4, nq = q_last - q_first + 1;
  if ((uint64_t)t * kAeadTileBlocks >= nq) return;
  const uint64_t left = nq - (uint64_t)t * kAeadTileBlocks;
  const uint32_t rows = (uint32_t)(left >= kAeadTileBlocks ? kAeadRows : (left + 63) / 64);
  const uint32_t *rk = keys[i].rk;
  const uint4 ctr = make_uint4(R.tag[0], R.tag[1], R.tag[2], R.tag[3] | 0x80000000u);
  const uint64_t Qb = q_first + (uint64_t)t * kAeadTileBlocks;
  // quad Q holds data bytes from c0 = 16 Q - dst; lane's block B = floor(c0 / 16) + 1,
  // the quad = bytes [d, d + 16) of KS(B - 1) || KS(B)
  const int64_t c0b = (int64_t)(16 * Qb) - (int64_t)R.dst;  // >= -27
  const int64_t B0 = (c0b + 48) / 16 - 3 + 1;
  const uint32_t d = (uint32_t)(0 - R.dst) & 15, e = (uint32_t)(R.src - R.dst) & 15;
  uint4 carry[1] = {make_uint4(ctr.x + (uint32_t)(B0 - 1), ctr.y, ctr.z, ctr.w)};
  aes256p<1>(tb, lane4, rk, carry);
  // one row: the keystream of its lanes' blocks and of the lane before (DPP
  // wave_shr; lane 0 takes the previous row's lane 63), the plaintext, the store
  auto row = [&](uint32_t r, const uint4 &ks) {
    const uint64_t Q = Qb + 64ull * r + lane;
    const uint4 kp = make_uint4((uint32_t)__builtin_amdgcn_update_dpp((int)carry[0].x, (int)ks.x, 0x138, 0xf, 0xf, false),
                                (uint32_t)__builtin_amdgcn_update_dpp((int)carry[0].y, (int)ks.y, 0x138, 0xf, 0xf, false),
                                (uint32_t)__builtin_amdgcn_update_dpp((int)carry[0].z, (int)ks.z, 0x138, 0xf, 0xf, false),
                                (uint32_t)__builtin_amdgcn_update_dpp((int)carry[0].w, (int)ks.w, 0x138, 0xf, 0xf, false));
    carry[0] = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)ks.x, 63), (uint32_t)__builtin_amdgcn_readlane((int)ks.y, 63),
                          (uint32_t)__builtin_amdgcn_readlane((int)ks.z, 63), (uint32_t)__builtin_amdgcn_readlane((int)ks.w, 63));
    const uint4 k16 = shift16(kp, ks, d);
    const uint64_t qa = 16 * Q;
    const uint4 p = load16(R.src + (qa - R.dst), R.src, R.src + R.len, e);
    if (Q <= q_last) store_quad(R, T, qa, u4xor(p, k16));
  };
#if MCDC_CTR_ILP == 2
#pragma unroll 1
  for (uint32_t r = 0; r < rows; r += 2) {  // two rows' blocks per AES call
    const uint32_t B = (uint32_t)(B0 + 64 * (int64_t)r + lane);
    uint4 ks[2] = {make_uint4(ctr.x + B, ctr.y, ctr.z, ctr.w), make_uint4(ctr.x + B + 64, ctr.y, ctr.z, ctr.w)};
    aes256p<2>(tb, lane4, rk, ks);
    row(r, ks[0]);
    if (r + 1 < rows) row(r + 1, ks[1]);
  }
#else
#pragma unroll 1
  for (uint32_t r = 0; r < rows; ++r) {
    const uint32_t B = (uint32_t)(B0 + 64 * (int64_t)r + lane);
    uint4 ks[1] = {make_uint4(ctr.x + B, ctr.y, ctr.z, ctr.w)};
    aes256p<1>(tb, lane4, rk, ks);
    row(r, ks[0]);
  }
#endif
}

// Persistent waves (kCtrWaves per block share the 64-KiB table) over the tiles.
__global__ __launch_bounds__(64 * kCtrWaves) void k_aead_ctr(int open, const AeadRec *__restrict__ rec,
                                                             const AeadKeys *__restrict__ keys,
                                                             const uint32_t *__restrict__ owner, uint64_t ntiles,
                                                             uint32_t *ctr) {
  __shared__ uint32_t tt[kTabPWords];
  fill_table_p(tt);
  const uint32_t lane = threadIdx.x & 63;
  const uint8_t *tb = reinterpret_cast<const uint8_t *>(tt);
  uint32_t tile = (MCDC_AEAD_PERSIST & 2) ? next_tile(ctr) : blockIdx.x * kCtrWaves + rfl(threadIdx.x >> 6);
  for (;;) {
    if (tile >= ntiles) break;
    ctr_tile(open, rec, keys, owner, tb, lane, MCDC_AES_2T ? 4 * (lane & 31) : 4 * lane, tile);
    if (!(MCDC_AEAD_PERSIST & 2)) break;
    tile = next_tile(ctr);
  }
}

// open: a blob that failed authentication gets zeros instead of its plaintext.
__global__ __launch_bounds__(256) void k_aead_zero(const AeadRec *__restrict__ rec, const uint32_t *__restrict__ owner,
                                                   const int32_t *__restrict__ status, uint64_t ntiles) {
  MCDC_VGPR_PAD(8);  // 8 used: not an exact fill (MCDC_VGPR_PAD)
  const uint32_t wv = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t tile = blockIdx.x * 4 + wv;
  if (tile >= ntiles) return;
  const uint32_t i = rfl(owner[tile]);
  if (status[i] == 0) return;
  const AeadRec &R = rec[i];
  const uint64_t T = R.len;
  if (T == 0) return;
  const uint32_t t = tile - (uint32_t)R.tile0;
  const uint64_t q_first = R.ext >> 4, q_last = (R.ext + T - 1) >> 4, nq = q_last - q_first + 1;
  for (uint64_t q = (uint64_t)t * kAeadTileBlocks + lane; q < nq && q < (uint64_t)(t + 1) * kAeadTileBlocks; q += 64) {
    const uint64_t qa = 16 * (q_first + q);
#pragma unroll
    for (uint32_t k = 0; k < 16; k += 1) {
      const uint64_t a = qa + k;
      if (a >= R.ext && a < R.ext + T) *reinterpret_cast<uint8_t *>(a) = 0;
    }
  }
}

// -------------------------------------------------------------- host ---
void aead_expand_key256(const uint8_t key[32], uint32_t rk[60]) {
  for (int i = 0; i < 8; ++i)
    rk[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 | (uint32_t)key[4 * i + 2] << 16 |
            (uint32_t)key[4 * i + 3] << 24;
  uint32_t rcon = 1;
  auto sub = [](uint32_t t) {
    return (uint32_t)kHostTab.sbox[t & 255] | (uint32_t)kHostTab.sbox[(t >> 8) & 255] << 8 |
           (uint32_t)kHostTab.sbox[(t >> 16) & 255] << 16 | (uint32_t)kHostTab.sbox[t >> 24] << 24;
  };
  for (int i = 8; i < 60; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 8 == 0) {
      t = sub((t >> 8) | (t << 24)) ^ rcon;
      rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11b : 0);
    } else if (i % 8 == 4) {
      t = sub(t);
    }
    rk[i] = rk[i - 8] ^ t;
  }
}

size_t aead_scan_tmp_bytes(uint64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n + 1);
  return b;
}

void launch_aead_sizes(int open, const uint64_t *ext, uint64_t n, uint64_t n_in, uint64_t *olen, uint64_t *tcnt,
                       uint64_t *ooff, uint64_t *toff, uint32_t *err, void *tmp, size_t tmp_bytes,
                       hipStream_t stream) {
  hipLaunchKernelGGL(k_aead_sizes, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, open, ext, n, n_in,
                     olen, tcnt, err);
  size_t b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, olen, ooff, (int)n + 1, stream);
  b = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, tcnt, toff, (int)n + 1, stream);
}

// Persistent grids: as many blocks as fit at once (k_aead_polyval: 32 KiB LDS,
// 4 waves -> 5 per CU; k_aead_ctr: 64 KiB LDS -> 2 per CU), never more than
// there are tiles; ctr[0], ctr[1]: the two launches' tile counters.
static void launch_tiles(int open, const AeadRec *rec, const AeadKeys *keys, const uint32_t *owner, uint64_t ntiles,
                         uint4 *tsum, uint32_t *ctr, int num_cus, bool polyval, hipStream_t stream) {
  if (!ntiles) return;
  if (polyval) {
    const uint64_t nb = (MCDC_AEAD_PERSIST & 1) ? std::min<uint64_t>((ntiles + 3) / 4, (uint64_t)num_cus * (160 / (4 * kPvTab * 16 / 1024)))
                                                : (ntiles + 3) / 4;
    hipLaunchKernelGGL(k_aead_polyval, dim3((unsigned)nb), dim3(256), 0, stream, rec, keys, owner, ntiles, tsum, ctr);
  } else {
    const uint64_t nb = (MCDC_AEAD_PERSIST & 2)
                            ? std::min<uint64_t>((ntiles + kCtrWaves - 1) / kCtrWaves, (uint64_t)num_cus * 2)
                            : (ntiles + kCtrWaves - 1) / kCtrWaves;
    hipLaunchKernelGGL(k_aead_ctr, dim3((unsigned)nb), dim3(64 * kCtrWaves), 0, stream, open, rec, keys, owner, ntiles,
                       ctr + 1);
  }
}

void launch_aead_seal(const AeadMaster &mk, const uint8_t *in, const uint64_t *ext, const uint32_t *nonces,
                      uint64_t n, uint8_t *out, const uint64_t *ooff, const uint64_t *toff, uint64_t ntiles,
                      AeadRec *rec, AeadKeys *keys, uint32_t *owner, uint4 *tsum, uint32_t *ctr, int num_cus,
                      hipStream_t stream) {
  const dim3 gb((unsigned)((n + 255) / 256));
  (void)hipMemsetAsync(ctr, 0, 8, stream);
  hipLaunchKernelGGL(k_aead_prep, gb, dim3(256), 0, stream, 0, mk, in, ext, nonces, n, out, ooff, toff, rec, keys,
                     owner);
  launch_tiles(0, rec, keys, owner, ntiles, tsum, ctr, num_cus, true, stream);
  hipLaunchKernelGGL(k_aead_tag, gb, dim3(256), 0, stream, 0, rec, keys, tsum, n, (int32_t *)nullptr);
  launch_tiles(0, rec, keys, owner, ntiles, tsum, ctr, num_cus, false, stream);
}

void launch_aead_open(const AeadMaster &mk, const uint8_t *in, const uint64_t *ext, uint64_t n, uint8_t *out,
                      const uint64_t *ooff, const uint64_t *toff, uint64_t ntiles, AeadRec *rec, AeadKeys *keys,
                      uint32_t *owner, uint4 *tsum, int32_t *status, uint32_t *ctr, int num_cus, hipStream_t stream) {
  const dim3 gb((unsigned)((n + 255) / 256));
  (void)hipMemsetAsync(ctr, 0, 8, stream);
  hipLaunchKernelGGL(k_aead_prep, gb, dim3(256), 0, stream, 1, mk, in, ext, (const uint32_t *)nullptr, n, out, ooff,
                     toff, rec, keys, owner);
  launch_tiles(1, rec, keys, owner, ntiles, tsum, ctr, num_cus, false, stream);
  launch_tiles(1, rec, keys, owner, ntiles, tsum, ctr, num_cus, true, stream);
  hipLaunchKernelGGL(k_aead_tag, gb, dim3(256), 0, stream, 1, rec, keys, tsum, n, status);
  if (ntiles) hipLaunchKernelGGL(k_aead_zero, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, stream, rec, owner,
                                 status, ntiles);
}

}  // namespace mcdc
