// chacha.hip -- ChaCha20-Poly1305 seal/open over device-resident record
// batches (gfx950).
//
// Replaces chacha20_poly1305_sealv / _openv_detached
// (crypto/cipher/e_chacha20poly1305.cc:117-333) -> CRYPTO_chacha_20
// (crypto/chacha/chacha.cc:100-224) + CRYPTO_poly1305_* (crypto/poly1305/
// poly1305.cc) / the fused chacha20_poly1305_seal_avx2 (chacha20_poly1305_
// x86_64.pl:861).  Design:
//
// * L = 2 lanes per record (kLanes below), 32 records per wave, 3 waves per
//   SIMD at ~150-170 VGPRs (4 lanes at 128 VGPRs / 4 waves spilled and ran
//   slower: the per-record serial Poly1305 work -- powers of r, lane tree,
//   final reduction -- is amortized over fewer blocks per lane).  The record's
//   ChaCha blocks u = 0..n (u = 0: the Poly1305 key block, counter 0; u >= 1:
//   data block u-1, counter u, RFC 8439) are dealt round-robin to the lanes:
//   one lane per 64-byte block, keystream XORed with the input in registers.
// * Registers: the powers of r and the block loop's multipliers live in LDS
//   (per record); record-aligned batches stage their blocks through LDS by
//   LDS-DMA (record-contiguous I/O).
// * Poly1305: the four 16-byte Poly blocks of data block d form one unit
//   U = M0 r^3 + M1 r^2 + M2 r + M3.  A lane folds its units with Horner's
//   rule in R = r^4 at stride L (multiplier R^L), one lazily reduced sum of
//   four products per unit; the L lane accumulators are rotated into exponent
//   order and tree-combined with R, R^2, R^4 -- the same lane algebra as the
//   GHASH of gcm.hip, here in GF(2^130-5) with 26-bit limbs.  A trailing
//   partial unit and the AD are folded in afterwards; the tag is
//   (((Z r) + L) r mod p + s) mod 2^128.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "iov_dev.h"

namespace bssl_amd {
namespace {

constexpr int kThreads = 256;
// Wave priority during a record group's start-up (loads, first ChaCha
// block): waves that start mid-kernel otherwise lose every issue arbitration
// to older waves and sit 60-100 K cycles before their first block (stamps,
// DESIGN.md 4.3).  Priority 2 for that phase: +2-5 % on config 3 (40-step
// runs, 1,061/1,072 -> 1,122/1,092 GiB/s).
constexpr int kStartPrio = 2;
// Lanes per record (round 3: 2 for every AEAD and layout, 32 records per
// wave, 3 waves per SIMD at ~150-170 VGPRs without spills).  Against 4 lanes
// (128 VGPRs, 4 waves, 27-43 spills), same box (profiles/r03/s13/): config 3
// at 128-byte alignment 1,192 vs 1,069-1,079 GiB/s, config3x 1,110-1,124 vs
// 999; the per-record work (key block, powers of r, lane tree, tag; for
// XChaCha one HChaCha20) is spread over twice the blocks per lane.
constexpr int kLanes = 2;
#define CHACHA_PRAGMA_(x) _Pragma(#x)
#define CHACHA_PRAGMA(x) CHACHA_PRAGMA_(x)
constexpr uint32_t kM26 = 0x3ffffff;
#ifndef CHACHA_IOV_HANDOFF
#define CHACHA_IOV_HANDOFF 1
#endif
constexpr bool kIovHandoff = CHACHA_IOV_HANDOFF != 0;

__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) {
  return __builtin_amdgcn_alignbit(v, v, 32 - n);
}

struct ChaState {
  uint32_t x[16];
};

#define QR(a, b, c, d)                 \
  a += b; d = rotl(d ^ a, 16);         \
  c += d; b = rotl(b ^ c, 12);         \
  a += b; d = rotl(d ^ a, 8);          \
  c += d; b = rotl(b ^ c, 7);

// Opaque copy of the key words: otherwise hipcc hoists the key-only first
// steps of the column round out of the block loop and keeps them live
// (registers).
__device__ __forceinline__ void launder_key(const uint32_t key[8], uint32_t k[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = key[i];
  asm volatile("" : "+v"(k[0]), "+v"(k[1]), "+v"(k[2]), "+v"(k[3]), "+v"(k[4]), "+v"(k[5]),
               "+v"(k[6]), "+v"(k[7]));
}

// The ChaCha20 block function over an already laundered key.
__device__ __forceinline__ void chacha_block_raw(const uint32_t key[8], uint32_t ctr,
                                                 const uint32_t nonce[3], uint32_t out[16]) {
  uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
  uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
  uint32_t x12 = ctr, x13 = nonce[0], x14 = nonce[1], x15 = nonce[2];
  CHACHA_PRAGMA(unroll 10)
  for (int i = 0; i < 10; i++) {
    QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15)
    QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14)
  }
  out[0] = x0 + 0x61707865;
  out[1] = x1 + 0x3320646e;
  out[2] = x2 + 0x79622d32;
  out[3] = x3 + 0x6b206574;
  out[4] = x4 + key[0];
  out[5] = x5 + key[1];
  out[6] = x6 + key[2];
  out[7] = x7 + key[3];
  out[8] = x8 + key[4];
  out[9] = x9 + key[5];
  out[10] = x10 + key[6];
  out[11] = x11 + key[7];
  out[12] = x12 + ctr;
  out[13] = x13 + nonce[0];
  out[14] = x14 + nonce[1];
  out[15] = x15 + nonce[2];
}

__device__ __forceinline__ void chacha_block(const uint32_t key[8], uint32_t ctr,
                                             const uint32_t nonce[3], uint32_t out[16]) {
  uint32_t k[8];
  launder_key(key, k);
  chacha_block_raw(k, ctr, nonce, out);
}

// HChaCha20 (CRYPTO_hchacha20, crypto/chacha/chacha.cc:43-63): the state of
// (key, 16-byte nonce) after 20 rounds, words 0-3 and 12-15 -- the
// XChaCha20-Poly1305 subkey (e_chacha20poly1305.cc:248-252).
__device__ __forceinline__ void hchacha20(uint32_t key[8], const uint32_t n[4]) {
  uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
  uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
  uint32_t x12 = n[0], x13 = n[1], x14 = n[2], x15 = n[3];
  CHACHA_PRAGMA(unroll 10)
  for (int i = 0; i < 10; i++) {
    QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15)
    QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14)
  }
  key[0] = x0; key[1] = x1; key[2] = x2; key[3] = x3;
  key[4] = x12; key[5] = x13; key[6] = x14; key[7] = x15;
}

// ---------------------------------------------------------------------------
// Poly1305 arithmetic modulo 2^130 - 5, radix 2^26.
struct P {
  uint32_t h[5];
};

__device__ __forceinline__ P pzero() { return P{{0, 0, 0, 0, 0}}; }

__device__ __forceinline__ P padd(P a, const P &b) {
#pragma unroll
  for (int i = 0; i < 5; i++) a.h[i] += b.h[i];
  return a;
}

// Block (16 bytes as 4 LE words) plus 2^128.
__device__ __forceinline__ P pblock(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3) {
  P m;
  m.h[0] = t0 & kM26;
  m.h[1] = ((t0 >> 26) | (t1 << 6)) & kM26;
  m.h[2] = ((t1 >> 20) | (t2 << 12)) & kM26;
  m.h[3] = ((t2 >> 14) | (t3 << 18)) & kM26;
  m.h[4] = (t3 >> 8) | (1u << 24);
  return m;
}

__device__ __forceinline__ uint64_t mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// a * r mod p (partially reduced; limbs < 2^26 except h1 < 2^26 + 2^7).
__device__ __forceinline__ P pmul(const P &a, const P &r) {
  const uint32_t s1 = r.h[1] * 5, s2 = r.h[2] * 5, s3 = r.h[3] * 5, s4 = r.h[4] * 5;
  uint64_t d0 = mul64(a.h[0], r.h[0]) + mul64(a.h[1], s4) + mul64(a.h[2], s3) +
                mul64(a.h[3], s2) + mul64(a.h[4], s1);
  uint64_t d1 = mul64(a.h[0], r.h[1]) + mul64(a.h[1], r.h[0]) + mul64(a.h[2], s4) +
                mul64(a.h[3], s3) + mul64(a.h[4], s2);
  uint64_t d2 = mul64(a.h[0], r.h[2]) + mul64(a.h[1], r.h[1]) + mul64(a.h[2], r.h[0]) +
                mul64(a.h[3], s4) + mul64(a.h[4], s3);
  uint64_t d3 = mul64(a.h[0], r.h[3]) + mul64(a.h[1], r.h[2]) + mul64(a.h[2], r.h[1]) +
                mul64(a.h[3], r.h[0]) + mul64(a.h[4], s4);
  uint64_t d4 = mul64(a.h[0], r.h[4]) + mul64(a.h[1], r.h[3]) + mul64(a.h[2], r.h[2]) +
                mul64(a.h[3], r.h[1]) + mul64(a.h[4], r.h[0]);
  P o;
  uint64_t c;
  o.h[0] = (uint32_t)d0 & kM26;
  c = d0 >> 26;
  d1 += c;
  o.h[1] = (uint32_t)d1 & kM26;
  c = d1 >> 26;
  d2 += c;
  o.h[2] = (uint32_t)d2 & kM26;
  c = d2 >> 26;
  d3 += c;
  o.h[3] = (uint32_t)d3 & kM26;
  c = d3 >> 26;
  d4 += c;
  o.h[4] = (uint32_t)d4 & kM26;
  c = d4 >> 26;
  uint64_t h0 = (uint64_t)o.h[0] + c * 5;
  o.h[0] = (uint32_t)h0 & kM26;
  o.h[1] += (uint32_t)(h0 >> 26);
  return o;
}

__device__ __forceinline__ P pshfl(const P &v, int src, int width) {
  P o;
#pragma unroll
  for (int i = 0; i < 5; i++) o.h[i] = __shfl(v.h[i], src, width);
  return o;
}

__device__ __forceinline__ P pshfl_down(const P &v, int d, int width) {
  P o;
#pragma unroll
  for (int i = 0; i < 5; i++) o.h[i] = __shfl_down(v.h[i], d, width);
  return o;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ uint32_t load_le32_bytes(const uint8_t *p, uint64_t avail) {
  uint32_t v = 0;
  for (int i = 0; i < 4; i++)
    if ((uint64_t)i < avail) v |= (uint32_t)p[i] << (8 * i);
  return v;
}

// Bytes [p, p + n) (n <= 16) as 4 little-endian words, zero past n, read
// with aligned dword loads: only dwords that hold at least one of the bytes
// are read (they lie in the same pages as those bytes), then funnel-shifted.
__device__ __forceinline__ void load16_partial(const uint8_t *p, uint32_t n, uint32_t w[4]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t *base = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t nd = n ? (sh + n + 3) / 4 : 0u;  // dwords touched
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = (uint32_t)k < nd ? base[k] : 0u;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t v = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    const uint32_t mask = n >= 4u * i + 4 ? 0xffffffffu
                          : n <= 4u * i   ? 0u
                                          : ((1u << (8 * (n - 4 * i))) - 1u);
    w[i] = v & mask;
  }
}

// Stores bytes [0, n) of the words y[] to p, which is 4-byte aligned: whole
// dwords, then one short and/or one byte (no byte-per-lane store loops).
__device__ __forceinline__ void store_words_partial(uint8_t *p, const uint32_t *y, uint32_t n) {
  uint32_t *pw = reinterpret_cast<uint32_t *>(p);
  const uint32_t nw = n / 4;
  for (uint32_t i = 0; i < nw; i++) pw[i] = y[i];
  const uint32_t r = n & 3;
  if (r) {
    const uint32_t last = y[nw];
    uint8_t *q = p + 4 * nw;
    if (r & 2) *reinterpret_cast<uint16_t *>(q) = (uint16_t)last;
    if (r & 1) q[r & 2] = (uint8_t)(last >> (8 * (r & 2)));
  }
}

// Final reduction and tag: (h mod p + s) mod 2^128 (poly1305.cc:255-313).
__device__ void poly_finish(P h, const uint32_t s[4], uint32_t tag[4]) {
  uint32_t c;
  c = h.h[1] >> 26; h.h[1] &= kM26; h.h[2] += c;
  c = h.h[2] >> 26; h.h[2] &= kM26; h.h[3] += c;
  c = h.h[3] >> 26; h.h[3] &= kM26; h.h[4] += c;
  c = h.h[4] >> 26; h.h[4] &= kM26; h.h[0] += c * 5;
  c = h.h[0] >> 26; h.h[0] &= kM26; h.h[1] += c;
  c = h.h[1] >> 26; h.h[1] &= kM26; h.h[2] += c;
  c = h.h[2] >> 26; h.h[2] &= kM26; h.h[3] += c;
  c = h.h[3] >> 26; h.h[3] &= kM26; h.h[4] += c;
  c = h.h[4] >> 26; h.h[4] &= kM26; h.h[0] += c * 5;
  c = h.h[0] >> 26; h.h[0] &= kM26; h.h[1] += c;
  // g = h + 5 - 2^130
  uint32_t g0 = h.h[0] + 5; c = g0 >> 26; g0 &= kM26;
  uint32_t g1 = h.h[1] + c; c = g1 >> 26; g1 &= kM26;
  uint32_t g2 = h.h[2] + c; c = g2 >> 26; g2 &= kM26;
  uint32_t g3 = h.h[3] + c; c = g3 >> 26; g3 &= kM26;
  uint32_t g4 = h.h[4] + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;  // all ones if h >= p
  h.h[0] = (h.h[0] & ~mask) | (g0 & mask);
  h.h[1] = (h.h[1] & ~mask) | (g1 & mask);
  h.h[2] = (h.h[2] & ~mask) | (g2 & mask);
  h.h[3] = (h.h[3] & ~mask) | (g3 & mask);
  h.h[4] = (h.h[4] & ~mask) | (g4 & mask);
  uint32_t w0 = h.h[0] | (h.h[1] << 26);
  uint32_t w1 = (h.h[1] >> 6) | (h.h[2] << 20);
  uint32_t w2 = (h.h[2] >> 12) | (h.h[3] << 14);
  uint32_t w3 = (h.h[3] >> 18) | (h.h[4] << 8);
  uint64_t f = (uint64_t)w0 + s[0];
  tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + s[1] + (f >> 32);
  tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + s[2] + (f >> 32);
  tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + s[3] + (f >> 32);
  tag[3] = (uint32_t)f;
}

struct RecordMeta {
  uint64_t off, len, ad_off, ad_len;
};

// Lazily reduced sum of products: d_i += a * r (no carry propagation).
struct PAcc {
  uint64_t d[5];
};

__device__ __forceinline__ PAcc pacc_zero() { return PAcc{{0, 0, 0, 0, 0}}; }

// Lazy product with the 5x multiples of r's limbs 1..4 supplied (s[i-1] =
// 5 r_i, precomputed once per record).
__device__ __forceinline__ void pmac_s(PAcc &acc, const P &a, const uint32_t *r,
                                       const uint32_t *s) {
  const uint32_t s1 = s[0], s2 = s[1], s3 = s[2], s4 = s[3];
  acc.d[0] += mul64(a.h[0], r[0]) + mul64(a.h[1], s4) + mul64(a.h[2], s3) +
              mul64(a.h[3], s2) + mul64(a.h[4], s1);
  acc.d[1] += mul64(a.h[0], r[1]) + mul64(a.h[1], r[0]) + mul64(a.h[2], s4) +
              mul64(a.h[3], s3) + mul64(a.h[4], s2);
  acc.d[2] += mul64(a.h[0], r[2]) + mul64(a.h[1], r[1]) + mul64(a.h[2], r[0]) +
              mul64(a.h[3], s4) + mul64(a.h[4], s3);
  acc.d[3] += mul64(a.h[0], r[3]) + mul64(a.h[1], r[2]) + mul64(a.h[2], r[1]) +
              mul64(a.h[3], r[0]) + mul64(a.h[4], s4);
  acc.d[4] += mul64(a.h[0], r[4]) + mul64(a.h[1], r[3]) + mul64(a.h[2], r[2]) +
              mul64(a.h[3], r[1]) + mul64(a.h[4], r[0]);
}


// Carry-propagate a lazy sum (at most 4 products of limbs < 2^27.1 and
// powers < 2^26.01: every d_i < 2^60).
__device__ __forceinline__ P preduce(PAcc a) {
  P o;
  uint64_t c;
  o.h[0] = (uint32_t)a.d[0] & kM26;
  c = a.d[0] >> 26;
  a.d[1] += c;
  o.h[1] = (uint32_t)a.d[1] & kM26;
  c = a.d[1] >> 26;
  a.d[2] += c;
  o.h[2] = (uint32_t)a.d[2] & kM26;
  c = a.d[2] >> 26;
  a.d[3] += c;
  o.h[3] = (uint32_t)a.d[3] & kM26;
  c = a.d[3] >> 26;
  a.d[4] += c;
  o.h[4] = (uint32_t)a.d[4] & kM26;
  c = a.d[4] >> 26;
  const uint64_t h0 = (uint64_t)o.h[0] + c * 5;
  o.h[0] = (uint32_t)h0 & kM26;
  o.h[1] += (uint32_t)(h0 >> 26);
  return o;
}

// A data block that reaches into the record's extra bytes (BatchDesc::extra;
// at most one per record): byte k < len from/to the record, k >= len from/to
// the extra arrays (XT kernels only).
__device__ __forceinline__ void crypt_block_x(const uint8_t *src, uint8_t *dst, uint64_t len,
                                           const uint8_t *xin, uint8_t *xout, uint64_t p0,
                                           uint32_t n, const uint32_t *ks, uint32_t *x,
                                           uint32_t *y) {
  for (int i = 0; i < 16; i++) {
    uint32_t w = 0;
    for (uint32_t t = 0; t < 4; t++) {
      const uint64_t k = p0 + 4 * i + t;
      if (4u * i + t < n) w |= (uint32_t)(k < len ? src[k] : xin[k - len]) << (8 * t);
    }
    x[i] = w;
    const uint32_t mask = n >= 4u * i + 4 ? 0xffffffffu
                          : n <= 4u * i   ? 0u
                                          : ((1u << (8 * (n - 4 * i))) - 1u);
    y[i] = (w ^ ks[i]) & mask;
  }
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t k = p0 + i;
    const uint8_t cb = (uint8_t)(y[i >> 2] >> (8 * (i & 3)));
    if (k < len)
      dst[k] = cb;
    else
      xout[k - len] = cb;
  }
}

// ChaCha20-Poly1305 over L lanes per record (64/L records per wave).
// ChaCha blocks u = 0..nblk of a record are dealt round-robin to the lanes
// (u = it*L + q): u = 0 is the Poly1305 key block (counter 0), u >= 1 the data
// block u-1 (counter u).  Poly1305 runs on the virtual sequence
// [Y_A, U_0, U_1, ...] of 4-block units, element v = u in lane u mod L, with
// Horner's rule in R = r^4 at stride L (multiplier R^L), then the rotation +
// log2(L)-level tree of gcm.hip's lane algebra.
// iovec records: the lane's whole block comes by LDS-DMA into the wave's
// staging area (loading it into VGPRs across the rounds measured the same).
// Occupancy: 3 waves per SIMD at 2 lanes per record.  (Round 4, same box,
// config 3, profiles/r04/s10/: 4 waves per SIMD (spills) 1,216 GiB/s, the
// block loop's multipliers read from LDS per product instead of in one batch
// 1,193, both 1,183, against 1,246.)
#define CHACHA_OCC __attribute__((amdgpu_waves_per_eu(L == 2 ? 3 : 4)))
// Record-contiguous I/O (COAL): a wave's loads and stores move whole
// per-record runs (L = 2: 8 records x 128 bytes per instruction), staged
// through LDS to the lane that owns each 64-byte block.  With the
// lane-per-block pattern each 16-byte access sits at a 64-byte lane stride:
// the same copy costs 1.32x the time and 1.3x the counted HBM bytes
// (tools/micro/calib_copy.hip).  Ciphertext stores carry the non-temporal
// hint (+2.3 % on config 3, same-box A/B).
// Per-record metadata without branches: a missing array (null pointer, the
// uniform-layout fields apply) is read at kMetaZero instead, so every load is
// issued unconditionally and they are all in flight together.  (Under the
// null-pointer branches hipcc waited for each load before issuing the next:
// ~8 serialized memory round trips per wave before its first block.)
__device__ const uint64_t kMetaZero[2] = {0, 0};

template <typename T>
__device__ __forceinline__ T meta_load(const T *arr, uint64_t i, bool active) {
  const T *p = arr && active ? arr + i : reinterpret_cast<const T *>(kMetaZero);
  return *p;
}

// One wave group: records pos = grp * (64 / L) + lane / L.
// IOV: iovec records walked in place (BatchDesc::iovecs; no extra bytes).
// COAL: the record-contiguous I/O (launch_chacha picks it for batches whose
// records all start 128-byte lines).  ANY: per-lane block I/O at any record
// alignment (uniform batches that are not 16-byte aligned; no extra bytes).
template <bool OPEN, int L, bool XT, bool XC, bool IOV, bool COAL, bool ANY>
__device__ __forceinline__ void chacha_group(const ChaChaKeyDev *__restrict__ keys,
                                             const BatchDesc &b, uint64_t grp) {
  __builtin_amdgcn_s_setprio(kStartPrio);
  static_assert(L == 2 || L == 4 || L == 8 || L == 16, "lanes per record");
  static_assert(!(IOV && XT), "iovec records carry no extra bytes");
  constexpr int kLog = L == 2 ? 1 : L == 4 ? 2 : L == 8 ? 3 : 4;
  const int lane = threadIdx.x & 63;
  const int q = lane & (L - 1);
  const uint64_t pos = grp * (64 / L) + lane / L;
  const bool active = pos < b.num_records;
  uint8_t vld = 1;
  const uint64_t rec = active && b.order ? (uint64_t)b.order[pos] : pos;  // sched.hip order
  RecordMeta m = {0, 0, 0, 0};
  uint32_t kidx = 0;
  if (!(b.offsets || b.lengths || b.ad_offsets || b.ad_lengths || b.key_index || b.valid)) {
    // Uniform layout, one key: no per-record loads.
    if (active) {
      m.off = rec * b.record_stride;
      m.len = b.record_len;
      m.ad_off = rec * b.ad_stride;
      m.ad_len = b.ad_len;
    }
  } else {
    const uint64_t off = meta_load(b.offsets, rec, active), len = meta_load(b.lengths, rec, active);
    const uint64_t ado = meta_load(b.ad_offsets, rec, active);
    const uint64_t adl = meta_load(b.ad_lengths, rec, active);
    const uint32_t ki = meta_load(b.key_index, rec, active);
    vld = meta_load(b.valid, rec, active);
    if (active) {
      m.off = b.offsets ? off : rec * b.record_stride;
      m.len = b.lengths ? len : b.record_len;
      m.ad_off = b.ad_offsets ? ado : rec * b.ad_stride;
      m.ad_len = b.ad_lengths ? adl : b.ad_len;
      kidx = b.key_index ? ki : 0u;
    }
  }
  // e_chacha20poly1305.cc:127-142: 12-byte nonce, < 2^32 - 1 blocks
  // (XChaCha20-Poly1305: 24-byte nonce, :241-244).
  constexpr uint32_t kNonceLen = XC ? 24 : 12;
  const bool bad = active && (kidx >= b.num_keys || b.nonce_len != kNonceLen ||
                              m.len + b.extra_len >= (uint64_t(1) << 32) * 64 - 64 ||
                              (b.valid && !vld));
  const bool live = active && !bad;
  uint32_t key[8], nonce[3];
  {
    const ChaChaKeyDev *kp = keys + (live ? kidx : 0u);
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = kp->k[i];
    // (Addressed as soon as the record index is known, not after the
    // validity checks: any in-range record's nonce is readable.)
    const bool nok = active && b.nonce_len == kNonceLen;
    const uint8_t *np = b.nonces + (nok ? rec * kNonceLen : 0);
    constexpr int kWords = kNonceLen / 4;
    uint32_t nw[kWords];
#pragma unroll
    for (int i = 0; i < kWords; i++)
      nw[i] = nok && (reinterpret_cast<uintptr_t>(np) & 3) == 0
                  ? reinterpret_cast<const uint32_t *>(np)[i]
                  : load_le32_bytes(np + 4 * i, nok ? 4 : 0);
    if constexpr (XC) {
      // key' = HChaCha20(key, nonce[0:16]), nonce' = 0^4 || nonce[16:24]
      // (e_chacha20poly1305.cc:248-252).
      hchacha20(key, nw);
      nonce[0] = 0;
      nonce[1] = nw[4];
      nonce[2] = nw[5];
    } else {
#pragma unroll
      for (int i = 0; i < 3; i++) nonce[i] = nw[i];
    }
  }
  // The lane's first AD block (block q), loaded now so its latency hides
  // under the first ChaCha block instead of stalling the Poly1305 setup.
  uint32_t adw[4] = {0, 0, 0, 0};
  // AD block k of an iovec record: bytes of its CRYPTO_IVEC chunks.
  auto ivec_block = [&](uint64_t k, uint32_t w[4]) {
    const uint4 v = ivec_load16(b.aadvecs, b.aadvec_start[rec], b.aadvec_start[rec + 1], 16 * k,
                                (uint32_t)umin64(m.ad_len - 16 * k, 16));
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  };
  {
    const uint8_t *ad = b.ad + (live ? m.ad_off : 0);
    const uint64_t k = (uint64_t)q;
    if (live && 16 * k < m.ad_len) {
      if constexpr (IOV)
        ivec_block(k, adw);
      else
        load16_partial(ad + 16 * k, (uint32_t)umin64(m.ad_len - 16 * k, 16), adw);
    }
  }
  // Message = the record's `in` bytes then b.extra_len extra bytes
  // (BatchDesc::extra, the TLS 1.3 inner type), whose ciphertext goes to
  // their own output.
  const uint32_t xlen = XT ? b.extra_len : 0;
  const uint64_t vlen = m.len + xlen;
  const uint8_t *xin = xlen ? batch_extra_in(b, rec) : nullptr;
  uint8_t *xout = xlen ? batch_extra_out(b, rec) : nullptr;
  const uint64_t nblk = live ? (vlen + 63) / 64 : 0;  // ChaCha data blocks
  const uint64_t npoly = live ? (vlen + 15) / 16 : 0;
  const uint64_t nunits = npoly / 4;                   // full 4-block units
  const uint32_t tail_blocks = (uint32_t)(npoly & 3);
  const uint8_t *src = b.in + m.off;
  uint8_t *dst = b.out + m.off;
  const bool aligned = !IOV && ((reinterpret_cast<uintptr_t>(src) |
                                 reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  // Slot u of the record (lane u mod L, iteration u / L) holds the Poly1305
  // key block for u = 0 and data block d = u - 1 - sh for u >= 1 + sh (ChaCha
  // counter d + 1).  sh = 1 leaves slot 1 idle so that, for a record on a
  // 128-byte boundary, each iteration's 256-byte run (data blocks
  // 4 it - 1 - sh ..) covers whole 128-byte lines instead of half lines at
  // both ends (the other half written one iteration later); the Poly1305
  // element order then starts with a zero element (Y_A at v = sh).
  constexpr bool kCoalL = COAL && (L == 4 || L == 2);
  constexpr bool kCoalSh = kCoalL && !IOV;
  // (Wave-uniform: 1 only if every live record of the wave is 128-byte
  // aligned, so the slot arithmetic stays scalar.)
  const uint64_t live_mask = __ballot(live);
  const uint32_t sh =
      kCoalSh && live_mask &&
              __ballot(live && ((reinterpret_cast<uintptr_t>(dst) & 127) == 0)) == live_mask
          ? 1u : 0u;
  // LDS: one 64-byte block per thread (the first ciphertext block while the
  // powers of r are built, then the staging area of the coalesced record
  // I/O: record slot r of the wave at r * 256, block q at + 64 q, its 16-byte
  // chunk j at + 16 ((j + q + r) mod 4) -- conflict-free both for the 16
  // chunks of a record and for the 4 chunks a lane reads of its own block).
  __shared__ uint4 s_c0[kThreads][4];
  constexpr bool kCoal = kCoalL && !IOV;
  // Per record slot: byte offset and the number of full 64-byte blocks the
  // coalesced path moves (0 unless the record is live and 16-byte aligned).
  __shared__ uint4 s_rinfo[kThreads / L];
  const int wbase = threadIdx.x & ~63;
  uint8_t *const stage = reinterpret_cast<uint8_t *>(&s_c0[wbase][0]);
  if (kCoal && q == 0) {
    const uint32_t nfull = live && aligned ? (uint32_t)(m.len / 64) : 0u;
    s_rinfo[threadIdx.x / L] = make_uint4((uint32_t)m.off, (uint32_t)(m.off >> 32), nfull, sh);
  }
  // Staging: the 64-byte block of wave lane t (record slot t / L, block
  // t mod L of the iteration's run) at t * 64, its 16-byte chunk j at
  // + 16 ((j + t + t / 4) mod 4): the 16 lanes of a ds_read_b128 lane group
  // read 16 distinct bank quads, for L = 4 and L = 2 alike.
  auto saddr = [](int t, int j) { return t * 64 + ((j + (t & 3) + (t >> 2)) & 3) * 16; };

  // Encrypt (or decrypt) the data block of ChaCha block u held in ks; returns
  // the ciphertext words (masked past the end) in c[].
  // Input of data block d = u-1 when it is a full aligned 64-byte block
  // (issued before the ChaCha rounds so the HBM latency hides under them).
  // iovec records (IOV): each lane walks the chunks with a cursor for its
  // loads and one for its stores (chunk index and the chunk's stream start,
  // as gcm.hip).  Between chunk boundaries only a running pointer moves: the
  // lane's next block is 64 L bytes further on, and while it lies inside the
  // chunk (`*_left` >= 64) it is four dwordx4 at any alignment.  A block
  // across chunks or the record's last block goes through 16-byte pieces
  // (iov_load2 / iov_store2, the byte walk over three or more chunks).
  uint64_t ld_c = 0, ld_cs = 0, st_c = 0, st_cs = 0;
  const uint8_t *ld_ptr = nullptr;
  uint8_t *st_ptr = nullptr;
  int64_t ld_left = -1, st_left = -1;
  // Store anchor handed over by the load cursor (as gcm.hip's kIovHandoff):
  // when prefetch walks the chunk table to a whole block inside one chunk, the
  // block's output address and the bytes left in its chunk, tagged with the
  // data block index; the block's store re-anchors its run from it without a
  // walk of its own (whose loads would wait for every older load and store).
  uint8_t *ho_ptr = nullptr;
  int64_t ho_left = -1;
  uint32_t ho_d = 0xffffffffu;
  bool pre_ok = false;  // pre[] holds the lane's whole current block
  if constexpr (IOV) {
    if (live) ld_c = st_c = b.iovec_start[rec];
  }
  auto prefetch = [&](uint64_t u, uint4 pre[4]) {
    const uint64_t d = u - 1 - sh;
    if constexpr (IOV) {
      // The lane's whole 64-byte block, when it lies in one chunk, goes to
      // the wave's staging area by LDS-DMA (four 16-byte pieces at any
      // alignment, piece i of lane l at + 1024 i + 16 l: no VGPRs held across
      // the rounds); anything else takes crypt_block's piece path.
      pre_ok = false;
      if (u >= 1 && d < nblk && m.len >= 64 * d + 64) {
        const uint8_t *gp = nullptr;
        if (ld_left >= 64) {
          gp = ld_ptr;
          ld_ptr += 64 * L;
          ld_left -= 64 * L;
        } else {
          const uint64_t p = 64 * d;
          IovCur k;
          iov_at(k, b, ld_c, ld_cs);
          iov_seek(k, b, p, b.iovec_start[rec + 1]);
          ld_c = k.c;
          ld_cs = k.cs;
          if (p + 64 <= k.ce) {
            gp = k.in + (p - k.cs);
            ld_ptr = gp + 64 * L;
            ld_left = (int64_t)(k.ce - p) - 64 * L;
            if constexpr (kIovHandoff) {
              ho_ptr = k.out + (p - k.cs);
              ho_left = (int64_t)(k.ce - p);
              ho_d = (uint32_t)d;
            }
          } else {
            ld_left = -1;
          }
        }
        if (gp) {
#pragma unroll
          for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void *>(gp + 16 * i),
                reinterpret_cast<__attribute__((address_space(3))) void *>(
                    reinterpret_cast<uintptr_t>(stage + 1024 * i)),
                16, 0, 0);
          pre_ok = true;
        }
      }
      return;
    }
    if constexpr (ANY) {
      // (Any alignment: one dwordx4 per 16 bytes, iov_dev.h load16_any.)
      if (u >= 1 + sh && d < nblk && m.len >= 64 * d + 64) {
#pragma unroll
        for (int i = 0; i < 4; i++) pre[i] = load16_any(src + 64 * d + 16 * i);
      }
      return;
    }
    if (u >= 1 + sh && d < nblk && aligned && m.len >= 64 * d + 64) {
      const uint4 *sp = reinterpret_cast<const uint4 *>(src + 64 * d);
#pragma unroll
      for (int i = 0; i < 4; i++) pre[i] = sp[i];
    }
  };
  auto crypt_block = [&](uint64_t u, const uint32_t ks[16], const uint4 pre[4], uint32_t c[16],
                         bool staged) {
    const uint64_t d = u - 1 - sh;
    const uint64_t rem = vlen - 64 * d;
    uint32_t x[16], y[16];
    if constexpr (IOV) {
      const uint64_t p = 64 * d;
      const uint32_t n = (uint32_t)umin64(rem, 64);
      const uint64_t c_end = b.iovec_start[rec + 1];
      uint8_t *my = stage + 16 * lane;  // piece i at + 1024 i
      if (pre_ok) {
        // Whole block from the LDS-DMA staging (the caller waited for it).
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint4 v = *reinterpret_cast<const uint4 *>(my + 1024 * i);
          x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) y[i] = x[i] ^ ks[i];
        if (st_left >= 64) {
#pragma unroll
          for (int i = 0; i < 4; i++)
            store16_any(st_ptr + 16 * i,
                        make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]));
          st_ptr += 64 * L;
          st_left -= 64 * L;
        } else if (kIovHandoff && ho_d == (uint32_t)d) {
#pragma unroll
          for (int i = 0; i < 4; i++)
            store16_any(ho_ptr + 16 * i,
                        make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]));
          st_ptr = ho_ptr + 64 * L;
          st_left = ho_left - 64 * L;
        } else {
          IovCur k;
          iov_at(k, b, st_c, st_cs);
          iov_seek(k, b, p, c_end);
          st_c = k.c;
          st_cs = k.cs;
          // (The output chunks have the input chunks' lengths, so a block
          // the loads found in one chunk lies in one output chunk too.)
          if (p + 64 <= k.ce) {
#pragma unroll
            for (int i = 0; i < 4; i++)
              store16_any(k.out + (p - k.cs) + 16 * i,
                          make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]));
            st_ptr = k.out + (p - k.cs) + 64 * L;
            st_left = (int64_t)(k.ce - p) - 64 * L;
          } else {  // (not reached: see above)
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const uint64_t pi = p + 16 * i;
              iov_seek(k, b, pi, c_end);
              const uint4 v = make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]);
              if (!iov_store2(b, k, pi, v, 16, c_end)) iov_scatter(b, k, pi, v, 16, c_end);
            }
            st_c = k.c;
            st_cs = k.cs;
            st_left = -1;
          }
        }
      } else if (n < 64 && ld_left >= (int64_t)n && st_left >= (int64_t)n) {
        // The record's last, partial block inside the chunks of the lane's
        // previous block (the running pointers): partial loads and stores at
        // any alignment, no cursor walk.
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t ni = n > 16u * i ? min(n - 16u * i, 16u) : 0u;
          uint4 v = make_uint4(0, 0, 0, 0);
          if (ni == 16)
            v = load16_any(ld_ptr + 16 * i);
          else if (ni)
            v = load_partial(ld_ptr + 16 * i, ni);
          const uint4 w = mask_block(make_uint4(v.x ^ ks[4 * i], v.y ^ ks[4 * i + 1],
                                                v.z ^ ks[4 * i + 2], v.w ^ ks[4 * i + 3]),
                                     ni);
          if (ni == 16)
            store16_any(st_ptr + 16 * i, w);
          else if (ni)
            store_partial(st_ptr + 16 * i, w, ni);
          x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
          y[4 * i] = w.x; y[4 * i + 1] = w.y; y[4 * i + 2] = w.z; y[4 * i + 3] = w.w;
        }
      } else if (IovCur k = iov_cur_at(b, ld_c, ld_cs, p, c_end);
                 p + n <= k.ce + iov_len_at(b, k.c + 1, c_end)) {
        // A block in this chunk and the next (the usual straddle, or a
        // partial block the running pointers do not cover): each 16-byte
        // piece is at most two partial accesses, one per chunk, and all of
        // them are issued together (the output chunks have the input chunks'
        // lengths).
        const IovecDev nx = k.c + 1 < c_end ? b.iovecs[k.c + 1] : IovecDev{nullptr, nullptr, 0};
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t ni = n > 16u * i ? min(n - 16u * i, 16u) : 0u;
          const uint64_t pi = p + 16 * i;
          const uint32_t n1 = pi < k.ce ? (uint32_t)umin64(ni, k.ce - pi) : 0u;
          const uint32_t n2 = ni - n1;
          const uint8_t *sa = k.in + (pi - k.cs);
          const uint8_t *sb = n2 ? nx.in + (pi + n1 - k.ce) : nx.in;
          const uint4 v1 = n1 == 16 ? load16_any(sa) : load_partial(sa, n1);
          const uint4 v2 = n2 == 16 ? load16_any(sb) : load_partial(sb, n2);
          const uint4 s2 = bytes_at(make_uint4(0, 0, 0, 0), v2, 16 - n1);  // v2 << 8 n1
          const uint4 v = make_uint4(v1.x | s2.x, v1.y | s2.y, v1.z | s2.z, v1.w | s2.w);
          const uint4 w = mask_block(make_uint4(v.x ^ ks[4 * i], v.y ^ ks[4 * i + 1],
                                                v.z ^ ks[4 * i + 2], v.w ^ ks[4 * i + 3]),
                                     ni);
          uint8_t *da = k.out + (pi - k.cs);
          if (n1 == 16)
            store16_any(da, w);
          else if (n1)
            store_partial(da, w, n1);
          if (n2)
            store_partial(nx.out + (pi + n1 - k.ce), bytes_at(w, make_uint4(0, 0, 0, 0), n1), n2);
          x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
          y[4 * i] = w.x; y[4 * i + 1] = w.y; y[4 * i + 2] = w.z; y[4 * i + 3] = w.w;
        }
        const bool next = p + n > k.ce;  // the block ended in the next chunk
        ld_c = st_c = next ? k.c + 1 : k.c;
        ld_cs = st_cs = next ? k.ce : k.cs;
        ld_left = st_left = -1;
      } else {
        // A block over three or more chunks: 16-byte pieces;
        // the keystream waits in the staging slot and each piece's
        // ciphertext (seal: output, open: input) replaces it there.
#pragma unroll
        for (int i = 0; i < 4; i++)
          *reinterpret_cast<uint4 *>(my + 1024 * i) =
              make_uint4(ks[4 * i], ks[4 * i + 1], ks[4 * i + 2], ks[4 * i + 3]);
        // (k: the input cursor, at the chunk holding p)
        IovCur ko;
        iov_at(ko, b, st_c, st_cs);
#pragma unroll 1
        for (int i = 0; i < 4; i++) {
          const uint32_t ni = n > 16u * i ? min(n - 16u * i, 16u) : 0u;
          uint4 v = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0);
          if (ni) {
            const uint64_t pi = p + 16 * i;
            iov_seek(k, b, pi, c_end);
            if (ni == 16 && pi + 16 <= k.ce)
              v = load16_any(k.in + (pi - k.cs));
            else if (!iov_load2(b, k, pi, ni, c_end, v))
              v = iov_gather(b, k, pi, ni, c_end);
            const uint4 kw = *reinterpret_cast<const uint4 *>(my + 1024 * i);
            w = mask_block(make_uint4(v.x ^ kw.x, v.y ^ kw.y, v.z ^ kw.z, v.w ^ kw.w), ni);
            iov_seek(ko, b, pi, c_end);
            if (ni == 16 && pi + 16 <= ko.ce)
              store16_any(ko.out + (pi - ko.cs), w);
            else if (!iov_store2(b, ko, pi, w, ni, c_end))
              iov_scatter(b, ko, pi, w, ni, c_end);
          }
          *reinterpret_cast<uint4 *>(my + 1024 * i) = OPEN ? v : w;
        }
        ld_c = k.c;
        ld_cs = k.cs;
        ld_left = -1;
        st_c = ko.c;
        st_cs = ko.cs;
        st_left = -1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint4 v = *reinterpret_cast<const uint4 *>(my + 1024 * i);
          x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
          y[4 * i] = v.x; y[4 * i + 1] = v.y; y[4 * i + 2] = v.z; y[4 * i + 3] = v.w;
        }
      }
    } else if (kCoal && staged && m.len >= 64 * d + 64 && aligned) {
      // Full block, coalesced I/O: input from the staging area, output back
      // to it (stored after the iteration by record-contiguous stores).
      uint8_t *my = stage + lane * 64;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint4 v = *reinterpret_cast<const uint4 *>(my + ((i + (lane & 3) + (lane >> 2)) & 3) * 16);
        x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int i = 0; i < 16; i++) y[i] = x[i] ^ ks[i];
#pragma unroll
      for (int i = 0; i < 4; i++)
        *reinterpret_cast<uint4 *>(my + ((i + (lane & 3) + (lane >> 2)) & 3) * 16) =
            make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]);
    } else if constexpr (ANY) {
      static_assert(!XT && !COAL && !IOV, "ANY kernels: plain per-lane records");
      uint8_t *dp = dst + 64 * d;
      const uint32_t n = (uint32_t)umin64(rem, 64);
      if (n == 64) {
        // A full block at any alignment (one dwordx4 per 16 bytes).
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint4 v = pre[i];
          x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) y[i] = x[i] ^ ks[i];
#pragma unroll
        for (int i = 0; i < 4; i++)
          store16_any(dp + 16 * i, make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]));
      } else {
        // The last, partial block: dword loads funnel-shifted to any
        // alignment; 16-byte, dword or byte stores by the destination's
        // alignment (store_partial).
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
          load16_partial(src + 64 * d + 16 * k, nk, x + 4 * k);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
          const uint32_t mask = n >= 4u * i + 4 ? 0xffffffffu
                                : n <= 4u * i   ? 0u
                                                : ((1u << (8 * (n - 4 * i))) - 1u);
          y[i] = (x[i] ^ ks[i]) & mask;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
          if (nk)
            store_partial(dp + 16 * k,
                          make_uint4(y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]), nk);
        }
      }
    } else if (m.len >= 64 * d + 64 && aligned) {
      uint4 *dp = reinterpret_cast<uint4 *>(dst + 64 * d);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint4 v = pre[i];
        x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int i = 0; i < 16; i++) y[i] = x[i] ^ ks[i];
#pragma unroll
      for (int i = 0; i < 4; i++)
        dp[i] = make_uint4(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]);
    } else if (!XT && aligned) {
      // The record's last, partial block: aligned dword loads (only dwords
      // holding record bytes), dword / short / byte stores.
      const uint8_t *sp = src + 64 * d;
      uint8_t *dp = dst + 64 * d;
      const uint32_t n = (uint32_t)umin64(rem, 64);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
        load16_partial(sp + 16 * k, nk, x + 4 * k);
      }
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint32_t mask = n >= 4u * i + 4 ? 0xffffffffu
                              : n <= 4u * i   ? 0u
                                              : ((1u << (8 * (n - 4 * i))) - 1u);
        y[i] = (x[i] ^ ks[i]) & mask;
      }
      store_words_partial(dp, y, n);
    } else if (!XT) {
      const uint8_t *sp = src + 64 * d;
      uint8_t *dp = dst + 64 * d;
      const uint32_t n = (uint32_t)umin64(rem, 64);
#pragma unroll
      for (int i = 0; i < 16; i++) {
        x[i] = load_le32_bytes(sp + 4 * i, n > 4u * i ? n - 4u * i : 0);
        const uint32_t mask = n >= 4u * i + 4 ? 0xffffffffu
                              : n <= 4u * i   ? 0u
                                              : ((1u << (8 * (n - 4 * i))) - 1u);
        y[i] = (x[i] ^ ks[i]) & mask;
      }
      for (uint32_t i = 0; i < n; i++) dp[i] = (uint8_t)(y[i >> 2] >> (8 * (i & 3)));
    } else {
      crypt_block_x(src, dst, m.len, xin, xout, 64 * d, (uint32_t)umin64(rem, 64), ks, x,
                    y);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) c[i] = OPEN ? x[i] : y[i];
  };

  // Iteration 0: lane 0 computes the Poly1305 key block (counter 0,
  // e_chacha20poly1305.cc:89-93), lanes 1+sh..L-1 the data blocks 0..L-2-sh.
  const int iters = wave_max((int)((nblk + 1 + sh + L - 1) / L));
  uint32_t ks[16], c0[16];
  uint4 pre[4];
  prefetch((uint64_t)q, pre);
  chacha_block(key, (uint32_t)q >= 1 + sh ? (uint32_t)q - sh : 0u, nonce, ks);
  const bool have0 = (uint32_t)q >= 1 + sh && (uint64_t)q - sh <= nblk;
  if constexpr (IOV) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (LDS-DMA, prefetch)
  if (have0) crypt_block((uint64_t)q, ks, pre, c0, false);
  __builtin_amdgcn_s_setprio(0);
  uint32_t kw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) kw[i] = __shfl(ks[i], 0, L);
  // The first block's ciphertext waits in LDS while the powers of r are
  // built (the register peak of the kernel otherwise).
  if (have0) {
#pragma unroll
    for (int i = 0; i < 4; i++)
      s_c0[threadIdx.x][i] = make_uint4(c0[4 * i], c0[4 * i + 1], c0[4 * i + 2], c0[4 * i + 3]);
  }
  P pw[kLog + 4];  // pw[k] = r^(2^k), k = 0 .. kLog + 2  (r^(4L))
  uint32_t s[4];
  {
    const uint32_t t0 = kw[0] & 0x0fffffff, t1 = kw[1] & 0x0ffffffc, t2 = kw[2] & 0x0ffffffc,
                   t3 = kw[3] & 0x0ffffffc;  // clamp (RFC 8439 2.5)
    pw[0].h[0] = t0 & kM26;
    pw[0].h[1] = ((t0 >> 26) | (t1 << 6)) & kM26;
    pw[0].h[2] = ((t1 >> 20) | (t2 << 12)) & kM26;
    pw[0].h[3] = ((t2 >> 14) | (t3 << 18)) & kM26;
    pw[0].h[4] = t3 >> 8;
    s[0] = kw[4];
    s[1] = kw[5];
    s[2] = kw[6];
    s[3] = kw[7];
#pragma unroll
    for (int k = 1; k <= kLog + 2; k++) pw[k] = pmul(pw[k - 1], pw[k - 1]);
  }
  // The record's powers of r go to LDS (slot per record, written by its lane
  // 0, read back by all L lanes as broadcasts): kept in registers across the
  // ChaCha rounds they cost ~35 VGPRs and thereby a wave per SIMD.
  // s_apow: the block loop's four multipliers R^L, r^3, r^2, r with their 5x
  // multiples, 16-byte aligned (one batch of ds_read_b128 per absorb);
  // s_pow: r^(2^k) for k = 2 .. kLog + 1 (the AD and lane trees), 5 limbs
  // each -- r and r^2 are read from s_apow.
  __shared__ uint32_t s_pow[kThreads / L][5 * kLog];
  __shared__ uint4 s_apow[kThreads / L][9];
  uint32_t *const mypow = s_pow[threadIdx.x / L];
  const uint32_t *const apw = reinterpret_cast<const uint32_t *>(s_apow[threadIdx.x / L]);
  if (q == 0) {
    const P r3v = pmul(pw[1], pw[0]);
#pragma unroll
    for (int k = 2; k <= kLog + 1; k++)
#pragma unroll
      for (int i = 0; i < 5; i++) mypow[5 * (k - 2) + i] = pw[k].h[i];
    const P *am[4] = {&pw[kLog + 2], &r3v, &pw[1], &pw[0]};
    uint32_t *ap = reinterpret_cast<uint32_t *>(s_apow[threadIdx.x / L]);
#pragma unroll
    for (int m = 0; m < 4; m++) {
#pragma unroll
      for (int i = 0; i < 5; i++) ap[9 * m + i] = am[m]->h[i];
#pragma unroll
      for (int i = 1; i < 5; i++) ap[9 * m + 4 + i] = am[m]->h[i] * 5;
    }
  }
  __builtin_amdgcn_wave_barrier();
  // r^(2^k), k = 0 .. kLog + 1, re-read at each use (the offset is laundered
  // so the loads are not hoisted out of the loops).
  auto pwr = [&](int k) {
    const uint32_t *base = k < 2 ? apw : mypow;
    uint32_t off = k == 0 ? 27u : k == 1 ? 18u : 5u * (k - 2);
    asm volatile("" : "+v"(off));
    P o;
#pragma unroll
    for (int i = 0; i < 5; i++) o.h[i] = base[off + i];
    return o;
  };

  // AD: exclusive Horner in r over the zero-padded 16-byte blocks, stride L.
  P ya = pzero();
  {
    const uint8_t *ad = b.ad + (live ? m.ad_off : 0);
    const uint64_t nab = live ? (m.ad_len + 15) / 16 : 0;
    const int wmax = wave_max((int)umin64(nab, 0x7fffffff));
    auto ad_block = [&](uint64_t k) {
      if constexpr (IOV) {
        uint32_t w[4];
        ivec_block(k, w);
        return pblock(w[0], w[1], w[2], w[3]);
      }
      const uint8_t *p = ad + 16 * k;
      const uint64_t avail = m.ad_len - 16 * k;
      return pblock(load_le32_bytes(p, avail), load_le32_bytes(p + 4, avail > 4 ? avail - 4 : 0),
                    load_le32_bytes(p + 8, avail > 8 ? avail - 8 : 0),
                    load_le32_bytes(p + 12, avail > 12 ? avail - 12 : 0));
    };
    if (wmax <= 1) {
      if (nab == 1) ya = pblock(adw[0], adw[1], adw[2], adw[3]);  // block 0 (lane 0's)
      if (kCoalSh) ya = pshfl(ya, 0, L);  // lane sh takes Y_A
    } else {
      P acc = pzero();
      for (uint64_t k = q; k < nab; k += L)
        acc = padd(pmul(acc, pwr(kLog)),
                   k == (uint64_t)q ? pblock(adw[0], adw[1], adw[2], adw[3]) : ad_block(k));
      P a = pshfl(acc, (q + (int)(nab % L)) & (L - 1), L);
#pragma unroll
      for (int t = 0; t < kLog; t++) {
        const int sh = 1 << t;
        const P mm = pmul(a, pwr(t));
        const P o = pshfl_down(a, sh, L);
        if ((q & (2 * sh - 1)) == 0) a = padd(mm, o);
      }
      ya = pshfl(a, 0, L);
    }
  }

  // Absorb data block d = u-1: a full unit folds into acc (acc*R^L + U with
  // lazy reduction), the trailing partial unit is kept in `tail`.
  P acc = ((uint32_t)q == sh && live) ? ya : pzero();
  P tail = pzero();
  auto absorb = [&](uint64_t u, const uint32_t c[16]) {
    const uint64_t d = u - 1 - sh;
    if (d < nunits) {
      PAcc t = pacc_zero();
      uint32_t ap[36];
      {
        uint32_t slot = threadIdx.x / L;
        asm volatile("" : "+v"(slot));  // re-read per block, not hoisted (registers)
#pragma unroll
        for (int i = 0; i < 9; i++) {
          const uint4 v = s_apow[slot][i];
          ap[4 * i] = v.x; ap[4 * i + 1] = v.y; ap[4 * i + 2] = v.z; ap[4 * i + 3] = v.w;
        }
      }
      pmac_s(t, acc, ap, ap + 5);
      pmac_s(t, pblock(c[0], c[1], c[2], c[3]), ap + 9, ap + 14);
      pmac_s(t, pblock(c[4], c[5], c[6], c[7]), ap + 18, ap + 23);
      pmac_s(t, pblock(c[8], c[9], c[10], c[11]), ap + 27, ap + 32);
      acc = padd(preduce(t), pblock(c[12], c[13], c[14], c[15]));
    } else {
      P tt = pblock(c[0], c[1], c[2], c[3]);
      // (constant indices: a runtime index would move c[] to scratch)
#pragma unroll
      for (uint32_t k = 1; k < 4; k++)
        if (k < tail_blocks)
          tt = padd(pmul(tt, pwr(0)), pblock(c[4 * k], c[4 * k + 1], c[4 * k + 2], c[4 * k + 3]));
      tail = tt;
    }
  };
  if (have0) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint4 v = s_c0[threadIdx.x][i];
      c0[4 * i] = v.x;
      c0[4 * i + 1] = v.y;
      c0[4 * i + 2] = v.z;
      c0[4 * i + 3] = v.w;
    }
    absorb((uint64_t)q, c0);
  }
  // Coalesced I/O: in instruction k, lane l moves 16-byte chunk cj = l mod 4
  // of the block of wave lane t = 16 k + l / 4 (record slot t / L, block
  // t mod L of the iteration: data block it L + t mod L - 1 - sh), so the 64
  // lanes cover 1 KiB of whole record runs (L = 4: 4 records x 256 bytes;
  // L = 2: 8 records x 128 bytes).
  const int cj = lane & 3;
  auto coal_addr = [&](int k, int it, uint64_t &addr) {
    const int t = 16 * k + (lane >> 2);
    uint32_t slot = wbase / L + t / L;
    asm volatile("" : "+v"(slot));  // re-read per use, not hoisted (registers)
    const uint4 inf = s_rinfo[slot];
    const uint64_t dd = (uint64_t)it * L + (t & (L - 1)) - 1 - inf.w;  // (it >= 1: no wrap)
    addr = ((uint64_t)inf.y << 32 | inf.x) + 64 * dd + 16 * cj;
    return dd < inf.z;
  };
  for (int it = 1; it < iters; it++) {
    const uint64_t u = (uint64_t)it * L + q;
    // Laundered ahead of the LDS-DMA loads: hipcc waits for every
    // outstanding LDS-DMA load at an inline asm statement, so none may sit
    // between the loads and the rounds.
    uint32_t kl[8];
    launder_key(key, kl);
    if constexpr (kCoal) {
      // Direct-to-LDS loads (global_load_lds_dwordx4, no VGPRs): instruction
      // k writes the wave's staging bytes [1024 k, 1024 k + 1024) lane-
      // linearly, so lane l lands in the block of wave lane t = 16 k + l / 4
      // at position p = l mod 4, and loads the chunk j whose swizzled
      // position (saddr) is p.
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint64_t a;
        const int t = 16 * k + (lane >> 2);
        const int j = (cj - (t & 3) - (t >> 2)) & 3;
        if (coal_addr(k, it, a))
          __builtin_amdgcn_global_load_lds(
              reinterpret_cast<const void *>(b.in + a - 16 * cj + 16 * j),
              reinterpret_cast<__attribute__((address_space(3))) void *>(
                  reinterpret_cast<uintptr_t>(stage + 1024 * k)),
              16, 0, 0);
      }
    } else {
      prefetch(u, pre);
    }
    chacha_block_raw(kl, (uint32_t)(u - sh), nonce, ks);
    if constexpr (kCoal || IOV) {
      // vmcnt(0): the LDS-DMA loads have landed.  The keystream words are
      // inputs so the rounds stay ahead of the wait (hipcc otherwise sinks
      // them below it and the load latency is exposed).
      asm volatile("s_waitcnt vmcnt(0)" ::"v"(ks[0]), "v"(ks[1]), "v"(ks[2]), "v"(ks[3]),
                   "v"(ks[4]), "v"(ks[5]), "v"(ks[6]), "v"(ks[7]), "v"(ks[8]), "v"(ks[9]),
                   "v"(ks[10]), "v"(ks[11]), "v"(ks[12]), "v"(ks[13]), "v"(ks[14]), "v"(ks[15])
                   : "memory");
    }
    if (u - sh <= nblk) {
      uint32_t c[16];
      crypt_block(u, ks, pre, c, true);
      absorb(u, c);
    }
    if constexpr (kCoal) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint64_t a;
        if (coal_addr(k, it, a)) {
          const uint4 v = *reinterpret_cast<const uint4 *>(stage + saddr(16 * k + (lane >> 2), cj));
          {
            uint4 *o = reinterpret_cast<uint4 *>(b.out + a);
            __builtin_nontemporal_store(v.x, &o->x);
            __builtin_nontemporal_store(v.y, &o->y);
            __builtin_nontemporal_store(v.z, &o->z);
            __builtin_nontemporal_store(v.w, &o->w);
          }
        }
      }
    }
  }

  // Combine the lanes: M = nunits + 1 virtual elements; lane p takes the
  // accumulator of lane (p + M mod L) and the tree weights position p by
  // R^(L-1-p).
  P z = pshfl(acc, (q + (int)((nunits + 1 + sh) % L)) & (L - 1), L);
#pragma unroll
  for (int t = 0; t < kLog; t++) {
    const int sh = 1 << t;
    const P mm = pmul(z, pwr(t + 2));
    const P o = pshfl_down(z, sh, L);
    if ((q & (2 * sh - 1)) == 0) z = padd(mm, o);
  }
  // Z = X * r^t + tail (tail held by the lane of unit `nunits`).
  tail = pshfl(tail, (int)((nunits + 1 + sh) % L), L);
  const int tmax = wave_max((int)tail_blocks);
  for (int k = 0; k < tmax; k++)
    if ((uint32_t)k < tail_blocks) z = pmul(z, pwr(0));
  if (tail_blocks) z = padd(z, tail);
  // h = ((Z r) + L) r with L = le64(ad_len) || le64(ct_len) (+2^128).
  const P lb = pblock((uint32_t)m.ad_len, (uint32_t)(m.ad_len >> 32), (uint32_t)vlen,
                      (uint32_t)(vlen >> 32));
  const P rr = pwr(0);
  const P h = pmul(padd(pmul(z, rr), lb), rr);
  uint32_t tag[4];
  poly_finish(h, s, tag);

  uint8_t *tagp = batch_tag(b, rec);
  int ok = live;
  if (q == 0) {
    if (OPEN && live) {
      // CRYPTO_memcmp (e_chacha20poly1305.cc:322-326) of the first tag_len
      // bytes: dword-aligned loads (one memory round trip instead of one per
      // byte), OR of XORs over the masked words.
      uint32_t t[4];
      load16_partial(tagp, b.tag_len, t);
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t mask = b.tag_len >= 4u * i + 4 ? 0xffffffffu
                              : b.tag_len <= 4u * i   ? 0u
                                                      : ((1u << (8 * (b.tag_len - 4 * i))) - 1u);
        diff |= (tag[i] & mask) ^ t[i];
      }
      ok = diff == 0;
    }
    if (active) {
      if (!OPEN) {
        const uint32_t tw[4] = {ok ? tag[0] : 0u, ok ? tag[1] : 0u, ok ? tag[2] : 0u,
                                ok ? tag[3] : 0u};
        if (b.tag_len == 16 && (reinterpret_cast<uintptr_t>(tagp) & 15) == 0)
          *reinterpret_cast<uint4 *>(tagp) = make_uint4(tw[0], tw[1], tw[2], tw[3]);
        else if ((reinterpret_cast<uintptr_t>(tagp) & 3) == 0)
          store_words_partial(tagp, tw, b.tag_len);
        else
          for (uint32_t i = 0; i < b.tag_len; i++) tagp[i] = (uint8_t)(tw[i >> 2] >> (8 * (i & 3)));
      }
      if (b.status) b.status[rec] = ok ? 1 : 0;
    }
  }
  ok = __shfl(ok, 0, L);
  if (active && !ok && IOV) {
    // clear_iovec (aead.cc.inc:310-333): the record's chunks.
    for (uint64_t c = b.iovec_start[rec]; c < b.iovec_start[rec + 1]; c++) {
      const IovecDev v = b.iovecs[c];
      for (uint64_t i = q; i < v.len; i += L) v.out[i] = 0;
    }
  } else if (active && !ok) {
    for (uint64_t j = q; j * 16 < m.len; j += L) {
      const uint64_t n = umin64(m.len - j * 16, 16);
      for (uint64_t i = 0; i < n; i++) dst[j * 16 + i] = 0;
    }
    if (q == 0)
      for (uint32_t i = 0; i < xlen; i++) xout[i] = 0;
  }
}

// One wave group per wave.  (A persistent form -- 4 or 8 workgroups per CU
// taking record groups from a grid-wide counter -- measured 7-8 % slower on
// configs 3 and 3x, profiles/r03/s10/.)
template <bool OPEN, int L, bool XT, bool XC, bool IOV, bool COAL, bool ANY>
__global__ __launch_bounds__(kThreads) CHACHA_OCC void chacha_poly_kernel(
    const ChaChaKeyDev *__restrict__ keys, BatchDesc b) {
  chacha_group<OPEN, L, XT, XC, IOV, COAL, ANY>(keys, b,
                                (uint64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6));
}

// ---------------------------------------------------------------------------
// One record of at most 16 KiB (the host-buffer EVP_AEAD calls, aead_api.cc
// one_record): latency, not throughput.  Thread t < 256 takes
// ChaCha block t + 1 (data block t) and the fifth wave the Poly1305 key block
// (counter 0); every load of the record -- which may sit in mapped host
// memory, one PCIe round trip each -- is issued first.  Poly1305 runs on the
// 16-byte blocks of pad16(AD) || pad16(C) || lengths staged in LDS, front-
// padded with zero blocks to T * c (which leaves Horner's sum unchanged):
// thread t < T folds its c consecutive blocks by Horner's rule in r, and a
// log2(T)-level tree joins the chunk sums, sum_t h_t r^(c (T-1-t)), with
// multipliers r^c, r^2c, r^4c, ...  (T = 64 chunks, one wave, up to 512
// blocks; else T = 256.)
constexpr int kOneBlocks = 256;               // data blocks: 16 KiB
constexpr int kOneThreads = kOneBlocks + 64;  // + the key-block wave
constexpr int kOnePoly = 2048;                // staged Poly1305 blocks (32 KiB)

// r^e for 1 <= e <= 8 (e wave-uniform).
__device__ __forceinline__ P ppow8(const P &r, uint32_t e) {
  P a = r;
  for (int k = 31 - __builtin_clz(e) - 1; k >= 0; k--) {
    a = pmul(a, a);
    if ((e >> k) & 1) a = pmul(a, r);
  }
  return a;
}

template <bool OPEN, bool XC>
__global__ __launch_bounds__(kOneThreads) void chacha_one_kernel(
    const ChaChaKeyDev *__restrict__ keys, BatchDesc b) {
  __shared__ uint4 s_pb[kOnePoly];
  __shared__ uint32_t s_r[5], s_s[4];
  __shared__ P s_part[kOneBlocks / 64];
  __shared__ int s_ok;
  const int t = threadIdx.x, lane = t & 63;
  constexpr uint32_t kNonceLen = XC ? 24 : 12;
  // (uniform one-record batch, launcher-checked: record 0 at b.in / b.ad)
  const uint64_t len = b.record_len, ad_len = b.ad_len;
  const bool live = b.nonce_len == kNonceLen;  // e_chacha20poly1305.cc:127-130, 241-244
  const uint32_t nad = (uint32_t)((ad_len + 15) / 16), nct = (uint32_t)((len + 15) / 16);
  const uint8_t *src = b.in;
  uint8_t *dst = b.out;
  // Loads first: the lane's 64-byte block, the nonce, the AD blocks.
  const uint32_t n = t < kOneBlocks && 64u * t < len ? (uint32_t)umin64(len - 64u * t, 64)
                                                     : 0u;
  uint4 x[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
    x[k] = nk == 16 ? load16_any(src + 64 * t + 16 * k)
           : nk     ? load_partial(src + 64 * t + 16 * k, nk)
                    : make_uint4(0, 0, 0, 0);
  }
  // (The nonce and a short AD come by value from the single-record host path,
  // BatchDesc::inl, so the keystream does not wait for them.)
  uint4 nw0 = make_uint4(0, 0, 0, 0), nw1 = make_uint4(0, 0, 0, 0);
  if (!XC && (b.inl & 1)) {
    nw0 = make_uint4(b.inl_nonce[0], b.inl_nonce[1], b.inl_nonce[2], 0);
  } else if (live) {
    nw0 = load_partial(b.nonces, XC ? 16 : 12);
    if (XC) nw1 = load_partial(b.nonces + 16, 8);
  }
  if (b.inl & 2) {
    if (t == 0 && nad) s_pb[0] = make_uint4(b.inl_ad[0], b.inl_ad[1], b.inl_ad[2], b.inl_ad[3]);
  } else {
    for (uint32_t a = t; a < nad; a += kOneThreads)
      s_pb[a] = load_partial(b.ad + 16 * a, (uint32_t)umin64(ad_len - 16 * a, 16));
  }
  uint32_t key[8], nonce[3];
#pragma unroll
  for (int i = 0; i < 8; i++) key[i] = keys->k[i];
  if constexpr (XC) {
    // key' = HChaCha20(key, nonce[0:16]), nonce' = 0^4 || nonce[16:24]
    // (e_chacha20poly1305.cc:248-252)
    const uint32_t n4[4] = {nw0.x, nw0.y, nw0.z, nw0.w};
    hchacha20(key, n4);
    nonce[0] = 0;
    nonce[1] = nw1.x;
    nonce[2] = nw1.y;
  } else {
    nonce[0] = nw0.x;
    nonce[1] = nw0.y;
    nonce[2] = nw0.z;
  }
  uint32_t ks[16];
  chacha_block(key, t < kOneBlocks ? (uint32_t)t + 1u : 0u, nonce, ks);
  uint4 y[4];
  if (t >= kOneBlocks) {
    if (t == kOneBlocks) {  // r (clamped, RFC 8439 2.5) and s of the key block
      const uint32_t t0 = ks[0] & 0x0fffffff, t1 = ks[1] & 0x0ffffffc, t2 = ks[2] & 0x0ffffffc,
                     t3 = ks[3] & 0x0ffffffc;
      s_r[0] = t0 & kM26;
      s_r[1] = ((t0 >> 26) | (t1 << 6)) & kM26;
      s_r[2] = ((t1 >> 20) | (t2 << 12)) & kM26;
      s_r[3] = ((t2 >> 14) | (t3 << 18)) & kM26;
      s_r[4] = t3 >> 8;
#pragma unroll
      for (int i = 0; i < 4; i++) s_s[i] = ks[4 + i];
    }
  } else if (n) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
      y[k] = mask_block(make_uint4(x[k].x ^ ks[4 * k], x[k].y ^ ks[4 * k + 1],
                                   x[k].z ^ ks[4 * k + 2], x[k].w ^ ks[4 * k + 3]),
                        nk);
      if (nk) {
        if (!OPEN) {  // the ciphertext (zeros for a dead record, aead.cc.inc:170-179)
          const uint4 o = live ? y[k] : make_uint4(0, 0, 0, 0);
          if (nk == 16)
            store16_any(dst + 64 * t + 16 * k, o);
          else
            store_partial(dst + 64 * t + 16 * k, o, nk);
        }
        s_pb[nad + 4 * t + k] = OPEN ? x[k] : y[k];  // Poly1305 reads the ciphertext
      }
    }
  }
  if (t == 0)  // le64(ad_len) || le64(ct_len)
    s_pb[nad + nct] = make_uint4((uint32_t)ad_len, (uint32_t)(ad_len >> 32), (uint32_t)len,
                                 (uint32_t)(len >> 32));
  __syncthreads();
  const uint32_t nblk = nad + nct + 1;
  const uint32_t T = nblk <= 512 ? 64u : (uint32_t)kOneBlocks;
  const uint32_t c = (nblk + T - 1) / T, pad = T * c - nblk;
  const P r = {{s_r[0], s_r[1], s_r[2], s_r[3], s_r[4]}};
  P h = pzero();
  if ((uint32_t)t < T) {
    for (uint32_t k = 0; k < c; k++) {
      const int64_t a = (int64_t)t * c + k - pad;  // (front padding: h stays 0)
      if (a >= 0) {
        const uint4 m = s_pb[a];
        h = pmul(padd(h, pblock(m.x, m.y, m.z, m.w)), r);
      }
    }
  }
  P rp = ppow8(r, c);  // r^(c 2^l) at level l
#pragma unroll
  for (int l = 0; l < 6; l++) {
    const P o = pshfl_down(h, 1 << l, 64);
    h = padd(pmul(h, rp), o);
    rp = pmul(rp, rp);
  }
  if (T > 64) {  // (block-uniform) the four waves' sums, Horner in r^(64c)
    if (lane == 0 && t < kOneBlocks) s_part[t >> 6] = h;
    __syncthreads();
    if (t == 0) {
      h = s_part[0];
#pragma unroll
      for (int w = 1; w < kOneBlocks / 64; w++) h = padd(pmul(h, rp), s_part[w]);
    }
  }
  if (t == 0) {
    uint32_t tag[4];
    poly_finish(h, s_s, tag);
    uint8_t *tagp = batch_tag(b, 0);
    int ok = live;
    if (OPEN && live) {  // CRYPTO_memcmp (e_chacha20poly1305.cc:322-326)
      const uint4 tr = load_partial(tagp, b.tag_len);
      const uint4 mine = mask_block(make_uint4(tag[0], tag[1], tag[2], tag[3]), b.tag_len);
      ok = ((tr.x ^ mine.x) | (tr.y ^ mine.y) | (tr.z ^ mine.z) | (tr.w ^ mine.w)) == 0;
    }
    if (!OPEN)
      store_partial(tagp, ok ? make_uint4(tag[0], tag[1], tag[2], tag[3]) : make_uint4(0, 0, 0, 0),
                    b.tag_len);
    if (b.status) b.status[0] = ok ? 1 : 0;
    s_ok = ok;
  }
  if (OPEN) {
    __syncthreads();
    if (t < kOneBlocks && n) {  // the plaintext, or zeros after a failed check
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t nk = n > 16u * k ? min(n - 16u * k, 16u) : 0u;
        const uint4 o = s_ok ? y[k] : make_uint4(0, 0, 0, 0);
        if (nk == 16)
          store16_any(dst + 64 * t + 16 * k, o);
        else if (nk)
          store_partial(dst + 64 * t + 16 * k, o, nk);
      }
    }
  }
  if (b.done) {  // completion word (aead_api.cc wait_record): after every store
    // Every thread waits for its own stores; one system-scope release then
    // covers them all.
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0) {
      __threadfence_system();
      __builtin_amdgcn_s_waitcnt(0);  // (the L2 write-back has finished)
      *reinterpret_cast<volatile uint32_t *>(b.done) = b.done_seq;
    }
  }
}

// Batches chacha_one_kernel takes: one contiguous record of at most 16 KiB,
// one key, no extra bytes, AD + record + lengths within the LDS staging.
bool one_record_batch(const BatchDesc &b) {
  if (b.num_records != 1 || b.key_index || b.iovecs || b.extra_len || b.offsets || b.lengths ||
      b.ad_offsets || b.ad_lengths || b.valid || b.order)
    return false;
  return b.record_len <= 64u * kOneBlocks &&
         (b.ad_len + 15) / 16 + (b.record_len + 15) / 16 + 1 <= (uint64_t)kOnePoly;
}

template <bool OPEN, bool XT, bool XC, bool IOV, bool COAL, bool ANY>
void launch_one(const ChaChaKeyDev *keys, const BatchDesc &b, hipStream_t s) {
  constexpr int L = kLanes;
  const uint64_t blocks = (b.num_records * L + kThreads - 1) / kThreads;
  hipLaunchKernelGGL((chacha_poly_kernel<OPEN, L, XT, XC, IOV, COAL, ANY>), dim3((unsigned)blocks),
                     dim3(kThreads), 0, s, keys, b);
}

template <bool XT, bool XC, bool IOV, bool COAL, bool ANY = false>
void launch_dir(const ChaChaKeyDev *keys, const BatchDesc &b, bool open, hipStream_t s) {
  open ? launch_one<true, XT, XC, IOV, COAL, ANY>(keys, b, s)
       : launch_one<false, XT, XC, IOV, COAL, ANY>(keys, b, s);
}

// Uniform batches whose records are not 16-byte aligned take the ANY kernels
// (one dwordx4 per 16 bytes at any address): 1350-byte records at a
// 1351-byte stride 994 against 158 GiB/s through the aligned kernels' byte
// path (profiles/r03/s16/).  Ragged batches keep the aligned kernels (an
// unaligned record there takes the byte path).
bool unaligned_uniform(const BatchDesc &b) {
  return !b.offsets &&
         ((reinterpret_cast<uintptr_t>(b.in) | reinterpret_cast<uintptr_t>(b.out) |
           b.record_stride) & 15) != 0;
}

// The record-contiguous I/O with the slot shift moves whole 128-byte lines
// only when every record starts one: a uniform layout with a 128-byte
// multiple stride and 128-byte-aligned buffers.  Otherwise each lane moves
// its own 64-byte block: config 3 at 16-byte alignment 1,059-1,069 GiB/s that
// way against 939-952 with the record-contiguous I/O (profiles/r03/s13/).
bool whole_lines(const BatchDesc &b) {
  return !b.offsets && b.record_stride % 128 == 0 &&
         ((reinterpret_cast<uintptr_t>(b.in) | reinterpret_cast<uintptr_t>(b.out)) & 127) == 0;
}

}  // namespace

bool chacha_takes_one_record_kernel(const BatchDesc &b) { return one_record_batch(b); }

int launch_chacha(const ChaChaKeyDev *keys, const BatchDesc &b, bool open, bool xchacha,
                  void *stream, const KernelEvents *ev) {
  if (b.num_records == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (one_record_batch(b)) {
    if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
    auto kern = xchacha ? (open ? chacha_one_kernel<true, true> : chacha_one_kernel<false, true>)
                        : (open ? chacha_one_kernel<true, false> : chacha_one_kernel<false, false>);
    hipLaunchKernelGGL(kern, dim3(1), dim3(kOneThreads), 0, s, keys, b);
    const int rc = (int)hipGetLastError();
    if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
    return rc;
  }
  if ((b.num_records * kLanes + kThreads - 1) / kThreads > 0x7fffffffu) return 1;
  BatchDesc bo = b;  // with the processing order of a ragged batch
  uint32_t *order = nullptr;
  if (wants_length_order(b)) {
    if (hipMallocAsync(reinterpret_cast<void **>(&order), (b.num_records + 128) * sizeof(uint32_t),
                       s) != hipSuccess)
      return 2;
    const int orc = build_length_order(b.lengths, b.num_records, order, order + b.num_records, s);
    if (orc) {
      hipFreeAsync(order, s);
      return orc;
    }
    bo.order = order;
  }
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
  const bool xt = b.extra_len != 0, coal = whole_lines(b);
  if (b.iovecs) {  // iovec records walked in place (never with extra bytes)
    xchacha ? launch_dir<false, true, true, false>(keys, bo, open, s)
            : launch_dir<false, false, true, false>(keys, bo, open, s);
  } else if (!xt && unaligned_uniform(b)) {
    xchacha ? launch_dir<false, true, false, false, true>(keys, bo, open, s)
            : launch_dir<false, false, false, false, true>(keys, bo, open, s);
  } else if (xchacha) {
    if (xt)
      coal ? launch_dir<true, true, false, true>(keys, bo, open, s)
           : launch_dir<true, true, false, false>(keys, bo, open, s);
    else
      coal ? launch_dir<false, true, false, true>(keys, bo, open, s)
           : launch_dir<false, true, false, false>(keys, bo, open, s);
  } else {
    if (xt)
      coal ? launch_dir<true, false, false, true>(keys, bo, open, s)
           : launch_dir<true, false, false, false>(keys, bo, open, s);
    else
      coal ? launch_dir<false, false, false, true>(keys, bo, open, s)
           : launch_dir<false, false, false, false>(keys, bo, open, s);
  }
  const int rc = (int)hipGetLastError();
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
  if (order) hipFreeAsync(order, s);
  return rc;
}

}  // namespace bssl_amd
