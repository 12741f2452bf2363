// gf128_ct.h -- constant-time GHASH multiplication on the integer VALU.
//
// GF(2^128) products whose operands are secret (derived from H or from the
// data) and that the conflict-free LDS byte table of gcm.hip does not cover:
// the record-end combine and tag (gcm.hip finish_record, the one-record
// kernel), the multi-block AD hash and the GHASH-derived J0 of non-96-bit
// nonces, the in-kernel byte tables of H^L (build_gpow) and the host key
// setup.  (gcm_siv.hip does not use it: its POLYVAL products go through
// per-record Shoup tables read by one ds_read_b128 lane group, DESIGN.md
// §4.8.)  The
// reference computes these on CPUs without carry-less multiply in the same
// spirit (crypto/fipsmodule/aes/gcm_nohw.cc.inc:38-82): carry-less products
// from ordinary integer multiplications whose operands are masked to every
// fourth bit ("holes"), so no carry reaches a bit that is kept.  Nothing here
// branches on or indexes memory by a secret; the multiplier's latency on
// gfx950 does not depend on its operands.  The algebra below is written from
// SP 800-38D (bit-reflected field, g = x^128 + x^7 + x^2 + x + 1) and checked
// against the oracle's bitwise GHASH multiply (tests/test_gf128_ct.py).
//
// Representation ("reversed domain"): the 16 bytes b0..b15 of a GHASH block
// as the big-endian integer V = b0 << 120 | ... | b15, in four 32-bit words,
// w[0] least significant.  Bit j of V is the coefficient of x^(127-j).  For
// a product a*b the caller supplies the multiplier prepared as b' = b / x
// (gf_prep), so the 256-bit carry-less product of the two words needs no
// realignment: its low 128 bits hold the reversed coefficients of degree
// 128..255 and its high 128 bits those of degree 0..127; the high-degree part
// is folded back with x^128 = x^7 + x^2 + x + 1 as shifts of the reversed
// integer (a multiplication by x^s is a right shift by s).
//
// Compiles for the host too (tests build it with g++).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BSSL_GF_HD __host__ __device__ __forceinline__
#else
#define BSSL_GF_HD static inline
#endif

namespace bssl_amd {

struct Gf128 {
  uint32_t w[4];  // reversed-domain value, w[0] least significant
};

// Carry-less 32 x 32 -> 64.  a_i / b_j keep the bits of a / b at positions
// = i / j (mod 4); the integer product a_i * b_j has its non-zero raw column
// sums only at positions = i + j (mod 4), each at most 8 (8 bits per part),
// so every sum fits its 4-bit window without reaching the next kept bit and
// bit p of the product is the parity of column p.  Products of one class are
// XORed and the class's bits kept.
BSSL_GF_HD uint64_t clmul32(uint32_t a, uint32_t b) {
  const uint32_t m0 = 0x11111111u, m1 = 0x22222222u, m2 = 0x44444444u, m3 = 0x88888888u;
  const uint64_t a0 = a & m0, a1 = a & m1, a2 = a & m2, a3 = a & m3;
  const uint64_t b0 = b & m0, b1 = b & m1, b2 = b & m2, b3 = b & m3;
  const uint64_t z0 = (a0 * b0) ^ (a1 * b3) ^ (a2 * b2) ^ (a3 * b1);
  const uint64_t z1 = (a0 * b1) ^ (a1 * b0) ^ (a2 * b3) ^ (a3 * b2);
  const uint64_t z2 = (a0 * b2) ^ (a1 * b1) ^ (a2 * b0) ^ (a3 * b3);
  const uint64_t z3 = (a0 * b3) ^ (a1 * b2) ^ (a2 * b1) ^ (a3 * b0);
  return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) |
         (z2 & 0x4444444444444444ull) | (z3 & 0x8888888888888888ull);
}

// Carry-less 64 x 64 -> 128 (Karatsuba over 32-bit halves: 3 clmul32).
BSSL_GF_HD void clmul64(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint32_t r[4]) {
  const uint64_t lo = clmul32(a0, b0), hi = clmul32(a1, b1);
  const uint64_t mid = clmul32(a0 ^ a1, b0 ^ b1) ^ lo ^ hi;
  r[0] = (uint32_t)lo;
  r[1] = (uint32_t)(lo >> 32) ^ (uint32_t)mid;
  r[2] = (uint32_t)hi ^ (uint32_t)(mid >> 32);
  r[3] = (uint32_t)(hi >> 32);
}

// a * b in GF(2^128), with bp = gf_prep(b).  9 clmul32 (two Karatsuba
// levels) and the reduction.
BSSL_GF_HD Gf128 gf_mul(Gf128 a, Gf128 bp) {
  uint32_t l[4], h[4], m[4];
  clmul64(a.w[0], a.w[1], bp.w[0], bp.w[1], l);
  clmul64(a.w[2], a.w[3], bp.w[2], bp.w[3], h);
  clmul64(a.w[0] ^ a.w[2], a.w[1] ^ a.w[3], bp.w[0] ^ bp.w[2], bp.w[1] ^ bp.w[3], m);
  for (int i = 0; i < 4; i++) m[i] ^= l[i] ^ h[i];
  // 256-bit product c = l ^ m << 64 ^ h << 128: c[0..3] low half, c[4..7] high.
  const uint32_t c0 = l[0], c1 = l[1], c2 = l[2] ^ m[0], c3 = l[3] ^ m[1];
  const uint32_t c4 = h[0] ^ m[2], c5 = h[1] ^ m[3], c6 = h[2], c7 = h[3];
  // Low half = reversed coefficients of degree 128..255 (t), high half = degree
  // 0..127.  t * (1 + x + x^2 + x^7): its bits shifted past x^127 (the low 7
  // bits of t moved to the top by the three shifts) are folded into t first.
  const uint32_t t0 = c0, t1 = c1, t2 = c2;
  const uint32_t t3 = c3 ^ (c0 << 31) ^ (c0 << 30) ^ (c0 << 25);
  auto shr = [&](int s, uint32_t out[4]) {
    out[0] = (t0 >> s) | (t1 << (32 - s));
    out[1] = (t1 >> s) | (t2 << (32 - s));
    out[2] = (t2 >> s) | (t3 << (32 - s));
    out[3] = t3 >> s;
  };
  uint32_t s1[4], s2[4], s7[4];
  shr(1, s1);
  shr(2, s2);
  shr(7, s7);
  Gf128 r;
  r.w[0] = c4 ^ t0 ^ s1[0] ^ s2[0] ^ s7[0];
  r.w[1] = c5 ^ t1 ^ s1[1] ^ s2[1] ^ s7[1];
  r.w[2] = c6 ^ t2 ^ s1[2] ^ s2[2] ^ s7[2];
  r.w[3] = c7 ^ t3 ^ s1[3] ^ s2[3] ^ s7[3];
  return r;
}

// b' = b / x (x^-1 = x^127 + x^6 + x + 1): the reversed integer shifted left
// by one; if b had an x^0 term (bit 127), g / x is added (bits 0, 121, 126,
// 127).  Constant time (the term is selected by a mask).
BSSL_GF_HD Gf128 gf_prep(Gf128 b) {
  const uint32_t top = 0u - (b.w[3] >> 31);
  Gf128 r;
  r.w[3] = (b.w[3] << 1) | (b.w[2] >> 31);
  r.w[2] = (b.w[2] << 1) | (b.w[1] >> 31);
  r.w[1] = (b.w[1] << 1) | (b.w[0] >> 31);
  r.w[0] = b.w[0] << 1;
  r.w[0] ^= top & 1u;
  r.w[3] ^= top & 0xc2000000u;
  return r;
}

// Block bytes -> reversed domain and back (big-endian words).
BSSL_GF_HD Gf128 gf_from_bytes(const uint8_t b[16]) {
  Gf128 r;
  for (int i = 0; i < 4; i++)
    r.w[3 - i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) |
                 ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
  return r;
}

BSSL_GF_HD void gf_to_bytes(Gf128 v, uint8_t b[16]) {
  for (int i = 0; i < 4; i++) {
    const uint32_t x = v.w[3 - i];
    b[4 * i] = (uint8_t)(x >> 24);
    b[4 * i + 1] = (uint8_t)(x >> 16);
    b[4 * i + 2] = (uint8_t)(x >> 8);
    b[4 * i + 3] = (uint8_t)x;
  }
}

}  // namespace bssl_amd
