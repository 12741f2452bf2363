// gcm.hip -- AES-GCM seal/open over device-resident record batches (gfx950).
//
// Replaces the reference's per-record CPU path
//   aead_aes_gcm_sealv_impl / _openv_detached_impl (crypto/fipsmodule/cipher/
//   e_aes.cc.inc:779-867) -> CRYPTO_gcm128_{init_ctx,aad,encrypt,decrypt,tag}
//   (crypto/fipsmodule/aes/gcm.cc.inc:298-604) -> aes_gcm_enc_update_vaes_avx512
//   (aes-gcm-avx512-x86_64.pl:845)
// with one kernel that processes many records at once.  Design:
//
// * Work split.  A 64-lane wavefront holds 4 records, 16 lanes ("a group") per
//   record.  Lane q of a group owns the record's 16-byte blocks j = q, q+16,
//   q+32, ...: it encrypts counter block inc32(J0, 1+j) (one thread per counter
//   block), XORs the plaintext (coalesced 256-byte runs per group) and folds
//   the ciphertext block into a private GHASH accumulator by Horner's rule with
//   multiplier H^16.  At the end of the record the 16 accumulators are rotated
//   into exponent order and combined by a 4-level tree (H, H^2, H^4, H^8)
//   inside the group; lane 0 finishes the tag (length block, x H, xor E_K(J0)).
// * AES.  T-table rounds, the tables in LDS and replicated once per LDS bank
//   (entry idx of table t for lane l at byte idx*256 + t*128 + (l%32)*4), so a
//   wave's 64 random lookups are bank-conflict free.  Only T0 and T1 are
//   stored; T2/T3 are the 16-bit rotations of T0/T1 and are folded into one
//   rotate per column.  Each lookup address is built with one v_perm_b32.
// * GHASH.  Multiplication by a fixed power of H is linear over GF(2): 32
//   lookups (one per nibble) of 16-byte entries in a 256-byte table per
//   nibble position.  A table spans all 64 banks and every lane of the wave
//   reads the same position's table at the same time, so ds_read_b128 is
//   conflict free.  Tables for H, H^2, H^4, H^8, H^16 (40 KiB) sit in LDS.
// * Round keys are wave-uniform and live in SGPRs.  A workgroup handles one
//   key at a time; records are visited in tiles of 32 and a tile whose
//   records use several keys is processed in one pass per distinct key.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <type_traits>

#include "internal.h"
#include "iov_dev.h"
#include "gcm_common.h"


namespace bssl_amd {
namespace {

// Waves per workgroup: one workgroup per CU (the LDS tables take 128 KiB),
// 16 waves at 128 VGPRs (4 -> 573, 8 -> 981, 16 -> 1,156 GiB/s, DESIGN.md
// §4.2).  Plaintext loads and ciphertext stores carry the non-temporal hint
// (each byte is touched once: +1.7 % on config 2).
constexpr int kWaves = 16;
constexpr int kRecPerWave = 4;

// ---------------------------------------------------------------------------
// Compile-time AES tables.
struct Tables {
  uint32_t te0[256];
};

constexpr uint8_t cx_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return p;
}

constexpr Tables make_tables() {
  Tables t{};
  for (int x = 0; x < 256; x++) {
    // inverse = x^254 (square-and-multiply), 0 -> 0
    uint8_t inv = 1, base = (uint8_t)x;
    for (int e = 254; e; e >>= 1) {
      if (e & 1) inv = cx_mul(inv, base);
      base = cx_mul(base, base);
    }
    if (!x) inv = 0;
    uint8_t s = inv, r = inv;
    for (int i = 0; i < 4; i++) {
      r = (uint8_t)((r << 1) | (r >> 7));
      s ^= r;
    }
    s ^= 0x63;
    uint8_t s2 = cx_mul(s, 2), s3 = cx_mul(s, 3);
    // Te0[x] bytes (2s, s, s, 3s): the column a row-0 byte contributes.
    t.te0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
  }
  return t;
}

__constant__ Tables kTables = make_tables();

// ---------------------------------------------------------------------------
// LDS layout of the T-table kernel (one static array at LDS address 0):
//   [0, 65536)       GHASH byte table of H^16, "lane-rotated": the product of
//                    (byte value e at byte position p) x H^16 at e*256 + p*16
//                    (16 positions side by side in one 256-byte row, so 16
//                    lanes reading 16 different positions never share a bank)
//   [65536, 131072)  AES T0/T1, replicated per bank (see header comment); the
//                    lookup address carries bit 16 (lane constants lc0/lc1)
//   [131072, ...)    tile plan (keys and record masks of the passes)
constexpr uint32_t kLdsAes = kG8Bytes;
constexpr uint32_t kAesLdsBytes = 256 * 256;
constexpr uint32_t kLdsPlan = kLdsAes + kAesLdsBytes;
constexpr uint32_t kLdsBasis = kLdsPlan + 64 * 16 + 16;  // 128 x 16 B (build_gpow)
constexpr uint32_t kLdsBytes = kLdsBasis + 128 * 16;
//   [kLdsBytes, ...) iovec kernels (GCM_IOV_LDS): per record slot (one per L
//                    lanes of the workgroup) the record's chunk range
//                    [c0, c_end) and its first kIovKc chunk descriptors
#ifndef GCM_IOV_LDS
#define GCM_IOV_LDS 1
#endif
constexpr bool kIovLds = GCM_IOV_LDS != 0;
template <int L>
constexpr uint32_t kIovKc = L == 4 ? 3u : 4u;
template <int L>
constexpr uint32_t kIovSlot = kIovSlotBytes<kIovKc<L>>;
template <int L, int THREADS>
constexpr uint32_t kLdsIovBytes = kLdsBytes + (kIovLds ? (THREADS / L) * kIovSlot<L> : 0u);

// ---------------------------------------------------------------------------
// AES.  State: 4 little-endian column words (byte r of word c = row r).
// Lookup address of the T(slot) entry for state byte k: v_perm puts byte k at
// bits 8..15 below which the lane/slot constant `lc` (bits 0..7) sits; byte 2
// of `lc` (the table base's bit 16) is carried along.
template <int K>
__device__ __forceinline__ uint32_t taddr(uint32_t lc, uint32_t s) {
  return __builtin_amdgcn_perm(lc, s, 0x0c060004u | (K << 8));
}

template <uint32_t TB>
__device__ __forceinline__ uint32_t tload(const uint8_t *smem, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(smem + TB + a);
}

// One full round column: rows come from columns (a, b, c, d); rkx is the round
// key word pre-rotated by 16:  T0[a0] ^ T1[b1] ^ rotl16(T0[c2] ^ T1[d3] ^ rkx).
template <uint32_t TB>
__device__ __forceinline__ uint32_t round_col(const uint8_t *smem, uint32_t lc0, uint32_t lc1,
                                              uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                              uint32_t rkx) {
  const uint32_t x0 = tload<TB>(smem, taddr<0>(lc0, a));
  const uint32_t x1 = tload<TB>(smem, taddr<1>(lc1, b));
  const uint32_t x2 = tload<TB>(smem, taddr<2>(lc0, c));
  const uint32_t x3 = tload<TB>(smem, taddr<3>(lc1, d));
  return xor3(x0, x1, rotl(xor3(x2, x3, rkx), 16));
}

template <uint32_t TB>
__device__ __forceinline__ uint32_t last_col(const uint8_t *smem, uint32_t lc0, uint32_t a,
                                             uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
  const uint32_t x0 = tload<TB>(smem, taddr<0>(lc0, a));
  const uint32_t x1 = tload<TB>(smem, taddr<1>(lc0, b));
  const uint32_t x2 = tload<TB>(smem, taddr<2>(lc0, c));
  const uint32_t x3 = tload<TB>(smem, taddr<3>(lc0, d));
  // S[x] is byte 1 (and byte 2) of Te0[x].
  const uint32_t lo = __builtin_amdgcn_perm(x1, x0, 0x0c0c0501u);
  const uint32_t hi = __builtin_amdgcn_perm(x3, x2, 0x06020c0cu);
  return xor3(lo, hi, rk);
}

struct RoundKeys {
  uint32_t w[15][4];
};

// One full AES round on all four columns.  All 16 lookups are issued before
// any is consumed so a wave keeps 16 LDS reads in flight (the per-column form
// lets hipcc wait after every 4).
template <uint32_t TB>
__device__ __forceinline__ void aes_round(uint32_t &s0, uint32_t &s1, uint32_t &s2,
                                          uint32_t &s3, const uint32_t *rkx,
                                          const uint8_t *smem, uint32_t lc0, uint32_t lc1) {
  const uint32_t a00 = taddr<0>(lc0, s0), a01 = taddr<1>(lc1, s1), a02 = taddr<2>(lc0, s2),
                 a03 = taddr<3>(lc1, s3);
  const uint32_t a10 = taddr<0>(lc0, s1), a11 = taddr<1>(lc1, s2), a12 = taddr<2>(lc0, s3),
                 a13 = taddr<3>(lc1, s0);
  const uint32_t a20 = taddr<0>(lc0, s2), a21 = taddr<1>(lc1, s3), a22 = taddr<2>(lc0, s0),
                 a23 = taddr<3>(lc1, s1);
  const uint32_t a30 = taddr<0>(lc0, s3), a31 = taddr<1>(lc1, s0), a32 = taddr<2>(lc0, s1),
                 a33 = taddr<3>(lc1, s2);
  const uint32_t x00 = tload<TB>(smem, a00), x01 = tload<TB>(smem, a01),
                 x02 = tload<TB>(smem, a02), x03 = tload<TB>(smem, a03);
  const uint32_t x10 = tload<TB>(smem, a10), x11 = tload<TB>(smem, a11),
                 x12 = tload<TB>(smem, a12), x13 = tload<TB>(smem, a13);
  const uint32_t x20 = tload<TB>(smem, a20), x21 = tload<TB>(smem, a21),
                 x22 = tload<TB>(smem, a22), x23 = tload<TB>(smem, a23);
  const uint32_t x30 = tload<TB>(smem, a30), x31 = tload<TB>(smem, a31),
                 x32 = tload<TB>(smem, a32), x33 = tload<TB>(smem, a33);
  s0 = xor3(x00, x01, rotl(xor3(x02, x03, rkx[0]), 16));
  s1 = xor3(x10, x11, rotl(xor3(x12, x13, rkx[1]), 16));
  s2 = xor3(x20, x21, rotl(xor3(x22, x23, rkx[2]), 16));
  s3 = xor3(x30, x31, rotl(xor3(x32, x33, rkx[3]), 16));
}

// AES rounds R0..NR on a state that already includes rounds < R0.
template <int NR, uint32_t TB, int R0 = 1>
__device__ __forceinline__ uint4 aes_rounds(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                            const RoundKeys &rk, const uint8_t *smem,
                                            uint32_t lc0, uint32_t lc1) {
#pragma unroll
  for (int r = R0; r < NR; r++) aes_round<TB>(s0, s1, s2, s3, rk.w[r], smem, lc0, lc1);
  const uint32_t a00 = taddr<0>(lc0, s0), a01 = taddr<1>(lc0, s1), a02 = taddr<2>(lc0, s2),
                 a03 = taddr<3>(lc0, s3);
  const uint32_t a10 = taddr<0>(lc0, s1), a11 = taddr<1>(lc0, s2), a12 = taddr<2>(lc0, s3),
                 a13 = taddr<3>(lc0, s0);
  const uint32_t a20 = taddr<0>(lc0, s2), a21 = taddr<1>(lc0, s3), a22 = taddr<2>(lc0, s0),
                 a23 = taddr<3>(lc0, s1);
  const uint32_t a30 = taddr<0>(lc0, s3), a31 = taddr<1>(lc0, s0), a32 = taddr<2>(lc0, s1),
                 a33 = taddr<3>(lc0, s2);
  const uint32_t x00 = tload<TB>(smem, a00), x01 = tload<TB>(smem, a01),
                 x02 = tload<TB>(smem, a02), x03 = tload<TB>(smem, a03);
  const uint32_t x10 = tload<TB>(smem, a10), x11 = tload<TB>(smem, a11),
                 x12 = tload<TB>(smem, a12), x13 = tload<TB>(smem, a13);
  const uint32_t x20 = tload<TB>(smem, a20), x21 = tload<TB>(smem, a21),
                 x22 = tload<TB>(smem, a22), x23 = tload<TB>(smem, a23);
  const uint32_t x30 = tload<TB>(smem, a30), x31 = tload<TB>(smem, a31),
                 x32 = tload<TB>(smem, a32), x33 = tload<TB>(smem, a33);
  // Last round: S[x] is byte 1 (and byte 2) of Te0[x].
  uint4 o;
  o.x = xor3(__builtin_amdgcn_perm(x01, x00, 0x0c0c0501u),
             __builtin_amdgcn_perm(x03, x02, 0x06020c0cu), rk.w[NR][0]);
  o.y = xor3(__builtin_amdgcn_perm(x11, x10, 0x0c0c0501u),
             __builtin_amdgcn_perm(x13, x12, 0x06020c0cu), rk.w[NR][1]);
  o.z = xor3(__builtin_amdgcn_perm(x21, x20, 0x0c0c0501u),
             __builtin_amdgcn_perm(x23, x22, 0x06020c0cu), rk.w[NR][2]);
  o.w = xor3(__builtin_amdgcn_perm(x31, x30, 0x0c0c0501u),
             __builtin_amdgcn_perm(x33, x32, 0x06020c0cu), rk.w[NR][3]);
  return o;
}

// E_K(J0) by the 4 lanes of a quad, one state column each (gcm.cc.inc:340-343):
// DPP quad permutations hand each lane the three other columns, so a round
// costs a lane 4 table lookups instead of 16 -- every lane of a record needs
// the same block, and the LDS cost is per wave-instruction.  In: the round-0
// state (J0 ^ rk0); out: column (lane & 3) of E_K(J0).
__device__ __forceinline__ uint32_t quad_rot(uint32_t v, int k) {
  // lane i of the quad gets lane (i + k) & 3: quad_perm [1,2,3,0] / [2,3,0,1] / [3,0,1,2]
  return k == 1 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x39, 0xf, 0xf, false)
       : k == 2 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false)
                : (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x93, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t quad_sel(uint32_t c, uint32_t a, uint32_t b, uint32_t d,
                                             uint32_t e) {
  return (c & 2) ? ((c & 1) ? e : d) : ((c & 1) ? b : a);
}
template <int NR, uint32_t TB>
__device__ __forceinline__ uint32_t ek0_quad(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                             const RoundKeys &rk, const uint8_t *smem,
                                             uint32_t lc0, uint32_t lc1) {
  const uint32_t c = threadIdx.x & 3;
  uint32_t w = quad_sel(c, s0, s1, s2, s3);
#pragma unroll
  for (int r = 1; r < NR; r++) {
    const uint32_t w1 = quad_rot(w, 1), w2 = quad_rot(w, 2), w3 = quad_rot(w, 3);
    const uint32_t kx = quad_sel(c, rk.w[r][0], rk.w[r][1], rk.w[r][2], rk.w[r][3]);
    w = round_col<TB>(smem, lc0, lc1, w, w1, w2, w3, kx);
  }
  const uint32_t w1 = quad_rot(w, 1), w2 = quad_rot(w, 2), w3 = quad_rot(w, 3);
  return last_col<TB>(smem, lc0, w, w1, w2, w3,
                      quad_sel(c, rk.w[NR][0], rk.w[NR][1], rk.w[NR][2], rk.w[NR][3]));
}
// All four columns of a quad's block in every lane of the quad.
__device__ __forceinline__ uint4 quad_gather(uint32_t w) {
  return make_uint4((uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x00, 0xf, 0xf, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x55, 0xf, 0xf, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xaa, 0xf, 0xf, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xff, 0xf, 0xf, false));
}

// ---------------------------------------------------------------------------
// Counter-mode cache of one AES stream (see process_records).
struct WindowCache {
  uint32_t win = 0xffffffffu, k1 = 0, k2 = 0, k3 = 0, l0 = 0, l1 = 0, l2 = 0, l3 = 0;

  template <uint32_t T>
  __device__ __forceinline__ void update(uint32_t ctr, uint32_t s3, uint32_t c0, uint32_t c1,
                                         uint32_t c2, const RoundKeys &rk,
                                         const uint8_t *smem, uint32_t lc0, uint32_t lc1) {
    if ((ctr >> 8) == win) return;
    win = ctr >> 8;
    k1 = round_col<T>(smem, lc0, lc1, c1, c2, s3, c0, rk.w[1][1]);
    k2 = round_col<T>(smem, lc0, lc1, c2, s3, c0, c1, rk.w[1][2]);
    k3 = round_col<T>(smem, lc0, lc1, s3, c0, c1, c2, rk.w[1][3]);
    l0 = tload<T>(smem, taddr<1>(lc1, k1)) ^
         rotl(tload<T>(smem, taddr<2>(lc0, k2)) ^ tload<T>(smem, taddr<3>(lc1, k3)) ^
                  rk.w[2][0], 16);
    l1 = tload<T>(smem, taddr<0>(lc0, k1)) ^ tload<T>(smem, taddr<1>(lc1, k2)) ^
         rotl(tload<T>(smem, taddr<2>(lc0, k3)) ^ rk.w[2][1], 16);
    l2 = tload<T>(smem, taddr<0>(lc0, k2)) ^ tload<T>(smem, taddr<1>(lc1, k3)) ^
         rotl(tload<T>(smem, taddr<3>(lc1, k1)) ^ rk.w[2][2], 16);
    l3 = tload<T>(smem, taddr<0>(lc0, k3)) ^
         rotl(tload<T>(smem, taddr<2>(lc0, k1)) ^ tload<T>(smem, taddr<3>(lc1, k2)) ^
                  rk.w[2][3], 16);
  }

  // Rounds 1 and 2 of a counter block whose round-0 word 3 is s3.
  template <uint32_t T>
  __device__ __forceinline__ void rounds12(uint32_t k0, uint32_t s3, uint32_t &u0, uint32_t &u1,
                                           uint32_t &u2, uint32_t &u3, const uint8_t *smem,
                                           uint32_t lc0, uint32_t lc1) const {
    const uint32_t t0 = k0 ^ rotl(tload<T>(smem, taddr<3>(lc1, s3)), 16);
    u0 = tload<T>(smem, taddr<0>(lc0, t0)) ^ l0;
    u1 = rotl(tload<T>(smem, taddr<3>(lc1, t0)), 16) ^ l1;
    u2 = rotl(tload<T>(smem, taddr<2>(lc0, t0)), 16) ^ l2;
    u3 = tload<T>(smem, taddr<1>(lc1, t0)) ^ l3;
  }
};

#include "gcm_rounds.inc"

// GHASH steps carried by middle round i (rounds 3..NR-1 -> i = 0..NR-4) of
// the one-block-per-lane kernel: AES-128 has 7 such rounds (3,3,2,2,2,2,2),
// AES-192/256 spread 2 per round over the first 8.
template <int NR>
constexpr int g_steps(int i) {
  if (NR == 10) return i < 2 ? 3 : 2;
  return i < 8 ? 2 : 0;
}
template <int NR>
constexpr int g_first(int i) {
  int t = 0;
  for (int k = 0; k < i; k++) t += g_steps<NR>(k);
  return t;
}

template <int T>
__device__ __forceinline__ uint32_t gh_word(const Gh8 &h) {
  return T < 4 ? h.r0 : T < 8 ? h.r1 : T < 12 ? h.r2 : h.r3;
}

// Middle rounds 3..NR-1 of one state (inline-asm rounds, gcm_rounds.inc),
// with round i carrying GHASH steps g_first(i) .. +g_steps(i) and, for the
// next block of the lane, its cached rounds 1 and 2 (software pipelining:
// the next iteration starts at round 3): round i = 0 issues the round-1
// lookup of `xs` (its round-0 word 3), round i = 1 the four round-2 lookups.
template <int I, int NR>
__device__ __forceinline__ void rounds_s1(uint32_t (&a)[4], const RoundKeys &rk, uint32_t lc0,
                                          uint32_t lc1, Gh8 &h, const uint32_t (&P)[4],
                                          uint32_t &xs, const WindowCache &wc, uint32_t k0,
                                          uint32_t (&nx)[4]) {
  constexpr int R = I + 3;
  if constexpr (R < NR) {
    constexpr int NG = g_steps<NR>(I);
    constexpr int T = g_first<NR>(I);
    constexpr int X = I == 0 ? 1 : I == 1 ? 4 : 0;
    uint32_t xo[X > 0 ? X : 1];
    if constexpr (NG > 0) {
      const uint32_t gr[3] = {gh_word<T>(h), gh_word<T + 1>(h),
                                            gh_word<(NG > 2 ? T + 2 : T)>(h)};
      const uint32_t gp[3] = {P[T >> 2], P[(T + 1) >> 2],
                                            P[(NG > 2 ? T + 2 : T) >> 2]};
      const uint32_t gsel[3] = {g8_sel<T>(), g8_sel<T + 1>(),
                                              g8_sel<(NG > 2 ? T + 2 : T)>()};
      v4u gv[NG > 0 ? NG : 1];
      if constexpr (X == 1 && NG == 3)
        asm_round_s1_x1_g3(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv, xs, xo);
      else if constexpr (X == 1 && NG == 2)
        asm_round_s1_x1_g2(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv, xs, xo);
      else if constexpr (X == 4 && NG == 3)
        asm_round_s1_x4_g3(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv, xs, xo);
      else if constexpr (X == 4 && NG == 2)
        asm_round_s1_x4_g2(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv, xs, xo);
      else if constexpr (NG == 3)
        asm_round_s1_x0_g3(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv);
      else
        asm_round_s1_x0_g2(a, rk.w[R], lc0, lc1, gr, gp, gsel, gv);
      if constexpr (NG == 3)
        h.g = xor4(xor4_3(h.g, as_uint4(gv[0]), as_uint4(gv[1])), as_uint4(gv[2]));
      else
        h.g = xor4_3(h.g, as_uint4(gv[0]), as_uint4(gv[1]));
      pin4(h.g);
    } else {
      if constexpr (X == 1)
        asm_round_s1_x1_g0(a, rk.w[R], lc0, lc1, xs, xo);
      else if constexpr (X == 4)
        asm_round_s1_x4_g0(a, rk.w[R], lc0, lc1, xs, xo);
      else
        asm_round_s1_x0_g0(a, rk.w[R], lc0, lc1);
    }
    if constexpr (X == 1) {
      xs = k0 ^ rotl(xo[0], 16);  // round-1 output word 0 of the next block
    } else if constexpr (X == 4) {
      // Round-2 output of the next block (WindowCache::rounds12), to nx.
      xo[0] ^= wc.l0;
      xo[1] = rotl(xo[1], 16) ^ wc.l1;
      xo[2] = rotl(xo[2], 16) ^ wc.l2;
      xo[3] ^= wc.l3;
    }
    if constexpr (X == 4) {
      nx[0] = xo[0];
      nx[1] = xo[1];
      nx[2] = xo[2];
      nx[3] = xo[3];
    }
    rounds_s1<I + 1, NR>(a, rk, lc0, lc1, h, P, xs, wc, k0, nx);
  }
}



// ---------------------------------------------------------------------------
// One AES block with T0 alone, replicated once per LDS bank (one-record kernel):
// entry x for lane l at tab[x * 32 + (l & 31)] (32 KiB), so every lookup of a
// wave is bank-conflict free whatever the index -- the same constant-time
// argument as the bulk kernel's tables, at half their size
// so more prologue workgroups fit per CU.  T1..T3 are rotations of T0; the
// middle round keys arrive pre-rotated by 16 (GcmKeyDev::rk).
template <int K>
__device__ __forceinline__ uint32_t t0r(const uint32_t *tab, uint32_t s, uint32_t lane) {
  return tab[__builtin_amdgcn_ubfe(s, 8 * K, 8) * 32 + lane];
}

template <int NR>
__device__ __forceinline__ uint4 aes_block_rep(uint4 in, const RoundKeys &rk, const uint32_t *tab) {
  const uint32_t l = threadIdx.x & 31;
  uint32_t s0 = in.x ^ rk.w[0][0], s1 = in.y ^ rk.w[0][1], s2 = in.z ^ rk.w[0][2],
           s3 = in.w ^ rk.w[0][3];
  auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kx) {
    // T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ kx), T1 = rotl8(T0)
    return xor3(t0r<0>(tab, a, l), rotl(t0r<1>(tab, b, l), 8),
                rotl(xor3(t0r<2>(tab, c, l), rotl(t0r<3>(tab, d, l), 8), kx), 16));
  };
#pragma unroll
  for (int r = 1; r < NR; r++) {
    const uint32_t *kx = rk.w[r];
    const uint32_t t0 = col(s0, s1, s2, s3, kx[0]), t1 = col(s1, s2, s3, s0, kx[1]),
                   t2 = col(s2, s3, s0, s1, kx[2]), t3 = col(s3, s0, s1, s2, kx[3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  // Last round: S[x] is byte 1 (and byte 2) of Te0[x].
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    return xor3(__builtin_amdgcn_perm(t0r<1>(tab, b, l), t0r<0>(tab, a, l), 0x0c0c0501u),
                __builtin_amdgcn_perm(t0r<3>(tab, d, l), t0r<2>(tab, c, l), 0x06020c0cu), k);
  };
  return make_uint4(last(s0, s1, s2, s3, rk.w[NR][0]), last(s1, s2, s3, s0, rk.w[NR][1]),
                    last(s2, s3, s0, s1, rk.w[NR][2]), last(s3, s0, s1, s2, rk.w[NR][3]));
}

// ---------------------------------------------------------------------------
// Bulk kernel: CTR keystream + GHASH + tag for the (up to) 4 records of a
// wave, 16 lanes per record.  `active` is per group (record in this key pass).
// `key` = the batch key (record-end products, finish_record).
// L = lanes per record (16: 4 records per wave, GHASH stride H^16; 32: 2
// records per wave, stride H^32 -- the byte table in LDS must be of H^L).
// RP: rotate the wave's issue priority every iteration ((prio_base + it) mod
// 4) -- in the tiled path all 16 waves must finish their units together, and
// with fixed priorities the SIMD arbiter's age order makes the youngest wave
// of each SIMD ~1.9x slower than the oldest.
#ifndef GCM_IOV_HANDOFF
#define GCM_IOV_HANDOFF 1
#endif
constexpr bool kIovHandoff = GCM_IOV_HANDOFF != 0;
#ifndef GCM_IOV_KEEP_END
#define GCM_IOV_KEEP_END 0
#endif
constexpr bool kIovKeepEnd = GCM_IOV_KEEP_END != 0;

// iovec block loads are temporal at every lane count (1350 B records 543-550 ->
// 637-644 GiB/s, 3000 B 712-719 -> 747-758, 16 KiB 954-967 -> 964-978; same
// boxes, profiles/r06/s19, s20).  (A/B: GCM_IOV_TLOAD=0, non-temporal.)
#ifndef GCM_IOV_TLOAD
#define GCM_IOV_TLOAD 1
#endif
// iovec block stores are temporal too (16 KiB 962 -> 1,002 GiB/s, 1350 B
// 643 -> 689, 3000 B 733 -> 770; same box, profiles/r06/s22).
#ifndef GCM_IOV_TSTORE
#define GCM_IOV_TSTORE 1
#endif
__device__ __forceinline__ void iov_store_blk(uint8_t *p, uint4 y) {
  if constexpr (GCM_IOV_TSTORE)
    store16_any(p, y);
  else
    store_blk_nt(p, y);
}
#ifndef GCM_TL_TSTORE
#define GCM_TL_TSTORE 0  // (A/B: temporal stores wherever the loads are temporal)
#endif
#ifndef GCM_TLOAD_ALL
#define GCM_TLOAD_ALL 0  // (A/B: temporal block loads at every lane count)
#endif

// TL: temporal record-block loads (non-IOV records; iovec records follow
// GCM_IOV_TLOAD).  The one-key kernel passes it at 4 lanes per record and at
// 16 (which it runs only for unaligned uniform batches, unaligned_uniform:
// 16 KiB records at the iovec layout's odd stride 1,092 -> 1,125 GiB/s, an
// unaligned block spans two lines and the neighbouring lane group wants the
// rest of each; profiles/r06/s21); the 8-lane aligned path keeps non-temporal
// loads (temporal: config 2 1,198 against 1,203-1,208, config 5 -0.8 %).
template <int NR, bool OPEN, bool XT, int L = 16, bool RP = false, bool IOV = false,
          bool TL = false>
__device__ __forceinline__ void process_records(const RoundKeys &rk, const BatchDesc &b,
                                                const UnitIn &in, const uint8_t *smem,
                                                const GcmKeyDev *key, uint32_t lc0, uint32_t lc1,
                                                int prio_base = 0) {
  static_assert(L == 16 || L == 8 || L == 4, "lanes per record");
  const int q = threadIdx.x & (L - 1);
  const uint64_t rec = in.rec;
  const bool active = in.active, live = in.live;
  const RecordMeta m = in.m;
  // J0 and the AD hash (gcm.cc.inc:298-398), in the record's lanes.
  uint4 j0 = make_uint4(0, 0, 0, 0);
  if (live) {
    if (b.nonce_len == 12)
      j0 = make_uint4(in.nonce.x, in.nonce.y, in.nonce.z, 0x01000000u);  // nonce || be32(1)
    else
      j0 = record_j0(b, rec, key->hpow_ct);
  }
  const bool many_ad = __ballot(live && m.ad_len > 16) != 0;
  const uint4 ya = many_ad ? record_ad_hash<L>(b, rec, m, live, true, key->hpow_ct) : in.ad0;
  // (< 2^32: the GCM length limit holds for a live record)
  const uint32_t nb = live ? (uint32_t)((m.len + m.xlen + 15) / 16) : 0u;
  const uint32_t ctr0 = bswap32(j0.w);
  // Extra bytes after the record (TLS 1.3 inner type, XT kernels): read from /
  // written to their own arrays by the byte path (BatchDesc::extra).
  const uint8_t *xin = XT ? batch_extra_in(b, rec) : nullptr;
  uint8_t *xout = XT ? batch_extra_out(b, rec) : nullptr;
  // Round 0 of the counter blocks: words 0..2 are constant per record.
  const uint32_t c0 = j0.x ^ rk.w[0][0], c1 = j0.y ^ rk.w[0][1], c2 = j0.z ^ rk.w[0][2];
  // E_K(J0), one column per lane of each quad (from the same bank-replicated
  // LDS tables; computed while the unit's first block is in flight).
  const uint32_t ek0w = ek0_quad<NR, 0>(c0, c1, c2, bswap32(ctr0) ^ rk.w[0][3], rk, smem, lc0, lc1);
  const uint8_t *src = b.in + m.off;
  uint8_t *dst = b.out + m.off;
  uint4 acc = (q == L - 1 && live) ? ya : make_uint4(0, 0, 0, 0);
  // GHASH lane constants (Gh8): rotation by gq bytes and the slot offsets.
  // gq = the lane's index in its 16-lane row whatever L is: the 16 lanes of a
  // ds_read_b128 lane group then always read 16 different slots (the
  // rotation only orders each lane's own 16 lookups).
  const int gq = threadIdx.x & 15;
  const bool rs1 = (gq >> 2) & 1, rs2 = (gq >> 3) & 1;  // (rotation by gq)
  const uint32_t rbs = (uint32_t)gq & 3u;
  uint32_t P[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) v |= (uint32_t)(((4 * k + i + gq) & 15) << 4) << (8 * i);
    P[k] = v;
  }
  // Counter-mode caching (Bernstein-Schwabe): within a 256-counter window only
  // byte 15 of the counter block changes, so round 1 needs one lookup (column
  // 0, row 3) and round 2 four; K0..K3 / L0..L3 hold the constant parts and
  // are recomputed when a lane's counter enters a new window.
  constexpr uint32_t T = 0;  // the table base (kLdsAes) rides in lc0/lc1
  const uint32_t k0 = tload<T>(smem, taddr<0>(lc0, c0)) ^ tload<T>(smem, taddr<1>(lc1, c1)) ^
                      rotl(tload<T>(smem, taddr<2>(lc0, c2)) ^ rk.w[1][0], 16);
  WindowCache wc;
  const int iters = group_max<L>((int)((nb + L - 1) / L));
  // Full 16-byte blocks of this lane's record, at any alignment (one
  // dwordx4 each, load_blk_nt); the partial last block takes the byte path.
  // (iovec records: their own paths below.)
  const uint32_t nfull = !IOV && live ? (uint32_t)(m.len / 16) : 0u;
  // iovec records (IOV): chunk cursors of the loads (one iteration ahead)
  // and of the stores.
  static_assert(!(IOV && XT), "iovec records carry no extra bytes");
  // Between chunk boundaries a lane carries only its run pointers: the next
  // block is 16·L bytes further on, and while it stays inside the chunk
  // (`*_left` >= 16) it is one dwordx4 at `*_ptr`.  Anything else (a chunk
  // boundary, the record's last block, the first block) takes the cursor
  // path: the chunk cursor (chunk index and its stream start; the rest is
  // reloaded from the chunk array) seeks, handles the block and re-anchors the
  // run.  (The compact state keeps the IOV kernel's hot loop free of spills.)
  uint64_t ld_c = 0, ld_cs = 0, st_c = 0, st_cs = 0;
  const uint8_t *ld_ptr = nullptr;
  uint8_t *st_ptr = nullptr;
  int32_t ld_left = -1, st_left = -1;
  // Store anchor handed over by the load cursor (kIovHandoff): when a load
  // walks the chunk table to a whole block inside one chunk, the output
  // address of that block (the output chunks have the input chunks' lengths)
  // and the bytes left in its chunk, tagged with the block index.  The store
  // of that block (one iteration later) then re-anchors its run without a
  // walk of its own: the walk's chunk-table loads, issued after the previous
  // stores and the next block's load, wait for all of them (vmcnt counts
  // loads and stores in issue order).
  uint8_t *ho_ptr = nullptr;
  int32_t ho_left = -1;
  uint32_t ho_j = 0xffffffffu;
  // End of the load cursor's chunk once walked (kIovKeepEnd; 0: not yet): a
  // load past it starts the walk at the next chunk, one dependent chunk-table
  // load instead of two.
  uint64_t ld_ce = 0;
  // The record's LDS slot (kIovLds, iov_dev.h IovDescL), the wave's own.
  constexpr uint32_t kc = kIovKc<L>;
  const uint8_t *const ls = smem + kLdsBytes + (uint32_t)(threadIdx.x / L) * kIovSlot<L>;
  if constexpr (IOV) {
    if (live) {
      ld_c = st_c = b.iovec_start[rec];
      if constexpr (kIovLds) iov_slot_fill<kc, L>(const_cast<uint8_t *>(ls), b, rec, ld_c, q);
      // (Seeding the running pointers here from the first chunk, so the first
      // load and store skip the cursor walk, measured neutral: 957-966 vs
      // 951-966 GiB/s, profiles/r04/s14/.)
    }
    if constexpr (kIovLds) iov_slot_sync();
  }
  // The walk's descriptor source and the record's chunk end.
  auto iov_src = [&](uint64_t &c_end) {
    if constexpr (kIovLds) {
      return iov_slot_src<kc>(ls, b, c_end);
    } else {
      c_end = b.iovec_start[rec + 1];
      return IovDescG{b.iovecs};
    }
  };
  // (Left undefined when not loaded: such a block is never stored or hashed
  // from this value, and a zero-fill would be a VALU write that the waitcnt
  // pass orders after the previous store.)
  auto load_full = [&](uint64_t j) {
    uint4 v;
    if constexpr (IOV) {
      if (ld_left >= 16) {
        v = GCM_IOV_TLOAD ? load16_any(ld_ptr) : load_blk_nt(ld_ptr);
        ld_ptr += 16 * L;
        ld_left -= 16 * L;
      } else {
        v = make_uint4(0, 0, 0, 0);
        const uint64_t p = j * 16;
        if (live && p < m.len) {  // (a dead record never walks the batch's chunks)
          uint64_t c_end;
          const auto d = iov_src(c_end);
          IovCur k;
          if (kIovKeepEnd && ld_ce && p >= ld_ce && ld_c + 1 < c_end)
            iov_at_d(k, d, ld_c + 1, ld_ce);
          else
            iov_at_d(k, d, ld_c, ld_cs);
          iov_seek_d(k, d, p, c_end);
          const uint32_t n = (uint32_t)umin64(m.len - p, 16);
          if (n == 16 && p + 16 <= k.ce) {
            v = GCM_IOV_TLOAD ? load16_any(k.in + (p - k.cs)) : load_blk_nt(k.in + (p - k.cs));
            if constexpr (kIovHandoff) {
              ho_ptr = k.out + (p - k.cs);
              ho_left = (int32_t)umin64(k.ce - p, 1u << 30);
              ho_j = (uint32_t)j;
            }
          } else if (!iov_load2_d(d, k, p, n, c_end, v))  // a straddle, the last block
            v = iov_gather_d(d, k, p, n, c_end);        // (three or more chunks)
          ld_c = k.c;
          ld_cs = k.cs;
          if constexpr (kIovKeepEnd) ld_ce = k.ce;
          ld_ptr = k.in + (p - k.cs) + 16 * L;
          ld_left = (int32_t)umin64(k.ce - p, 1u << 30) - 16 * L;
        }
      }
      return v;
    }
    if (j < nfull) {
      // (TL at L = 4 as the stores below: config G 850-883 -> 888-904
      // GiB/s, same box, profiles/r06/s17)
      if constexpr (TL || GCM_TLOAD_ALL)
        v = load16_any(src + (uint64_t)j * 16);
      else
        v = load_blk_nt(src + (uint64_t)j * 16);
    }
    return v;
  };
  // One iteration: block j = it*16 + q, plaintext (if full) already in x,
  // its AES state after the cached rounds 1-2 in `cur` (computed during the
  // previous iteration).  The GHASH multiply of the accumulator (acc * H^16,
  // its input known from the previous iteration) and rounds 1-2 of the next
  // block j + 16 are interleaved with this block's rounds 3..NR.
  uint32_t cur[4];
  {
    const uint32_t ctr = ctr0 + 1u + (uint32_t)q;  // block q
    const uint32_t s3 = bswap32(ctr) ^ rk.w[0][3];
    wc.update<T>(ctr, s3, c0, c1, c2, rk, smem, lc0, lc1);
    wc.rounds12<T>(k0, s3, cur[0], cur[1], cur[2], cur[3], smem, lc0, lc1);
  }
  auto step = [&](int it, uint4 x) {
    if constexpr (RP) {
      switch ((prio_base + it) & 3) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
      }
    }
    const uint32_t j = (uint32_t)it * L + q;
    const uint32_t ctrn = ctr0 + 1u + (uint32_t)(j + L);  // next block, inc32 mod 2^32
    uint32_t xs = bswap32(ctrn) ^ rk.w[0][3];
    wc.update<T>(ctrn, xs, c0, c1, c2, rk, smem, lc0, lc1);
    Gh8 h;
    g8_rotate(h, acc, rs1, rs2, rbs);
    h.g = make_uint4(0, 0, 0, 0);
    uint32_t sa[4] = {cur[0], cur[1], cur[2], cur[3]};
    rounds_s1<0, NR>(sa, rk, lc0, lc1, h, P, xs, wc, k0, cur);
    asm_last_s1(sa, rk.w[NR], lc0);
    const uint4 ks = make_uint4(sa[0], sa[1], sa[2], sa[3]);
    uint4 y = xor4(x, ks);
    if constexpr (IOV) {
      if (st_left >= 16) {
        iov_store_blk(st_ptr, y);
        st_ptr += 16 * L;
        st_left -= 16 * L;
      } else if (kIovHandoff && ho_j == j) {  // (j < nb: a whole block was loaded)
        iov_store_blk(ho_ptr, y);
        st_ptr = ho_ptr + 16 * L;
        st_left = ho_left - 16 * L;
      } else if (j < nb) {
        const uint64_t p = (uint64_t)j * 16;
        const uint32_t n = (uint32_t)umin64(m.len - p, 16);
        uint64_t c_end;
        const auto d = iov_src(c_end);
        IovCur k;
        iov_at_d(k, d, st_c, st_cs);
        iov_seek_d(k, d, p, c_end);
        if (n == 16 && p + 16 <= k.ce) {
          iov_store_blk(k.out + (p - k.cs), y);
        } else {
          y = mask_block(y, n);
          if (!iov_store2_d(d, k, p, y, n, c_end)) iov_scatter_d(d, k, p, y, n, c_end);
        }
        st_c = k.c;
        st_cs = k.cs;
        st_ptr = k.out + (p - k.cs) + 16 * L;
        st_left = (int32_t)umin64(k.ce - p, 1u << 30) - 16 * L;
      }
      if (j < nb) acc = xor4(h.g, OPEN ? x : y);
      return;
    }
    if (j < nfull) {
      // (L = 4: temporal stores, +2 % on config G's 64-byte runs, same box;
      // non-temporal ones for the longer runs of L = 8 / 16, profiles/r05/r5s19)
      if constexpr (L == 4 || (TL && GCM_TL_TSTORE))
        store_blk(dst + (uint64_t)j * 16, y);
      else
        store_blk_nt(dst + (uint64_t)j * 16, y);
    } else if (j < nb) {
      const uint32_t n = (uint32_t)umin64(m.len + m.xlen - (uint64_t)j * 16, 16);
      if constexpr (XT) {
        y = crypt_partial_x(src, dst, m.len, xin, xout, (uint64_t)j * 16, ks, n, x);
      } else {
        x = load_partial(src + (uint64_t)j * 16, n);
        y = mask_block(xor4(x, ks), n);
        store_partial(dst + (uint64_t)j * 16, y, n);
      }
    }
    if (j < nb) {
      acc = xor4(h.g, OPEN ? x : y);
    }
  };
  // Plaintext is loaded one iteration ahead into two alternating buffers (the
  // loop is unrolled twice so no register copy forces an early wait): the load
  // for iteration it+1 is issued before iteration it's store, so waiting for
  // it never waits for a store (vmcnt counts loads and stores in issue order)
  // and its latency hides under a whole iteration of AES + GHASH.
  uint4 x0;
  if constexpr (IOV)
    x0 = load_full(q);
  else
    x0 = in.x0;
  int it = 0;
  for (; it + 1 < iters; it += 2) {
    const uint4 x1 = load_full((uint64_t)(it + 1) * L + q);
    step(it, x0);
    x0 = load_full((uint64_t)(it + 2) * L + q);
    step(it + 1, x1);
  }
  if (it < iters) step(it, x0);
  finish_record<OPEN, L>(acc, nb, m, quad_gather(ek0w), b, rec, active, live, dst,
                         key->hpow_ct);
}

// The AES tables of the bulk kernels, replicated per bank: entry idx, slot t,
// lane l at kLdsAes + idx*256 + t*128 + l*4.  Slot 1 holds T1 = rotl8(T0).
template <int THREADS>
__device__ __forceinline__ void fill_aes_tables(uint8_t *smem, int tid) {
  for (int e = tid; e < 256 * 64; e += THREADS) {
    const int idx = e >> 6, slot = (e >> 5) & 1;
    const uint32_t v = kTables.te0[idx];
    reinterpret_cast<uint32_t *>(smem + kLdsAes)[e] = slot ? rotl(v, 8) : v;
  }
}

// One-key bulk kernel (the ctx API: configs 2, 4, G; no key_index).  One
// workgroup of W = 16 waves per CU (the LDS tables take 128 KiB; declared for
// 1024 threads so it compiles into 128 VGPRs).  Each wave takes the next unit
// of 64 / L records (in processing order) from a grid-wide counter, so waves
// that the SIMD arbiter favours (older waves issue first) simply process more
// units instead of waiting at a per-tile barrier for the slowest wave
// (DESIGN.md §4.2).  L: lanes per record -- 4 for uniform batches of records
// up to 4 KiB on 64-byte runs (runs_in_lines) and the short records of
// ragged and iovec batches, 8 (8 records per wave, GHASH stride H^8) for other
// one-key batches and iovec records of 2-4 KiB, 16 for iovec records of 4 KiB
// or more and unaligned uniform batches of long records (unaligned_uniform);
// the keyset kernel keeps 16.
// (A kernel of its own, apart from the keyset kernel, so each gets its own
// register allocation.)
template <int NR, bool OPEN, bool XT, int W, bool IOV = false, int L = 16>
__global__ __launch_bounds__(1024) void gcm_kernel(const GcmKeyDev *__restrict__ keys,
                                                    BatchDesc b, uint32_t *__restrict__ units) {
  constexpr int kThreads = W * 64;
  __shared__ __attribute__((aligned(16))) uint8_t smem[IOV ? kLdsIovBytes<L, kThreads> : kLdsBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const uint64_t n = b.num_records;
  // Processing positions of this launch (BatchDesc::split_lo/_hi); a launch
  // for an empty length class ends before building its tables.
  uint64_t lo = 0, hi = n;
  if (b.split_lo) lo = *b.split_lo;
  if (b.split_hi) hi = *b.split_hi;
  if (lo >= hi) return;
  fill_aes_tables<kThreads>(smem, tid);
  const uint32_t lc0 = kLdsAes + (uint32_t)(lane & 31) * 4u;
  const uint32_t lc1 = lc0 + 128u;
  if constexpr (L == 16)
    build_g8<kThreads>(smem, reinterpret_cast<const uint4 *>(keys[0].htab16), tid);
  else
    build_gpow<kThreads, kLdsBasis>(smem, keys[0].hpow_ct[L], tid);
  __syncthreads();
  RoundKeys rk;
#pragma unroll
  for (int r = 0; r <= NR; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) rk.w[r][c] = keys[0].rk[r][c];
  auto claim = [&]() {
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(units, 1u);
    return u;
  };
  for (;;) {
    const uint64_t first = lo + (uint64_t)__builtin_amdgcn_readlane(claim(), 0) * (64 / L);
    if (first >= hi) break;
    UnitIn in;
    unit_load<XT, IOV>(in, b, first + lane / L, lane & (L - 1), hi);
    process_records<NR, OPEN, XT, L, false, IOV, L == 4 || L == 16>(rk, b, in, smem, keys, lc0,
                                                                     lc1);
  }
}

// Keyset bulk kernel (key_index per record: BSSL_AMD_KEYSET, config 5): the
// records are visited in tiles of W * 4; a tile whose records use several
// keys is processed in one pass per distinct key, since the LDS byte table is
// per key.
// Tiles from a grid-wide counter (round 6: config 5 1,084-1,091 -> 1,110 GiB/s
// against the blockIdx-strided order, same box, profiles/r06/s5): a CU that
// finishes its tiles early takes the next one instead of idling at the end.
#ifndef GCM_KEYSET_DYN
#define GCM_KEYSET_DYN 1
#endif
#ifndef GCM_KEYSET_RP
#define GCM_KEYSET_RP 1  // (A/B: 0 = no per-iteration priority rotation)
#endif
template <int NR, bool OPEN, bool XT, int W>
__global__ __launch_bounds__(1024) void gcm_keyset_kernel(const GcmKeyDev *__restrict__ keys,
                                                           BatchDesc b, uint32_t *__restrict__ tiles) {
  constexpr int kThreads = W * 64;
  constexpr int kRecPerTile = W * kRecPerWave;
  static_assert(kRecPerTile <= 64, "one wave plans a tile with ballots");
  __shared__ __attribute__((aligned(16))) uint8_t smem[kLdsBytes];
  // Pass list of the current tile: key and 64-bit record mask per pass.
  uint32_t *s_pass_key = reinterpret_cast<uint32_t *>(smem + kLdsPlan);
  uint64_t *s_pass_mask = reinterpret_cast<uint64_t *>(smem + kLdsPlan + 64 * 4);
  int *s_npass = reinterpret_cast<int *>(smem + kLdsPlan + 64 * 16);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  fill_aes_tables<kThreads>(smem, tid);
  const uint32_t lc0 = kLdsAes + (uint32_t)(lane & 31) * 4u;
  const uint32_t lc1 = lc0 + 128u;
  uint32_t loaded = 0xffffffffu;
  const uint64_t n = b.num_records;
#if GCM_KEYSET_DYN  // (tiles from a grid-wide counter; 0: blockIdx order, round 5)
  uint64_t *s_tile = reinterpret_cast<uint64_t *>(smem + kLdsPlan + 64 * 16 + 8);
  for (uint64_t base = 0;;) {
    __syncthreads();
    if (tid == 0) *s_tile = (uint64_t)atomicAdd(tiles, 1u) * kRecPerTile;
    __syncthreads();
    base = *s_tile;
    if (base >= n) break;
#else
  for (uint64_t base = (uint64_t)blockIdx.x * kRecPerTile; base < n;
       base += (uint64_t)gridDim.x * kRecPerTile) {
#endif
    __syncthreads();
    if (wave == 0) {
      // Plan the tile: one pass per distinct key, in record order.
      const uint64_t i = base + lane;
      uint32_t k = (lane < kRecPerTile && i < n) ? (b.key_index ? b.key_index[rec_at(b, i)] : 0u)
                                                 : 0xffffffffu;
      if (k != 0xffffffffu && k >= b.num_keys) k = 0;  // flagged dead by the prologue
      uint64_t pending = __ballot(k != 0xffffffffu);
      int np = 0;
      while (pending) {
        const uint32_t kk = __shfl(k, __builtin_ctzll(pending), 64);
        const uint64_t mask = __ballot(k == kk) & pending;
        if (lane == 0) {
          s_pass_key[np] = kk;
          s_pass_mask[np] = mask;
        }
        pending &= ~mask;
        np++;
      }
      if (lane == 0) *s_npass = np;
    }
    __syncthreads();
    const int npass = *s_npass;
    for (int pi = 0; pi < npass; pi++) {
      const uint32_t k = __builtin_amdgcn_readfirstlane(s_pass_key[pi]);
      const uint64_t mask = s_pass_mask[pi];
      if (k != loaded) {
        __syncthreads();
        // Byte table of H^16 from the key's nibble tables (power 4): entry
        // (e, p) = T[2p][e >> 4] ^ T[2p+1][e & 15] (key_setup.cc layout).
        build_g8<kThreads>(smem, reinterpret_cast<const uint4 *>(keys[k].htab16), tid);
        __syncthreads();
        loaded = k;
      }
      RoundKeys rk;
#pragma unroll
      for (int r = 0; r <= NR; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) rk.w[r][c] = keys[k].rk[r][c];
      const int t = wave * kRecPerWave + g;
      const bool active = (mask >> t) & 1;
      UnitIn in;
      unit_load<XT, false>(in, b, active ? base + t : n, lane & 15, n);
      process_records<NR, OPEN, XT, 16, GCM_KEYSET_RP != 0>(rk, b, in, smem, keys + k, lc0, lc1,
                                                           wave >> 2);
      __builtin_amdgcn_s_setprio(0);
    }
  }
}

// ---------------------------------------------------------------------------
// One record: the host-buffer calls (EVP_AEAD_CTX_seal / open / seal_scatter,
// aead.cc.inc:163-209 -- SSLAEADContext::SealScatter makes them one record at
// a time, ssl/ssl_aead_ctx.cc:299-381) as one launch of one workgroup with no
// unit counter and no 128 KiB table build.  Thread t encrypts counter block t,
// every load in flight at once (the record may sit in mapped host memory);
// AES from T0 replicated per bank (32 KiB); GHASH by lanes 0..15 at stride 16.
// Two shapes (THREADS): records of up to 256 blocks (4 KiB) take 256 threads
// and the key's nibble table of H^16 copied to LDS (8 KiB; in each lookup the
// 16 lanes read the same nibble position, so a lane's bank quad is its nibble
// value's and equal values share an address -- conflict-free whatever the
// data); longer records take 1024 threads and the bulk kernels' lane-rotated
// byte table of H^16 (64 KiB, built while the record loads are in flight; 16
// lookups per GHASH step instead of 32): 16 KiB records 48 -> 39 us, while a
// 1350-byte record lost 0.5 us to the build (profiles/r04/s13/).  Open
// computes the tag first and writes the plaintext (or zeros) after the check.
constexpr int kOneMaxBlocks = 1024;  // 16 KiB: threads per workgroup

// acc * H^16 from the lane-rotated byte table (g8_rotate / g8_load, as the
// bulk kernels' GHASH: the 16 lanes of a ds_read_b128 lane group read 16
// different slots in every step, whatever the data).
__device__ __forceinline__ uint4 g8_mul16(uint4 acc, bool rs1, bool rs2, uint32_t rbs,
                                          const uint32_t (&P)[4], const uint8_t *g8) {
  Gh8 h;
  g8_rotate(h, acc, rs1, rs2, rbs);
  uint4 r = xor4_3(g8_load<0>(h, P, g8), g8_load<1>(h, P, g8), g8_load<2>(h, P, g8));
  r = xor4_3(r, g8_load<3>(h, P, g8), g8_load<4>(h, P, g8));
  r = xor4_3(r, g8_load<5>(h, P, g8), g8_load<6>(h, P, g8));
  r = xor4_3(r, g8_load<7>(h, P, g8), g8_load<8>(h, P, g8));
  r = xor4_3(r, g8_load<9>(h, P, g8), g8_load<10>(h, P, g8));
  r = xor4_3(r, g8_load<11>(h, P, g8), g8_load<12>(h, P, g8));
  r = xor4_3(r, g8_load<13>(h, P, g8), g8_load<14>(h, P, g8));
  return xor4(r, g8_load<15>(h, P, g8));
}

// x * H^16 from the nibble table (key_setup.cc layout: position 2k = the high
// nibble of byte k, 2k + 1 the low one).
__device__ __forceinline__ uint4 nib_mul16(uint4 x, const uint4 *htab) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  uint4 r = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t byte = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    r = xor4_3(r, htab[(2 * k) * 16 + (byte >> 4)], htab[(2 * k + 1) * 16 + (byte & 15u)]);
  }
  return r;
}

template <int NR, bool OPEN, int THREADS>
__global__ __launch_bounds__(THREADS) void gcm_one_kernel(const GcmKeyDev *__restrict__ keys,
                                                          BatchDesc b) {
  constexpr bool kByte = THREADS == kOneMaxBlocks;  // byte table (else the nibble table)
  __shared__ __attribute__((aligned(16))) uint8_t g8[kByte ? kG8Bytes : 16];
  __shared__ uint4 htab[kByte ? 1 : 32 * 16];
  __shared__ uint32_t t0tab[256 * 32];
  __shared__ uint4 cblk[THREADS];
  __shared__ uint4 s_lh;  // len block x H ^ E_K(J0), from wave 1
  __shared__ uint32_t s_ok;
  const int t = threadIdx.x;
  const GcmKeyDev *key = keys;
  const RecordMeta m = record_meta(b, 0);
  const bool live = record_live(b, 0, m);
  const uint8_t *src = b.in + m.off;
  uint8_t *dst = b.out + m.off;
  // The tables' loads first (device memory), then every load of the record
  // (it may sit in mapped host memory, one PCIe round trip each), together:
  // this thread's block, for open the received tag.  The nonce and a short AD
  // come by value from the single-record host path (BatchDesc::inl), and the
  // barrier below orders only the LDS writes, so the rounds run while the
  // record is in flight (vmcnt counts in issue order: the tables' loads, issued
  // first, complete without waiting for the record's).
  const uint32_t nbytes = (uint32_t)m.len;  // (<= 16 KiB: the launcher checks)
  const uint32_t nb = (nbytes + 15) / 16;
  const uint32_t n = (uint32_t)t < nb ? min(nbytes - 16u * t, 16u) : 0u;
  for (int e = t; e < 256 * 32; e += THREADS) t0tab[e] = kTables.te0[e >> 5];
  if constexpr (kByte)
    build_g8<THREADS>(g8, reinterpret_cast<const uint4 *>(key->htab16), t);
  else
    for (int e = t; e < 32 * 16; e += THREADS) htab[e] = reinterpret_cast<const uint4 *>(key->htab16)[e];
  uint4 ad0 = make_uint4(0, 0, 0, 0), nonce = make_uint4(0, 0, 0, 0), tr = ad0;
  if (b.inl & 1)
    nonce = make_uint4(b.inl_nonce[0], b.inl_nonce[1], b.inl_nonce[2], 0);
  else if (live && b.nonce_len == 12)
    nonce = load_partial(b.nonces, 12);  // (every thread's J0)
  if (b.inl & 2)
    ad0 = make_uint4(b.inl_ad[0], b.inl_ad[1], b.inl_ad[2], b.inl_ad[3]);
  else if (t < 64 && live && m.ad_len)
    ad0 = ad_block(b, 0, m, 0);
  __builtin_amdgcn_sched_barrier(0);
  uint4 x = make_uint4(0, 0, 0, 0);
  if (n == 16)
    x = load16_any(src + 16 * t);
  else if (n)
    x = load_partial(src + 16 * t, n);
  if (OPEN && t == 0 && live) tr = load_partial(batch_tag(b, 0), b.tag_len);  // the received tag
  RoundKeys rk;
#pragma unroll
  for (int r = 0; r <= NR; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) rk.w[r][c] = key->rk[r][c];
  const uint4 j0 = !live ? make_uint4(0, 0, 0, 0)
                   : b.nonce_len == 12 ? make_uint4(nonce.x, nonce.y, nonce.z, 0x01000000u)
                                       : record_j0(b, 0, key->hpow_ct);
  const uint32_t ctr0 = bswap32(j0.w);
  // Barrier over the LDS tables only (no wait for the record's loads).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  // (Only threads with a block run the rounds: the waves past the record's
  // end issue no LDS lookups -- for a 1350-byte record 2 of the 16 waves.)
  uint4 y = make_uint4(0, 0, 0, 0);
  if (n) {
    const uint4 ks = aes_block_rep<NR>(
        make_uint4(j0.x, j0.y, j0.z, bswap32(ctr0 + 1u + (uint32_t)t)), rk, t0tab);
    y = mask_block(xor4(x, ks), n);
    if (!OPEN) {  // seal: the ciphertext (zeros for a dead record, aead.cc.inc:170-179)
      if (n == 16)
        store16_any(dst + 16 * t, live ? y : make_uint4(0, 0, 0, 0));
      else
        store_partial(dst + 16 * t, live ? y : make_uint4(0, 0, 0, 0), n);
    }
    cblk[t] = OPEN ? x : y;  // the GHASH input is the ciphertext
  }
  uint4 ya = make_uint4(0, 0, 0, 0);
  if (t < 64) ya = m.ad_len > 16 ? record_ad_hash<16>(b, 0, m, live, true, key->hpow_ct) : ad0;
  __syncthreads();
  if (t >= 64 && t < 128) {
    // Wave 1, during wave 0's GHASH: the tag's record-independent part, len
    // block x H ^ E_K(J0) (gcm.cc.inc:576-604, 340-343).
    Gf128 lb = {{(uint32_t)(m.len << 3), (uint32_t)(m.len >> 29), (uint32_t)(m.ad_len << 3),
                 (uint32_t)(m.ad_len >> 29)}};
    const uint4 lh = xor4(from_gf(gf_mul(lb, gf_load(key->hpow_ct[1]))),
                          aes_block_rep<NR>(j0, rk, t0tab));
    if (t == 64) s_lh = lh;
  }
  uint4 zs = make_uint4(0, 0, 0, 0);
  if (t < 16) {
    const int q = t;
    uint4 acc = (q == 15 && live) ? ya : make_uint4(0, 0, 0, 0);
    const bool rs1 = (q >> 2) & 1, rs2 = (q >> 3) & 1;  // (lane constants of process_records)
    const uint32_t rbs = (uint32_t)q & 3u;
    uint32_t P[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t v = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) v |= (uint32_t)(((4 * k + i + q) & 15) << 4) << (8 * i);
      P[k] = v;
    }
    const uint32_t iters = live ? (nb + 15) / 16 : 0u;
    for (uint32_t it = 0; it < iters; it++) {
      const uint32_t j = 16 * it + q;
      uint4 h;
      if constexpr (kByte)
        h = g8_mul16(acc, rs1, rs2, rbs, P, g8);
      else
        h = nib_mul16(acc, htab);
      if (j < nb) acc = xor4(h, cblk[j]);
    }
    // Record end (finish_record's algebra) with the tag's last x H folded into
    // the lane weights: tag = sum_q acc_q H^(17-p) ^ len x H ^ E_K(J0).
    const int r = (int)((nb + 1) & 15);
    const int p = (q - r + 1) & 15;
    Gf128 z = gf_mul(to_gf(acc), gf_load(key->hpow_ct[17 - p]));
#pragma unroll
    for (int i = 0; i < 4; i++) z.w[i] = row_xor16(z.w[i]);
    zs = from_gf(z);
  }
  __syncthreads();  // (s_lh)
  if (t == 0) {
    const uint4 tag = xor4(zs, s_lh);
    int ok = live;
    if (OPEN && live) {  // CRYPTO_memcmp (e_aes.cc.inc:860-864)
      const uint4 mine = mask_block(tag, b.tag_len);
      ok = ((tr.x ^ mine.x) | (tr.y ^ mine.y) | (tr.z ^ mine.z) | (tr.w ^ mine.w)) == 0;
    }
    if (!OPEN) store_partial(batch_tag(b, 0), ok ? tag : make_uint4(0, 0, 0, 0), b.tag_len);
    if (b.status) b.status[0] = ok ? 1 : 0;
    s_ok = (uint32_t)ok;
  }
  if (OPEN) {
    __syncthreads();
    if (n) {  // the plaintext, or zeros after a failed check (aead.cc.inc:539-547)
      const uint4 o = s_ok ? y : make_uint4(0, 0, 0, 0);
      if (n == 16)
        store16_any(dst + 16 * t, o);
      else
        store_partial(dst + 16 * t, o, n);
    }
  }
  if (b.done) {  // completion word (aead_api.cc wait_record): after every store
    // Every thread waits for its own stores; one system-scope release then
    // covers them all (a fence in every wave cost ~4 us here: 16 L2 writebacks).
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0) {
      __threadfence_system();
      __builtin_amdgcn_s_waitcnt(0);  // (the L2 write-back has finished)
      *reinterpret_cast<volatile uint32_t *>(b.done) = b.done_seq;
    }
  }
}

// Batches the one-record kernel takes: one record of at most 16 KiB, one key,
// contiguous, no extra bytes.
bool one_record_batch(const BatchDesc &b) {
  if (b.num_records != 1 || b.key_index || b.iovecs || b.extra_len) return false;
  const uint64_t len = b.lengths ? ~uint64_t(0) : b.record_len;  // (arrays: device-resident)
  return len <= 16u * kOneMaxBlocks;
}

// Lanes per record of the one-key kernel: 4 (stride H^4, 16 records per
// wave) for uniform batches of records up to 4 KiB -- config G (1350 bytes)
// 760-766 GiB/s at 8 lanes, 889-893 at 4, same box (profiles/r04/s19/): a
// record's start and end are spread over twice the blocks per lane; 8 (stride
// H^8) for other batches; 16 for iovec records and for uniform batches of
// records of 4 KiB or more that are not 16-byte aligned, where a lane group's 16 L-byte
// run costs an extra cache line per run -- relatively twice as much at L = 8.
// 16 KiB records at a 16,385-byte stride: 823 GiB/s at L = 8, 1,076 at L = 16
// (aligned: 1,146-1,177); 1350-byte records at a 1351-byte stride: 755 at
// L = 8, 422 at L = 16, where the per-record work dominates; iovec records of
// 16 KiB 784 / 961 (profiles/r04/s10/, s11/).
bool unaligned_uniform(const BatchDesc &b) {
  return !b.offsets && b.record_len >= 4096 &&
         ((reinterpret_cast<uintptr_t>(b.in) | reinterpret_cast<uintptr_t>(b.out) |
           b.record_stride) & 15) != 0;
}

// 4 lanes per record only when every record starts a 64-byte run (each
// group's 64-byte run then stays in one 128-byte line): 1M x 1350-byte records
// at a 1360-byte stride 646-659 GiB/s at 4 lanes against 757-761 at 8, and
// 4000-byte records 786-804 against 986-993 (profiles/r04/s24/); at a
// 1408-byte stride (config G) 4 lanes are the faster.
bool runs_in_lines(const BatchDesc &b) {
  return ((reinterpret_cast<uintptr_t>(b.in) | reinterpret_cast<uintptr_t>(b.out) |
           b.record_stride) & 63) == 0;
}

// Lanes per record of the iovec length classes of 4 KiB or more and below
// 2 KiB (the class between takes 8).  Round 5 (profiles/r05/r5s25): 8 lanes
// for the long class 817 against 911-932 GiB/s (16 KiB records in three
// chunks), 8 for the short class 474 against 505 (1350 B).
#ifndef GCM_IOV_LONG_L
#define GCM_IOV_LONG_L 16
#endif
#ifndef GCM_IOV_SHORT_L
#define GCM_IOV_SHORT_L 4
#endif
constexpr int kIovLongL = GCM_IOV_LONG_L, kIovShortL = GCM_IOV_SHORT_L;
#ifndef GCM_ONEKEY_L
#define GCM_ONEKEY_L 8  // (A/B: lanes per record of aligned one-key batches)
#endif

template <int NR, bool OPEN>
int launch_nr(const GcmKeyDev *keys, const BatchDesc &b, hipStream_t s, const KernelEvents *ev) {
  if (one_record_batch(b)) {
    if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
    if (b.record_len <= 16 * 256)
      hipLaunchKernelGGL((gcm_one_kernel<NR, OPEN, 256>), dim3(1), dim3(256), 0, s, keys, b);
    else
      hipLaunchKernelGGL((gcm_one_kernel<NR, OPEN, kOneMaxBlocks>), dim3(1), dim3(kOneMaxBlocks), 0,
                         s, keys, b);
    const int rc = (int)hipGetLastError();
    if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
    return rc;
  }
  const int num_cus = device_cu_count();
  if (!num_cus) return 1;
  // The unit counters of the one-key kernels (64 bytes each, zeroed).
  uint32_t *units = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&units), 64, s) != hipSuccess) return 2;
  if (hipMemsetAsync(units, 0, 64, s) != hipSuccess) {
    hipFreeAsync(units, s);
    return 2;
  }
  BatchDesc bo = b;  // with the processing order of a ragged batch
  uint32_t *order = nullptr;
  if (wants_length_order(b)) {
    if (hipMallocAsync(reinterpret_cast<void **>(&order), (b.num_records + 128) * sizeof(uint32_t),
                       s) != hipSuccess) {
      hipFreeAsync(units, s);
      return 2;
    }
    const int orc = build_length_order(b.lengths, b.num_records, order, order + b.num_records, s);
    if (orc) {
      hipFreeAsync(order, s);
      hipFreeAsync(units, s);
      return orc;
    }
    bo.order = order;
  }
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
  {
    const uint64_t tiles = (b.num_records + kWaves * kRecPerWave - 1) / (kWaves * kRecPerWave);
    const unsigned grid = (unsigned)(tiles < (uint64_t)num_cus ? tiles : (uint64_t)num_cus);
    if (b.key_index) {
      if (b.extra_len)
        hipLaunchKernelGGL((gcm_keyset_kernel<NR, OPEN, true, kWaves>), dim3(grid),
                           dim3(kWaves * 64), 0, s, keys, bo, units + 12);
      else
        hipLaunchKernelGGL((gcm_keyset_kernel<NR, OPEN, false, kWaves>), dim3(grid),
                           dim3(kWaves * 64), 0, s, keys, bo, units + 12);
    } else if (b.iovecs && order) {  // (one key: the ctx API)
      // iovec records in length order (their totals are `lengths`): 16 lanes
      // for the records of 4 KiB or more, 8 from 2 KiB, 4 below (1M x 1350 B
      // in three chunks 370 -> 520 GiB/s, 512K x 3000 B 534 -> 680 against
      // 4 lanes for both; profiles/r04/s24/, s26/).  A launch whose class is
      // empty ends at once (gcm_kernel).
      BatchDesc bl = bo, bm = bo, bs = bo;
      bl.split_hi = bm.split_lo = order + b.num_records + kSplitWord;
      bm.split_hi = bs.split_lo = order + b.num_records + kSplitWord2k;
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, true, kIovLongL>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bl, units);
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, true, 8>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bm, units + 4);
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, true, kIovShortL>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bs, units + 8);
    } else if (b.iovecs) {
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, true, 16>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bo, units);
    } else if (b.extra_len) {
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, true, kWaves, false, 8>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bo, units);
    } else if (unaligned_uniform(b)) {
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, false, 16>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bo, units);
    } else if (!b.lengths && b.record_len <= 4096 && runs_in_lines(b)) {
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, false, 4>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bo, units);
    } else if (order) {
      // A ragged batch in length order: the records of 4 KiB or more at 8
      // lanes, then the shorter ones at 4 (each launch with its own counter).
      BatchDesc bl = bo, bs = bo;
      bl.split_hi = bs.split_lo = order + b.num_records + kSplitWord;
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, false, 8>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bl, units);
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, false, 4>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bs, units + 8);
    } else {
      hipLaunchKernelGGL((gcm_kernel<NR, OPEN, false, kWaves, false, GCM_ONEKEY_L>), dim3(grid),
                         dim3(kWaves * 64), 0, s, keys, bo, units);
    }
  }
  int rc = (int)hipGetLastError();
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
  if (order) hipFreeAsync(order, s);
  hipFreeAsync(units, s);
  return rc;
}

}  // namespace

#ifndef BSSL_AMD_MIX_TU  // (gcm_mix.hip includes this file for process_records)
namespace {
std::atomic<int> g_gcm_engine{-1};
std::atomic<int> g_gcm_mix_nb{4};
}  // namespace

int gcm_mix_waves() { return g_gcm_mix_nb.load(std::memory_order_relaxed); }

int gcm_engine() {
  int e = g_gcm_engine.load(std::memory_order_relaxed);
  if (e >= 0) return e;
  const char *v = getenv("BSSL_AMD_GCM_MODE");
  e = v && (!strcmp(v, "bs") || !strcmp(v, "bs16")) ? kGcmEngineBitsliced : kGcmEngineTable;
  if (v && !strncmp(v, "mix", 3)) {  // (experimental mixed engine, gcm_mix.hip: mix2|mix4|mix6)
    e = kGcmEngineMix;
    g_gcm_mix_nb.store(v[3] == '2' ? 2 : v[3] == '6' ? 6 : 4, std::memory_order_relaxed);
  }
  int expect = -1;
  g_gcm_engine.compare_exchange_strong(expect, e, std::memory_order_relaxed);
  return g_gcm_engine.load(std::memory_order_relaxed);
}

int set_gcm_engine(int engine) {
  if (engine != kGcmEngineTable && engine != kGcmEngineBitsliced) return -1;
  const int prev = gcm_engine();
  g_gcm_engine.store(engine, std::memory_order_relaxed);
  return prev;
}

int set_gcm_mix(int nb) {
  if (nb != 2 && nb != 4 && nb != 6) return -1;
  const int prev = gcm_engine();
  g_gcm_mix_nb.store(nb, std::memory_order_relaxed);
  g_gcm_engine.store(kGcmEngineMix, std::memory_order_relaxed);
  return prev;
}

bool gcm_takes_one_record_kernel(const BatchDesc &b, int engine) {
  return engine != kGcmEngineBitsliced && one_record_batch(b);
}

int launch_gcm(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr, void *stream,
               const KernelEvents *ev, int engine) {
  if (b.num_records == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (engine == kGcmEngineBitsliced) return launch_gcm_bs(keys, b, open, nr, s, ev);
  if (engine == kGcmEngineMix && gcm_mix_eligible(b, nr))
    return launch_gcm_mix(keys, b, open, gcm_mix_waves(), s, ev);
  switch (nr) {
    case 10: return open ? launch_nr<10, true>(keys, b, s, ev) : launch_nr<10, false>(keys, b, s, ev);
    case 12: return open ? launch_nr<12, true>(keys, b, s, ev) : launch_nr<12, false>(keys, b, s, ev);
    case 14: return open ? launch_nr<14, true>(keys, b, s, ev) : launch_nr<14, false>(keys, b, s, ev);
    default: return 1;
  }
}
#endif  // BSSL_AMD_MIX_TU

}  // namespace bssl_amd
