// bs16_aes.h -- bitsliced AES on 16 blocks per lane, two state columns per
// register (gfx950 VALU).  Register (r, h, b) holds bit b of state row r for
// column h in its low 16 bits (block n in bit n) and for column h + 2 in its
// high 16 bits (block n in bit 16 + n): 64 VGPRs of state, and every SubBytes
// / MixColumns operation still works on 32 bit-slots.  See gcm.hip
// (process_records_bs16, gcm_prologue_bs16) and DESIGN.md §4.2b.
#pragma once
#include "bs_aes.h"

namespace bssl_amd {

__device__ __forceinline__ uint32_t swap16(uint32_t v) {
  return __builtin_amdgcn_perm(v, v, 0x01000302u);
}

// Round-key mask of register (r, h, b): bit b of row r of round-key columns h
// (low half) and h + 2 (high half), spread to 0 / 0xffff per half.
__device__ __forceinline__ uint32_t bs16_kmask(const uint32_t w[4], int r, int h, int b) {
  const uint32_t lo = (w[h] >> (8 * r + b)) & 1u, hi = (w[h + 2] >> (8 * r + b)) & 1u;
  return (lo | (hi << 16)) * 0xffffu;
}

// MixColumns + AddRoundKey of column pair h (bs_mix_column's network).
// km[r][b]: the round key's masks of this pair (bs16_kmask).
__device__ __forceinline__ void bs16_mix(const uint32_t a[4][8], uint32_t o[4][8],
                                         const uint32_t km[4][8]) {
  uint32_t t[8];
#pragma unroll
  for (int b = 0; b < 8; b++) t[b] = bs_xor3(a[0][b], a[1][b], a[2][b]) ^ a[3][b];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t *x = a[r], *y = a[(r + 1) & 3];
    uint32_t v[8];
#pragma unroll
    for (int b = 0; b < 8; b++) v[b] = bs_xor3(t[b], x[b], km[r][b]);
    const uint32_t u7 = x[7] ^ y[7];
    o[r][0] = u7 ^ v[0];
    o[r][1] = bs_xor3(x[0], y[0], u7) ^ v[1];
    o[r][2] = bs_xor3(x[1], y[1], v[2]);
    o[r][3] = bs_xor3(x[2], y[2], u7) ^ v[3];
    o[r][4] = bs_xor3(x[3], y[3], u7) ^ v[4];
    o[r][5] = bs_xor3(x[4], y[4], v[5]);
    o[r][6] = bs_xor3(x[5], y[5], v[6]);
    o[r][7] = bs_xor3(x[6], y[6], v[7]);
  }
}

// AES rounds 1..NR on the 16-block register pairs (round 0 is in p already).
// Row r of new pair h comes from old pair (h + r) & 1, half-swapped when
// ((h + r) >> 1) & 1 (ShiftRows on the column pairs {h, h + 2}).
// Round keys: the FIPS-197 words of round rd, wave-uniform (UNIFORM: spread
// into the per-register masks on the scalar unit; a per-key table of the 64
// masks per round, read by scalar loads, measured the same) or per lane (the
// prologue's E_K(J0) of keyset records: masks on the VALU).
template <int NR, bool UNIFORM = true>
__device__ __forceinline__ void bs16_cipher(uint32_t (&p)[4][2][8],
                                            const uint32_t *__restrict__ rkp) {
#pragma unroll 1
  for (int rd = 1; rd <= NR; rd++) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
      w[i] = UNIFORM ? (uint32_t)__builtin_amdgcn_readfirstlane(rkp[4 * rd + i]) : rkp[4 * rd + i];
    auto kmask = [&](int r, int h, int b) { return bs16_kmask(w, r, h, b); };
    const bool last = rd == NR;
    uint32_t np[4][2][8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t a[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        sbox_planes(p[r][(h + r) & 1], a[r]);
        if (((h + r) >> 1) & 1) {
#pragma unroll
          for (int b = 0; b < 8; b++) a[r][b] = swap16(a[r][b]);
        }
      }
      if (!last) {
        uint32_t km[4][8], o[4][8];
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) km[r][b] = kmask(r, h, b);
        bs16_mix(a, o, km);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = o[r][b];
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = a[r][b] ^ kmask(r, h, b);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int b = 0; b < 8; b++) p[r][h][b] = np[r][h][b];
  }
}

// One round (SubBytes, ShiftRows, MixColumns unless LAST, AddRoundKey) with
// the AddRoundKey masks of the key's precomputed table (GcmKeyDev::bsmask:
// 64 words per round, mask of register (r, h, b) at 32*h + 8*r + b; `m` is
// wave-uniform, so the masks arrive by scalar loads).  C1: the SubBytes
// outputs of the pair-0 groups (r, 0) are supplied in c1 instead of computed
// (round 1 of counter blocks, where those groups hold J0 words 0 and 2,
// the same in every slot: counter-mode caching).
template <bool LAST, bool C1>
__device__ __forceinline__ void bs16_round_tab(uint32_t (&p)[4][2][8],
                                               const uint32_t *__restrict__ m,
                                               const uint32_t (*c1)[8]) {
  uint32_t np[4][2][8];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t a[4][8];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (C1 && ((h + r) & 1) == 0) {
#pragma unroll
        for (int b = 0; b < 8; b++) a[r][b] = c1[r][b];
      } else {
        sbox_planes(p[r][(h + r) & 1], a[r]);
      }
      if (((h + r) >> 1) & 1) {
#pragma unroll
        for (int b = 0; b < 8; b++) a[r][b] = swap16(a[r][b]);
      }
    }
    if (!LAST) {
      uint32_t km[4][8], o[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 8; b++) km[r][b] = m[32 * h + 8 * r + b];
      bs16_mix(a, o, km);
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 8; b++) np[r][h][b] = o[r][b];
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 8; b++) np[r][h][b] = a[r][b] ^ m[32 * h + 8 * r + b];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int b = 0; b < 8; b++) p[r][h][b] = np[r][h][b];
}

// Rounds 1..NR with the key's AddRoundKey mask table (bs16_round_tab).
// Rounds R0..NR with the key's AddRoundKey mask table: one loop whose body
// branches to the last round's form inside (peeling the last round out, or
// branching around whole rounds, measured spills in the loop: the register
// allocator handles the loop-carried state better this way).
// `hook(rd)` runs at the start of round rd (between rounds, where only the
// state is live: e.g. a prefetch of the chunk's record bytes).
struct BsNoHook {
  __device__ void operator()(int) const {}
};

template <int NR, int R0 = 1, class Hook = BsNoHook>
__device__ __forceinline__ void bs16_rounds_tab(uint32_t (&p)[4][2][8],
                                                const uint32_t *__restrict__ mk,
                                                const Hook &hook = Hook()) {
#pragma unroll 1
  for (int rd = R0; rd <= NR; rd++) {
    hook(rd);
    const uint32_t *__restrict__ m = mk + 64 * rd;
    const bool last = rd == NR;
    uint32_t np[4][2][8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t a[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        sbox_planes(p[r][(h + r) & 1], a[r]);
        if (((h + r) >> 1) & 1) {
#pragma unroll
          for (int b = 0; b < 8; b++) a[r][b] = swap16(a[r][b]);
        }
      }
      if (!last) {
        uint32_t km[4][8], o[4][8];
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) km[r][b] = m[32 * h + 8 * r + b];
        bs16_mix(a, o, km);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = o[r][b];
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = a[r][b] ^ m[32 * h + 8 * r + b];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int b = 0; b < 8; b++) p[r][h][b] = np[r][h][b];
  }
}

template <int NR>
__device__ __forceinline__ void bs16_cipher_tab(uint32_t (&p)[4][2][8],
                                                const uint32_t *__restrict__ mk) {
  bs16_rounds_tab<NR, 1>(p, mk);
}

// The same for counter blocks whose pair-0 groups are the same in every slot
// (columns 0 and 2 of J0 ^ rk0): their round-1 SubBytes outputs come in c1
// (computed once per record), and p's pair 0 is not read.
template <int NR, class Hook = BsNoHook>
__device__ __forceinline__ void bs16_cipher_ctr(uint32_t (&p)[4][2][8], const uint32_t (&c1)[4][8],
                                                const uint32_t *__restrict__ mk,
                                                const Hook &hook = Hook()) {
  bs16_round_tab<false, true>(p, mk + 64, c1);
  bs16_rounds_tab<NR, 2>(p, mk, hook);
}

}  // namespace bssl_amd
