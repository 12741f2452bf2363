// bs_aes.h -- bitsliced AES on 32 blocks per lane (gfx950 VALU).
//
// State layout: p[i][b] is bit b (0 = LSB) of state byte i (FIPS-197 byte
// order, byte i = row i%4 of column i/4) for 32 blocks, block n in bit n.
// SubBytes is the Boyar-Peralta circuit (bs_sbox.inc, generated and checked
// exhaustively by tools/sbox/); ShiftRows is a renaming of byte indices;
// MixColumns and AddRoundKey are XOR networks whose key bits are wave-uniform
// masks (0 or ~0) derived from the round-key words in SGPRs.  hipcc folds the
// 2-input logic into 3-input v_bitop3_b32 on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bssl_amd {

#include "bs_sbox.inc"

// Round-key mask of byte i, bit b: 0 or 0xffffffff (wave-uniform).
__device__ __forceinline__ uint32_t bs_kmask(const uint32_t w[4], int i, int b) {
  return 0u - ((w[i >> 2] >> (8 * (i & 3) + b)) & 1u);
}

__device__ __forceinline__ uint32_t bs_xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// out_r = 2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3} ^ k_r for one column whose
// byte planes are a[r][b], written as xtime(u_r) ^ v_r with
// u_r = a_r ^ a_{r+1}, v_r = t ^ a_r ^ k_r and t = a0 ^ a1 ^ a2 ^ a3;
// xtime on planes: bit0 = u7, bit1 = u0^u7, bit2 = u1, bit3 = u2^u7,
// bit4 = u3^u7, bit5..7 = u4..u6.  20 ops per row + 16 for t (v_bitop3).
__device__ __forceinline__ void bs_mix_column(const uint32_t a[4][8], uint32_t o[4][8],
                                              const uint32_t w[4], int col) {
  uint32_t t[8];
#pragma unroll
  for (int b = 0; b < 8; b++) t[b] = bs_xor3(a[0][b], a[1][b], a[2][b]) ^ a[3][b];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t *x = a[r], *y = a[(r + 1) & 3];
    uint32_t v[8];
#pragma unroll
    for (int b = 0; b < 8; b++) v[b] = bs_xor3(t[b], x[b], bs_kmask(w, 4 * col + r, b));
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

// One middle round: SubBytes, ShiftRows, MixColumns, AddRoundKey(w).
// ShiftRows reads across columns, so results go to a second buffer; with
// every index a compile-time constant the copy back is register renaming.
__device__ __forceinline__ void bs_round(uint32_t p[16][8], const uint32_t w[4]) {
  uint32_t np[16][8];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    uint32_t a[4][8], o[4][8];
#pragma unroll
    for (int r = 0; r < 4; r++) sbox_planes(p[r + 4 * ((c + r) & 3)], a[r]);
    bs_mix_column(a, o, w, c);
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int b = 0; b < 8; b++) np[4 * c + r][b] = o[r][b];
  }
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) p[i][b] = np[i][b];
}

// Last round (SubBytes, ShiftRows, AddRoundKey(w)) of output column c only,
// as the 32 planes of output word c: o[8 * r + b] = bit b of row r.
__device__ __forceinline__ void bs_last_round_col(const uint32_t p[16][8], const uint32_t w[4],
                                                  int c, uint32_t o[32]) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uint32_t a[8];
    sbox_planes(p[r + 4 * ((c + r) & 3)], a);
#pragma unroll
    for (int b = 0; b < 8; b++) o[8 * r + b] = a[b] ^ bs_kmask(w, 4 * c + r, b);
  }
}

// One swap-move stage of the transpose: exchange bits >= S (within each
// 2S-bit group) of row k with bits < S of row k+S, for rows k with bit S clear.
template <int S>
__device__ __forceinline__ void bs_transpose_stage(uint32_t m[32]) {
  constexpr uint32_t kMask = S == 16 ? 0x0000ffffu : S == 8 ? 0x00ff00ffu
                           : S == 4 ? 0x0f0f0f0fu : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    if (k & S) continue;
    const uint32_t a = m[k], b = m[k + S];
    const uint32_t t = ((a >> S) ^ b) & kMask;
    m[k] = a ^ (t << S);
    m[k + S] = b ^ t;
  }
}

// 32x32 bit-matrix transpose in place: bit n of m[k] <-> bit k of m[n].
__device__ __forceinline__ void bs_transpose32(uint32_t m[32]) {
  bs_transpose_stage<16>(m);
  bs_transpose_stage<8>(m);
  bs_transpose_stage<4>(m);
  bs_transpose_stage<2>(m);
  bs_transpose_stage<1>(m);
}

}  // namespace bssl_amd
