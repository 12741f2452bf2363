// key_sched.h -- the per-key AES-GCM tables (GcmKeyDev, internal.h), one
// implementation for the host (EVP_AEAD_CTX_init of one key, key_setup.cc)
// and the device (keysets: one lane per key, gcm_key_setup_kernel).  The
// analogue of the reference's CRYPTO_gcm128_init_aes_key
// (crypto/fipsmodule/aes/gcm.cc.inc:253-296) -> aes_ctr_set_key
// (crypto/fipsmodule/aes/aes.cc.inc:168-208): the FIPS-197 key schedule
// (section 5.2; the reference's aes_nohw_setup_key_128/192/256,
// aes_nohw.cc.inc:935-1114), H = E_K(0^128), and the GHASH multipliers the
// kernels use (H^1..H^17 prepared for the constant-time VALU product, the
// nibble table of H^16, the bitsliced engine's AddRoundKey masks).
//
// Constant time like the reference's key schedule: the S-box is the
// Boyar-Peralta circuit on bit-planes (sbox_portable.inc; the reference's
// aes_nohw_sub_bytes is the same circuit, aes_nohw.cc.inc:508), GF(2^128)
// products are gf128_ct.h's masked integer multiplications, and nothing
// branches on or indexes memory by key-derived data.
#pragma once
#include <stdint.h>
#include <string.h>

#include "gf128_ct.h"
#include "internal.h"

namespace bssl_amd {

#include "sbox_portable.inc"

// 8x8 bit-matrix transpose of x's bytes: bit 8*i + j <-> bit 8*j + i.
BSSL_GF_HD uint64_t ks_tr8(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x ^= t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x ^= t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x ^= t ^ (t << 28);
  return x;
}

// SubBytes of the 16 bytes of w[0..3] (byte j of the block = byte j % 4 of
// word j / 4): bit-planes by two 8x8 transposes, the circuit, back.
BSSL_GF_HD void ks_sub4(uint32_t w[4]) {
  const uint64_t lo = ks_tr8((uint64_t)w[0] | ((uint64_t)w[1] << 32));
  const uint64_t hi = ks_tr8((uint64_t)w[2] | ((uint64_t)w[3] << 32));
  uint32_t in[8], out[8];
  for (int k = 0; k < 8; k++)
    in[k] = (uint32_t)((lo >> (8 * k)) & 0xff) | ((uint32_t)((hi >> (8 * k)) & 0xff) << 8);
  sbox_bits(in, out);
  uint64_t olo = 0, ohi = 0;
  for (int k = 0; k < 8; k++) {
    olo |= (uint64_t)(out[k] & 0xff) << (8 * k);
    ohi |= (uint64_t)((out[k] >> 8) & 0xff) << (8 * k);
  }
  olo = ks_tr8(olo);
  ohi = ks_tr8(ohi);
  w[0] = (uint32_t)olo;
  w[1] = (uint32_t)(olo >> 32);
  w[2] = (uint32_t)ohi;
  w[3] = (uint32_t)(ohi >> 32);
}

// SubWord (FIPS-197 5.2) of one little-endian word.
BSSL_GF_HD uint32_t ks_subword(uint32_t x) {
  uint32_t w[4] = {x, 0, 0, 0};
  ks_sub4(w);
  return w[0];
}

BSSL_GF_HD uint32_t ks_rotr8(uint32_t x, int n) { return (x >> (8 * n)) | (x << (32 - 8 * n)); }

// xtime on each byte of a word.
BSSL_GF_HD uint32_t ks_xtime4(uint32_t u) {
  return ((u & 0x7f7f7f7fu) << 1) ^ (((u >> 7) & 0x01010101u) * 0x1bu);
}

// The FIPS-197 schedule as little-endian words (word i = bytes 4i..4i+3);
// returns the number of rounds, 0 for a bad key length.
BSSL_GF_HD int ks_expand(const uint8_t *key, int key_len, uint32_t rk[60]) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return 0;
  const int nk = key_len / 4, nr = nk + 6;
  for (int i = 0; i < nk; i++)
    rk[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) |
            ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
  uint32_t rcon = 1;
  for (int i = nk; i < 4 * (nr + 1); i++) {
    uint32_t t = rk[i - 1];
    if (i % nk == 0) {
      t = ks_subword(ks_rotr8(t, 1)) ^ rcon;  // RotWord on bytes = rotate right by 8
      rcon = ks_xtime4(rcon) & 0xffu;
    } else if (nk == 8 && i % nk == 4) {
      t = ks_subword(t);
    }
    rk[i] = rk[i - nk] ^ t;
  }
  return nr;
}

// E_K of one block held as four little-endian column words.
BSSL_GF_HD void ks_encrypt(const uint32_t *rk, int nr, uint32_t s[4]) {
  for (int c = 0; c < 4; c++) s[c] ^= rk[c];
  for (int r = 1; r <= nr; r++) {
    ks_sub4(s);
    uint32_t t[4];
    for (int c = 0; c < 4; c++)  // ShiftRows: row j of column c from column c + j
      t[c] = (s[c] & 0xffu) | (s[(c + 1) & 3] & 0xff00u) | (s[(c + 2) & 3] & 0xff0000u) |
             (s[(c + 3) & 3] & 0xff000000u);
    if (r != nr)
      for (int c = 0; c < 4; c++) {  // MixColumns
        const uint32_t a = t[c], a1 = ks_rotr8(a, 1);
        t[c] = a ^ a1 ^ ks_rotr8(a, 2) ^ ks_rotr8(a, 3) ^ a ^ ks_xtime4(a ^ a1);
      }
    for (int c = 0; c < 4; c++) s[c] = t[c] ^ rk[4 * r + c];
  }
}

BSSL_GF_HD uint32_t ks_bswap(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// Multiply by x in GCM's reflected order on the reversed-domain value (a
// right shift of the big-endian integer, reduced by 0xE1 || 0^120).
BSSL_GF_HD Gf128 ks_mulx(Gf128 v) {
  const uint32_t carry = 0u - (v.w[0] & 1u);
  v.w[0] = (v.w[0] >> 1) | (v.w[1] << 31);
  v.w[1] = (v.w[1] >> 1) | (v.w[2] << 31);
  v.w[2] = (v.w[2] >> 1) | (v.w[3] << 31);
  v.w[3] = (v.w[3] >> 1) ^ (carry & 0xE1000000u);
  return v;
}

// Wipes key-derived temporaries (the reference cleanses key state,
// OPENSSL_cleanse).  On the device the setup kernel's arrays indexed by the
// key length (the round keys, the raw key bytes) live in private scratch
// memory, which outlives the kernel and is handed to later ones unwiped, so
// the device form overwrites them through volatile stores the compiler cannot
// drop.
BSSL_GF_HD void ks_wipe(void *p, size_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (((uintptr_t)p | n) % 4 == 0) {
    volatile uint32_t *q = static_cast<volatile uint32_t *>(p);
    for (size_t i = 0; i < n / 4; i++) q[i] = 0;
  } else {
    volatile uint8_t *q = static_cast<volatile uint8_t *>(p);
    for (size_t i = 0; i < n; i++) q[i] = 0;
  }
#else
  explicit_bzero(p, n);
#endif
}

// Every field of *out (all of it written, padding zeroed); false (nothing
// written) for a bad key length.  `out` may be device memory (one lane per
// key) or host memory.
BSSL_GF_HD bool gcm_key_tables(const uint8_t *key, int key_len, GcmKeyDev *out) {
  uint32_t rk[60];
  const int nr = ks_expand(key, key_len, rk);
  if (!nr) return false;
  for (int r = 0; r < 15; r++)
    for (int c = 0; c < 4; c++) {
      const uint32_t v = r <= nr ? rk[4 * r + c] : 0u;
      out->rk[r][c] = (r == 0 || r == nr) ? v : ((v << 16) | (v >> 16));
      out->rk_plain[r][c] = v;
    }
  out->nr = (uint32_t)nr;
  out->key_bytes = (uint32_t)key_len;
  out->pad[0] = out->pad[1] = 0;
  // The bitsliced engine's AddRoundKey masks (GcmKeyDev::bsmask).
  for (int r = 0; r < 15; r++)
    for (int i = 0; i < 64; i++) {
      const int h = i >> 5, bit = (i & 31);  // bit = 8 * row + b
      const uint32_t lo = r <= nr ? (rk[4 * r + h] >> bit) & 1u : 0u;
      const uint32_t hi = r <= nr ? (rk[4 * r + h + 2] >> bit) & 1u : 0u;
      out->bsmask[r][i] = (lo * 0xffffu) | (hi * 0xffff0000u);
    }
  // H = E_K(0^128) (gcm.cc.inc:270-272), in the reversed domain: the
  // big-endian integer of its 16 bytes.
  uint32_t s[4] = {0, 0, 0, 0};
  ks_encrypt(rk, nr, s);
  Gf128 h;
  for (int c = 0; c < 4; c++) h.w[3 - c] = ks_bswap(s[c]);
  const Gf128 hp = gf_prep(h);
  // H^1 .. H^17 as multipliers (gf_prep); H^16 kept for the nibble table.
  for (int j = 0; j < 4; j++) out->hpow_ct[0][j] = 0;
  Gf128 hk = h, h16 = h;
  for (int k = 1; k <= 17; k++) {
    const Gf128 g = gf_prep(hk);
    for (int j = 0; j < 4; j++) out->hpow_ct[k][j] = g.w[j];
    if (k == 16) h16 = hk;
    hk = gf_mul(hk, hp);
  }
  // htab16[2k + half][val] = (nibble val at nibble position 2k + half) * H^16:
  // the XOR of the basis elements H^16 * x^(8k + 4 half + t) for the set bits
  // (3 - t) of val (public), as little-endian words of the GCM-order bytes.
  Gf128 v = h16;
  for (int pos = 0; pos < 32; pos++) {
    Gf128 b[4];
    for (int t = 0; t < 4; t++) {
      b[t] = v;
      v = ks_mulx(v);
    }
    for (int val = 0; val < 16; val++) {
      uint32_t e[4] = {0, 0, 0, 0};
      for (int t = 0; t < 4; t++)
        if ((val >> (3 - t)) & 1)
          for (int j = 0; j < 4; j++) e[j] ^= b[t].w[j];
      for (int j = 0; j < 4; j++) out->htab16[pos][val][j] = ks_bswap(e[3 - j]);
    }
    ks_wipe(b, sizeof(b));
  }
  ks_wipe(rk, sizeof(rk));
  ks_wipe(s, sizeof(s));
  ks_wipe(&h, sizeof(h));
  ks_wipe(&hk, sizeof(hk));
  ks_wipe(&h16, sizeof(h16));
  ks_wipe(&v, sizeof(v));
  return true;
}

}  // namespace bssl_amd
