/* aead_oracle.c -- plain-C restatement of the reference bulk-AEAD algorithms.
 *
 * TEST INFRASTRUCTURE ONLY (see aead_oracle.h).  Deliberately simple and
 * table-driven: this is the checker, not a product path, and it is never
 * constant-time.  Every function cites the reference code whose semantics it
 * restates; the restatement is written from the specifications (FIPS-197,
 * NIST SP 800-38D, RFC 8439), not from the reference sources.
 */
#include "aead_oracle.h"

#include <string.h>

/* ------------------------------------------------------------------------- */
/* AES (FIPS-197).  Reference semantics: crypto/fipsmodule/aes/aes.cc.inc:28-84
 * (block function dispatch) and aes_nohw.cc.inc:935-961,1069-1114 (key
 * schedules for 128/192/256-bit keys).  The S-box is generated from its
 * definition (multiplicative inverse in GF(2^8) followed by the affine map)
 * rather than typed in. */

static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

static uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) p ^= a;
    uint8_t hi = a & 0x80;
    a <<= 1;
    if (hi) a ^= 0x1b;
    b >>= 1;
  }
  return p;
}

static void sbox_init(void) {
  if (g_sbox_ready) return;
  for (int x = 0; x < 256; x++) {
    /* inverse = x^254 */
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, base = (uint8_t)x;
      int e = 254;
      while (e) {
        if (e & 1) r = gf8_mul(r, base);
        base = gf8_mul(base, base);
        e >>= 1;
      }
      inv = r;
    }
    uint8_t s = inv;
    uint8_t y = inv;
    for (int i = 0; i < 4; i++) {
      y = (uint8_t)((y << 1) | (y >> 7));
      s ^= y;
    }
    g_sbox[x] = s ^ 0x63;
  }
  g_sbox_ready = 1;
}

/* Expanded key as bytes: (Nr+1)*16 bytes.  Returns Nr or 0 on bad length. */
static int aes_expand(const uint8_t *key, size_t key_len, uint8_t rk[240]) {
  sbox_init();
  int nk = (int)(key_len / 4);
  if (key_len != 16 && key_len != 24 && key_len != 32) return 0;
  int nr = nk + 6;
  int total = 4 * (nr + 1);
  memcpy(rk, key, key_len);
  uint8_t rcon = 1;
  for (int i = nk; i < total; i++) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % nk == 0) {
      uint8_t t0 = t[0];
      t[0] = g_sbox[t[1]] ^ rcon;
      t[1] = g_sbox[t[2]];
      t[2] = g_sbox[t[3]];
      t[3] = g_sbox[t0];
      rcon = gf8_mul(rcon, 2);
    } else if (nk > 6 && i % nk == 4) {
      for (int j = 0; j < 4; j++) t[j] = g_sbox[t[j]];
    }
    for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - nk) + j] ^ t[j];
  }
  return nr;
}

static void aes_encrypt_rk(const uint8_t *rk, int nr, const uint8_t in[16],
                           uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
  for (int round = 1; round <= nr; round++) {
    uint8_t t[16];
    /* SubBytes + ShiftRows: byte (row r, col c) <- s(row r, col c+r). */
    for (int c = 0; c < 4; c++)
      for (int r = 0; r < 4; r++) t[4 * c + r] = g_sbox[s[4 * ((c + r) & 3) + r]];
    if (round != nr) {
      for (int c = 0; c < 4; c++) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2],
                a3 = t[4 * c + 3];
        t[4 * c + 0] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
        t[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
        t[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
        t[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
      }
    }
    for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk[16 * round + i];
  }
  memcpy(out, s, 16);
}

void oracle_aes_encrypt_block(const uint8_t *key, size_t key_len,
                              const uint8_t in[16], uint8_t out[16]) {
  uint8_t rk[240];
  int nr = aes_expand(key, key_len, rk);
  if (!nr) {
    memset(out, 0, 16);
    return;
  }
  aes_encrypt_rk(rk, nr, in, out);
}

/* ------------------------------------------------------------------------- */
/* GHASH multiply, NIST SP 800-38D Algorithm 1 (bit 0 = MSB of byte 0).  The
 * reference computes the same product in POLYVAL form
 * (crypto/fipsmodule/aes/gcm_nohw.cc.inc:197-304); results are identical. */
void oracle_gf128_mul(uint8_t x[16], const uint8_t h[16]) {
  uint8_t z[16] = {0}, v[16];
  memcpy(v, h, 16);
  for (int i = 0; i < 128; i++) {
    if ((x[i >> 3] >> (7 - (i & 7))) & 1)
      for (int j = 0; j < 16; j++) z[j] ^= v[j];
    int lsb = v[15] & 1;
    for (int j = 15; j > 0; j--) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
  }
  memcpy(x, z, 16);
}

static void ghash_update(uint8_t x[16], const uint8_t h[16], const uint8_t *p,
                         size_t len) {
  while (len) {
    size_t n = len < 16 ? len : 16;
    for (size_t i = 0; i < n; i++) x[i] ^= p[i];
    oracle_gf128_mul(x, h);
    p += n;
    len -= n;
  }
}

static void store_be64(uint8_t *p, uint64_t v) {
  for (int i = 7; i >= 0; i--) {
    p[i] = (uint8_t)v;
    v >>= 8;
  }
}

/* Core of CRYPTO_gcm128_{init_ctx,aad,encrypt/decrypt,finish}
 * (crypto/fipsmodule/aes/gcm.cc.inc:298-604).  `encrypt` selects whether
 * GHASH runs over the output (seal) or the input (open). */
static int gcm_crypt(const uint8_t *key, size_t key_len, const uint8_t *iv,
                     size_t iv_len, const uint8_t *in, size_t len,
                     const uint8_t *ad, size_t ad_len, uint8_t *out,
                     uint8_t full_tag[16], int encrypt) {
  uint8_t rk[240];
  int nr = aes_expand(key, key_len, rk);
  if (!nr) return 0;
  if (iv_len == 0) return 0; /* e_aes.cc.inc:790-793 */
  /* gcm.cc.inc:409: message limit 2^36 - 32 bytes; :368 AAD limit 2^61. */
  if ((uint64_t)len > ((UINT64_C(1) << 36) - 32)) return 0;
  if ((uint64_t)ad_len > (UINT64_C(1) << 61)) return 0;

  uint8_t h[16] = {0};
  aes_encrypt_rk(rk, nr, h, h); /* H = E_K(0^128), gcm.cc.inc:270-272 */

  uint8_t j0[16] = {0};
  if (iv_len == 12) { /* gcm.cc.inc:316-319 */
    memcpy(j0, iv, 12);
    j0[15] = 1;
  } else { /* gcm.cc.inc:320-338 */
    ghash_update(j0, h, iv, iv_len);
    uint8_t lb[16] = {0};
    store_be64(lb + 8, (uint64_t)iv_len << 3);
    for (int i = 0; i < 16; i++) j0[i] ^= lb[i];
    oracle_gf128_mul(j0, h);
  }
  uint32_t ctr = ((uint32_t)j0[12] << 24) | ((uint32_t)j0[13] << 16) |
                 ((uint32_t)j0[14] << 8) | j0[15];
  uint8_t ek0[16];
  aes_encrypt_rk(rk, nr, j0, ek0);

  uint8_t x[16] = {0};
  ghash_update(x, h, ad, ad_len);
  if (!encrypt) ghash_update(x, h, in, len);

  uint8_t cb[16];
  memcpy(cb, j0, 12);
  for (size_t off = 0; off < len; off += 16) {
    ctr++; /* inc32: wraps modulo 2^32 */
    cb[12] = (uint8_t)(ctr >> 24);
    cb[13] = (uint8_t)(ctr >> 16);
    cb[14] = (uint8_t)(ctr >> 8);
    cb[15] = (uint8_t)ctr;
    uint8_t ks[16];
    aes_encrypt_rk(rk, nr, cb, ks);
    size_t n = len - off < 16 ? len - off : 16;
    for (size_t i = 0; i < n; i++) out[off + i] = in[off + i] ^ ks[i];
  }
  if (encrypt) ghash_update(x, h, out, len);

  uint8_t lb[16];
  store_be64(lb, (uint64_t)ad_len << 3);
  store_be64(lb + 8, (uint64_t)len << 3);
  for (int i = 0; i < 16; i++) x[i] ^= lb[i];
  oracle_gf128_mul(x, h);
  for (int i = 0; i < 16; i++) full_tag[i] = x[i] ^ ek0[i];
  return 1;
}

int oracle_aes_gcm_seal(const uint8_t *key, size_t key_len,
                        const uint8_t *nonce, size_t nonce_len,
                        const uint8_t *in, size_t in_len, const uint8_t *ad,
                        size_t ad_len, uint8_t *out, uint8_t *tag,
                        size_t tag_len) {
  uint8_t full[16];
  if (tag_len > 16) return 0;
  if (!gcm_crypt(key, key_len, nonce, nonce_len, in, in_len, ad, ad_len, out,
                 full, 1)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  memcpy(tag, full, tag_len);
  return 1;
}

int oracle_aes_gcm_open(const uint8_t *key, size_t key_len,
                        const uint8_t *nonce, size_t nonce_len,
                        const uint8_t *in, size_t in_len, const uint8_t *ad,
                        size_t ad_len, const uint8_t *tag, size_t tag_len,
                        uint8_t *out) {
  uint8_t full[16];
  if (tag_len > 16 ||
      !gcm_crypt(key, key_len, nonce, nonce_len, in, in_len, ad, ad_len, out,
                 full, 0)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  uint8_t diff = 0;
  for (size_t i = 0; i < tag_len; i++) diff |= full[i] ^ tag[i];
  if (diff) { /* e_aes.cc.inc:860-864, zero-on-error aead.cc.inc:539-547 */
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* ChaCha20, RFC 8439 section 2.3; reference crypto/chacha/chacha.cc:154-224
 * (32-bit block counter in word 12, nonce in words 13-15). */

static uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
static uint32_t load_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

#define QR(a, b, c, d)  \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

static void chacha_block(uint8_t out[64], const uint8_t key[32],
                         const uint8_t nonce[12], uint32_t counter) {
  uint32_t in[16], x[16];
  in[0] = 0x61707865; in[1] = 0x3320646e; in[2] = 0x79622d32; in[3] = 0x6b206574;
  for (int i = 0; i < 8; i++) in[4 + i] = load_le32(key + 4 * i);
  in[12] = counter;
  for (int i = 0; i < 3; i++) in[13 + i] = load_le32(nonce + 4 * i);
  memcpy(x, in, sizeof(x));
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; i++) {
    uint32_t v = x[i] + in[i];
    out[4 * i] = (uint8_t)v;
    out[4 * i + 1] = (uint8_t)(v >> 8);
    out[4 * i + 2] = (uint8_t)(v >> 16);
    out[4 * i + 3] = (uint8_t)(v >> 24);
  }
}

void oracle_chacha20(uint8_t *out, const uint8_t *in, size_t len,
                     const uint8_t key[32], const uint8_t nonce[12],
                     uint32_t counter) {
  uint8_t ks[64];
  for (size_t off = 0; off < len; off += 64) {
    chacha_block(ks, key, nonce, counter++);
    size_t n = len - off < 64 ? len - off : 64;
    for (size_t i = 0; i < n; i++) out[off + i] = in[off + i] ^ ks[i];
  }
}

/* ------------------------------------------------------------------------- */
/* Poly1305, RFC 8439 section 2.5; reference crypto/poly1305/poly1305.cc:54-313.
 * Arithmetic modulo 2^130-5 with three 64-bit limbs (44/44/42 bits) and
 * unsigned __int128 products. */

typedef struct {
  uint64_t r[3], h[3], pad[2];
  uint8_t buf[16];
  size_t buf_len;
} poly_state;

static void poly_init(poly_state *st, const uint8_t key[32]) {
  uint64_t t0 = 0, t1 = 0;
  for (int i = 7; i >= 0; i--) t0 = (t0 << 8) | key[i];
  for (int i = 15; i >= 8; i--) t1 = (t1 << 8) | key[i];
  /* clamp r (RFC 8439 2.5.1) */
  t0 &= UINT64_C(0x0ffffffc0fffffff);
  t1 &= UINT64_C(0x0ffffffc0ffffffc);
  st->r[0] = t0 & UINT64_C(0xfffffffffff);
  st->r[1] = ((t0 >> 44) | (t1 << 20)) & UINT64_C(0xfffffffffff);
  st->r[2] = (t1 >> 24) & UINT64_C(0x3ffffffffff);
  st->h[0] = st->h[1] = st->h[2] = 0;
  uint64_t p0 = 0, p1 = 0;
  for (int i = 23; i >= 16; i--) p0 = (p0 << 8) | key[i];
  for (int i = 31; i >= 24; i--) p1 = (p1 << 8) | key[i];
  st->pad[0] = p0;
  st->pad[1] = p1;
  st->buf_len = 0;
}

static void poly_block(poly_state *st, const uint8_t m[16], uint64_t hibit) {
  typedef unsigned __int128 u128;
  const uint64_t M44 = UINT64_C(0xfffffffffff), M42 = UINT64_C(0x3ffffffffff);
  uint64_t t0 = 0, t1 = 0;
  for (int i = 7; i >= 0; i--) t0 = (t0 << 8) | m[i];
  for (int i = 15; i >= 8; i--) t1 = (t1 << 8) | m[i];
  uint64_t h0 = st->h[0] + (t0 & M44);
  uint64_t h1 = st->h[1] + (((t0 >> 44) | (t1 << 20)) & M44);
  uint64_t h2 = st->h[2] + (((t1 >> 24) & M42) | (hibit << 40));
  uint64_t r0 = st->r[0], r1 = st->r[1], r2 = st->r[2];
  uint64_t s1 = r1 * (5 << 2), s2 = r2 * (5 << 2);
  u128 d0 = (u128)h0 * r0 + (u128)h1 * s2 + (u128)h2 * s1;
  u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * s2;
  u128 d2 = (u128)h0 * r2 + (u128)h1 * r1 + (u128)h2 * r0;
  uint64_t c = (uint64_t)(d0 >> 44);
  h0 = (uint64_t)d0 & M44;
  d1 += c;
  c = (uint64_t)(d1 >> 44);
  h1 = (uint64_t)d1 & M44;
  d2 += c;
  c = (uint64_t)(d2 >> 42);
  h2 = (uint64_t)d2 & M42;
  h0 += c * 5;
  c = h0 >> 44;
  h0 &= M44;
  h1 += c;
  st->h[0] = h0;
  st->h[1] = h1;
  st->h[2] = h2;
}

static void poly_update(poly_state *st, const uint8_t *m, size_t len) {
  while (len) {
    size_t take = 16 - st->buf_len;
    if (take > len) take = len;
    memcpy(st->buf + st->buf_len, m, take);
    st->buf_len += take;
    m += take;
    len -= take;
    if (st->buf_len == 16) {
      poly_block(st, st->buf, 1);
      st->buf_len = 0;
    }
  }
}

static void poly_finish(poly_state *st, uint8_t tag[16]) {
  const uint64_t M44 = UINT64_C(0xfffffffffff), M42 = UINT64_C(0x3ffffffffff);
  if (st->buf_len) {
    uint8_t b[16] = {0};
    memcpy(b, st->buf, st->buf_len);
    b[st->buf_len] = 1;
    poly_block(st, b, 0);
  }
  uint64_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  /* g = h + 5 - 2^130; select g if non-negative */
  uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
  uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
  uint64_t g2 = h2 + c - (UINT64_C(1) << 42);
  uint64_t mask = (g2 >> 63) - 1; /* all-ones when g2 did not borrow */
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  /* h = h + pad mod 2^128 */
  uint64_t lo = h0 | (h1 << 44);
  uint64_t hi = (h1 >> 20) | (h2 << 24);
  uint64_t nlo = lo + st->pad[0];
  uint64_t carry = nlo < lo;
  uint64_t nhi = hi + st->pad[1] + carry;
  for (int i = 0; i < 8; i++) {
    tag[i] = (uint8_t)(nlo >> (8 * i));
    tag[8 + i] = (uint8_t)(nhi >> (8 * i));
  }
}

void oracle_poly1305(uint8_t tag[16], const uint8_t *msg, size_t len,
                     const uint8_t key[32]) {
  poly_state st;
  poly_init(&st, key);
  poly_update(&st, msg, len);
  poly_finish(&st, tag);
}

/* calc_tag_pre / calc_tag_post, crypto/cipher/e_chacha20poly1305.cc:84-115 */
static int chacha_poly_crypt(const uint8_t key[32], const uint8_t *nonce,
                             size_t nonce_len, const uint8_t *in,
                             size_t in_len, const uint8_t *ad, size_t ad_len,
                             uint8_t *out, uint8_t full_tag[16], int encrypt) {
  if (nonce_len != 12) return 0; /* e_chacha20poly1305.cc:127-130 */
  /* e_chacha20poly1305.cc:138-142: at most 2^32 blocks of 64 bytes. */
  if ((uint64_t)in_len >= (UINT64_C(1) << 32) * 64 - 64) return 0;
  static const uint8_t zeros[16] = {0};
  uint8_t pkey[64];
  memset(pkey, 0, sizeof(pkey));
  oracle_chacha20(pkey, pkey, 32, key, nonce, 0);
  poly_state st;
  poly_init(&st, pkey);
  poly_update(&st, ad, ad_len);
  if (ad_len % 16) poly_update(&st, zeros, 16 - ad_len % 16);
  if (!encrypt) poly_update(&st, in, in_len);
  oracle_chacha20(out, in, in_len, key, nonce, 1);
  if (encrypt) poly_update(&st, out, in_len);
  if (in_len % 16) poly_update(&st, zeros, 16 - in_len % 16);
  uint8_t lens[16];
  for (int i = 0; i < 8; i++) {
    lens[i] = (uint8_t)((uint64_t)ad_len >> (8 * i));
    lens[8 + i] = (uint8_t)((uint64_t)in_len >> (8 * i));
  }
  poly_update(&st, lens, 16);
  poly_finish(&st, full_tag);
  return 1;
}

int oracle_chacha20_poly1305_seal(const uint8_t key[32], const uint8_t *nonce,
                                  size_t nonce_len, const uint8_t *in,
                                  size_t in_len, const uint8_t *ad,
                                  size_t ad_len, uint8_t *out, uint8_t *tag,
                                  size_t tag_len) {
  uint8_t full[16];
  if (tag_len > 16 || !chacha_poly_crypt(key, nonce, nonce_len, in, in_len, ad,
                                         ad_len, out, full, 1)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  memcpy(tag, full, tag_len);
  return 1;
}

int oracle_chacha20_poly1305_open(const uint8_t key[32], const uint8_t *nonce,
                                  size_t nonce_len, const uint8_t *in,
                                  size_t in_len, const uint8_t *ad,
                                  size_t ad_len, const uint8_t *tag,
                                  size_t tag_len, uint8_t *out) {
  uint8_t full[16];
  if (tag_len > 16 || !chacha_poly_crypt(key, nonce, nonce_len, in, in_len, ad,
                                         ad_len, out, full, 0)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  uint8_t diff = 0;
  for (size_t i = 0; i < tag_len; i++) diff |= full[i] ^ tag[i];
  if (diff) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* AES-GCM-SIV (RFC 8452); reference crypto/cipher/e_aesgcmsiv.cc:533-867
 * (the portable path).  POLYVAL is evaluated through GHASH exactly as the
 * reference does (:604-682): H' = mulX_GHASH(ByteReverse(H)), blocks
 * byte-reversed, result byte-reversed. */

static void siv_byte_reverse(uint8_t b[16]) { /* e_aesgcmsiv.cc:624-629 */
  for (int i = 0; i < 8; i++) {
    uint8_t t = b[i];
    b[i] = b[15 - i];
    b[15 - i] = t;
  }
}

/* e_aesgcmsiv.cc:634-645: b as a little-endian 128-bit integer V; V >>= 1,
 * 0xe1 into the top byte if bit 0 was set; written back big-endian. */
static void siv_reverse_and_mulX_ghash(uint8_t b[16]) {
  uint8_t v[16];
  const int carry = b[0] & 1;
  for (int i = 0; i < 16; i++)
    v[i] = (uint8_t)((b[i] >> 1) | (i < 15 ? (uint8_t)(b[i + 1] << 7) : 0));
  if (carry) v[15] ^= 0xe1;
  for (int i = 0; i < 16; i++) b[i] = v[15 - i];
}

typedef struct {
  uint8_t h[16]; /* mulX_GHASH(ByteReverse(auth key)) */
  uint8_t s[16]; /* GHASH-order accumulator */
} siv_polyval;

static void siv_polyval_init(siv_polyval *p, const uint8_t key[16]) {
  memcpy(p->h, key, 16);
  siv_reverse_and_mulX_ghash(p->h);
  memset(p->s, 0, 16);
}

/* Zero-padded 16-byte blocks of `in` (e_aesgcmsiv.cc:697-711). */
static void siv_polyval_update(siv_polyval *p, const uint8_t *in, size_t len) {
  for (size_t o = 0; o < len; o += 16) {
    uint8_t blk[16] = {0};
    memcpy(blk, in + o, len - o < 16 ? len - o : 16);
    siv_byte_reverse(blk);
    for (int i = 0; i < 16; i++) p->s[i] ^= blk[i];
    oracle_gf128_mul(p->s, p->h);
  }
}

/* gcm_siv_polyval (e_aesgcmsiv.cc:686-736): POLYVAL over AD || PT || lengths,
 * XOR the nonce, clear the top bit. */
static void siv_tag_input(const uint8_t auth_key[16], const uint8_t *ad, size_t ad_len,
                          const uint8_t *pt, size_t pt_len, const uint8_t nonce[12],
                          uint8_t out[16]) {
  siv_polyval p;
  siv_polyval_init(&p, auth_key);
  siv_polyval_update(&p, ad, ad_len);
  siv_polyval_update(&p, pt, pt_len);
  uint8_t lens[16];
  for (int i = 0; i < 8; i++) {
    lens[i] = (uint8_t)(((uint64_t)ad_len * 8) >> (8 * i));
    lens[8 + i] = (uint8_t)(((uint64_t)pt_len * 8) >> (8 * i));
  }
  siv_polyval_update(&p, lens, 16);
  memcpy(out, p.s, 16);
  siv_byte_reverse(out);
  for (int i = 0; i < 12; i++) out[i] ^= nonce[i];
  out[15] &= 0x7f;
}

/* gcm_siv_keys (e_aesgcmsiv.cc:750-780): AES_K(le32(i) || nonce)[0:8] for
 * i = 0..3 (AES-128) or 0..5 (AES-256): 16-byte auth key, then the record's
 * encryption key. */
static void siv_record_keys(const uint8_t *key, size_t key_len, const uint8_t nonce[12],
                            uint8_t auth_key[16], uint8_t enc_key[32]) {
  uint8_t material[48];
  const int blocks = key_len == 32 ? 6 : 4;
  for (int i = 0; i < blocks; i++) {
    uint8_t ctr[16] = {0}, ks[16];
    ctr[0] = (uint8_t)i;
    memcpy(ctr + 4, nonce, 12);
    oracle_aes_encrypt_block(key, key_len, ctr, ks);
    memcpy(material + 8 * i, ks, 8);
  }
  memcpy(auth_key, material, 16);
  memcpy(enc_key, material + 16, key_len);
}

/* gcm_siv_crypt (e_aesgcmsiv.cc:571-601): CTR from the tag with byte 15 |=
 * 0x80 and a little-endian 32-bit counter in bytes 0..3. */
static void siv_ctr(const uint8_t *enc_key, size_t key_len, const uint8_t tag[16],
                    const uint8_t *in, uint8_t *out, size_t len) {
  uint8_t ctr[16], ks[16];
  memcpy(ctr, tag, 16);
  ctr[15] |= 0x80;
  for (size_t o = 0; o < len; o += 16) {
    oracle_aes_encrypt_block(enc_key, key_len, ctr, ks);
    uint32_t c = (uint32_t)ctr[0] | ((uint32_t)ctr[1] << 8) | ((uint32_t)ctr[2] << 16) |
                 ((uint32_t)ctr[3] << 24);
    c++;
    ctr[0] = (uint8_t)c; ctr[1] = (uint8_t)(c >> 8); ctr[2] = (uint8_t)(c >> 16);
    ctr[3] = (uint8_t)(c >> 24);
    for (size_t i = 0; i < 16 && o + i < len; i++) out[o + i] = in[o + i] ^ ks[i];
  }
}

/* aead_aes_gcm_siv_sealv (e_aesgcmsiv.cc:782-823).  tag_len must be 16
 * (aead_aes_gcm_siv_init, :542-548). */
int oracle_aes_gcm_siv_seal(const uint8_t *key, size_t key_len, const uint8_t *nonce,
                            size_t nonce_len, const uint8_t *in, size_t in_len,
                            const uint8_t *ad, size_t ad_len, uint8_t *out, uint8_t *tag,
                            size_t tag_len) {
  if ((key_len != 16 && key_len != 32) || tag_len != 16 || nonce_len != 12 ||
      (uint64_t)in_len > (UINT64_C(1) << 36) || (uint64_t)ad_len >= (UINT64_C(1) << 61)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  uint8_t auth_key[16], enc_key[32], t[16];
  siv_record_keys(key, key_len, nonce, auth_key, enc_key);
  siv_tag_input(auth_key, ad, ad_len, in, in_len, nonce, t);
  oracle_aes_encrypt_block(enc_key, key_len, t, t);
  siv_ctr(enc_key, key_len, t, in, out, in_len);
  memcpy(tag, t, 16);
  return 1;
}

/* aead_aes_gcm_siv_openv_detached (e_aesgcmsiv.cc:825-867). */
int oracle_aes_gcm_siv_open(const uint8_t *key, size_t key_len, const uint8_t *nonce,
                            size_t nonce_len, const uint8_t *in, size_t in_len,
                            const uint8_t *ad, size_t ad_len, const uint8_t *tag,
                            size_t tag_len, uint8_t *out) {
  if ((key_len != 16 && key_len != 32) || tag_len != 16 || nonce_len != 12 ||
      (uint64_t)in_len > (UINT64_C(1) << 36) || (uint64_t)ad_len >= (UINT64_C(1) << 61)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  uint8_t auth_key[16], enc_key[32], t[16];
  siv_record_keys(key, key_len, nonce, auth_key, enc_key);
  siv_ctr(enc_key, key_len, tag, in, out, in_len);
  siv_tag_input(auth_key, ad, ad_len, out, in_len, nonce, t);
  oracle_aes_encrypt_block(enc_key, key_len, t, t);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= t[i] ^ tag[i];
  if (diff) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  return 1;
}

/* HChaCha20 (draft-irtf-cfrg-xchacha-03 section 2.2); reference
 * CRYPTO_hchacha20, crypto/chacha/chacha.cc:43-63: the ChaCha20 state of
 * (key, 16-byte nonce) after 20 rounds, words 0-3 and 12-15, no feed-forward. */
void oracle_hchacha20(uint8_t out[32], const uint8_t key[32],
                      const uint8_t nonce[16]) {
  uint32_t x[16];
  x[0] = 0x61707865; x[1] = 0x3320646e; x[2] = 0x79622d32; x[3] = 0x6b206574;
  for (int i = 0; i < 8; i++) x[4 + i] = load_le32(key + 4 * i);
  for (int i = 0; i < 4; i++) x[12 + i] = load_le32(nonce + 4 * i);
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 8; i++) {
    const uint32_t v = x[i < 4 ? i : i + 8];
    out[4 * i] = (uint8_t)v;
    out[4 * i + 1] = (uint8_t)(v >> 8);
    out[4 * i + 2] = (uint8_t)(v >> 16);
    out[4 * i + 3] = (uint8_t)(v >> 24);
  }
}

/* XChaCha20-Poly1305 (crypto/cipher/e_chacha20poly1305.cc:233-256, 310-330):
 * 24-byte nonce, key' = HChaCha20(key, nonce[0:16]), nonce' = 0^4 || nonce[16:24],
 * then ChaCha20-Poly1305 under (key', nonce'). */
static int xchacha_derive(const uint8_t key[32], const uint8_t *nonce,
                          size_t nonce_len, uint8_t dkey[32], uint8_t dnonce[12]) {
  if (nonce_len != 24) return 0; /* e_chacha20poly1305.cc:241-244 */
  oracle_hchacha20(dkey, key, nonce);
  memset(dnonce, 0, 4);
  memcpy(dnonce + 4, nonce + 16, 8);
  return 1;
}

int oracle_xchacha20_poly1305_seal(const uint8_t key[32], const uint8_t *nonce,
                                   size_t nonce_len, const uint8_t *in,
                                   size_t in_len, const uint8_t *ad,
                                   size_t ad_len, uint8_t *out, uint8_t *tag,
                                   size_t tag_len) {
  uint8_t dkey[32], dnonce[12];
  if (!xchacha_derive(key, nonce, nonce_len, dkey, dnonce)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  return oracle_chacha20_poly1305_seal(dkey, dnonce, 12, in, in_len, ad, ad_len,
                                       out, tag, tag_len);
}

int oracle_xchacha20_poly1305_open(const uint8_t key[32], const uint8_t *nonce,
                                   size_t nonce_len, const uint8_t *in,
                                   size_t in_len, const uint8_t *ad,
                                   size_t ad_len, const uint8_t *tag,
                                   size_t tag_len, uint8_t *out) {
  uint8_t dkey[32], dnonce[12];
  if (!xchacha_derive(key, nonce, nonce_len, dkey, dnonce)) {
    if (in_len) memset(out, 0, in_len);
    return 0;
  }
  return oracle_chacha20_poly1305_open(dkey, dnonce, 12, in, in_len, ad, ad_len,
                                       tag, tag_len, out);
}

/* ------------------------------------------------------------------------- */

size_t oracle_batch(int aead, int seal, const uint8_t *keys, size_t key_len,
                    const uint32_t *key_index, size_t n, const uint8_t *in,
                    uint8_t *out, const uint64_t *offsets,
                    const uint64_t *lens, const uint8_t *nonces,
                    size_t nonce_len, const uint8_t *ad,
                    const uint64_t *ad_offsets, const uint64_t *ad_lens,
                    uint8_t *tags, size_t tag_len, uint8_t *status,
                    int threads) {
  sbox_init();
  size_t failed = 0;
  long long nn = (long long)n;
  (void)threads;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : failed) num_threads(threads > 0 ? threads : 1)
  for (long long i = 0; i < nn; i++) {
    const uint8_t *k = keys + key_len * (key_index ? key_index[i] : 0);
    const uint8_t *ni = nonces + (size_t)i * nonce_len;
    const uint8_t *ai = ad + ad_offsets[i];
    int ok;
    if (aead == ORACLE_AES_GCM) {
      ok = seal ? oracle_aes_gcm_seal(k, key_len, ni, nonce_len, in + offsets[i],
                                      lens[i], ai, ad_lens[i], out + offsets[i],
                                      tags + (size_t)i * tag_len, tag_len)
                : oracle_aes_gcm_open(k, key_len, ni, nonce_len, in + offsets[i],
                                      lens[i], ai, ad_lens[i],
                                      tags + (size_t)i * tag_len, tag_len,
                                      out + offsets[i]);
    } else if (aead == ORACLE_AES_GCM_SIV) {
      ok = seal ? oracle_aes_gcm_siv_seal(k, key_len, ni, nonce_len, in + offsets[i], lens[i],
                                          ai, ad_lens[i], out + offsets[i],
                                          tags + (size_t)i * tag_len, tag_len)
                : oracle_aes_gcm_siv_open(k, key_len, ni, nonce_len, in + offsets[i], lens[i],
                                          ai, ad_lens[i], tags + (size_t)i * tag_len, tag_len,
                                          out + offsets[i]);
    } else if (aead == ORACLE_XCHACHA20_POLY1305) {
      ok = seal ? oracle_xchacha20_poly1305_seal(
                      k, ni, nonce_len, in + offsets[i], lens[i], ai,
                      ad_lens[i], out + offsets[i], tags + (size_t)i * tag_len,
                      tag_len)
                : oracle_xchacha20_poly1305_open(
                      k, ni, nonce_len, in + offsets[i], lens[i], ai,
                      ad_lens[i], tags + (size_t)i * tag_len, tag_len,
                      out + offsets[i]);
    } else {
      ok = seal ? oracle_chacha20_poly1305_seal(
                      k, ni, nonce_len, in + offsets[i], lens[i], ai,
                      ad_lens[i], out + offsets[i], tags + (size_t)i * tag_len,
                      tag_len)
                : oracle_chacha20_poly1305_open(
                      k, ni, nonce_len, in + offsets[i], lens[i], ai,
                      ad_lens[i], tags + (size_t)i * tag_len, tag_len,
                      out + offsets[i]);
    }
    if (status) status[i] = (uint8_t)ok;
    if (!ok) failed++;
  }
  return failed;
}
