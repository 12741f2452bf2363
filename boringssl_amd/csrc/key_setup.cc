// key_setup.cc -- per-key setup on the host, the analogue of the reference's
// CRYPTO_gcm128_init_aes_key (crypto/fipsmodule/aes/gcm.cc.inc:253-296):
// AES key schedule (FIPS-197 section 5.2, as aes_nohw.cc.inc:935-961,
// 1069-1114), H = E_K(0^128), and the GHASH multiplication tables the kernels
// stage in LDS.  Runs once per key at EVP_AEAD_CTX_init / keyset creation; the
// record data never touches this code.
#include <string.h>

#include "gf128_ct.h"
#include "internal.h"

namespace bssl_amd {

void secure_zero(void *p, size_t n) {
  if (n) explicit_bzero(p, n);
}

namespace {

struct SboxTable {
  uint8_t s[256];
  SboxTable() {
    // S-box from its definition: inverse in GF(2^8) mod x^8+x^4+x^3+x+1,
    // then the affine map (FIPS-197 section 5.1.1).
    auto mul = [](uint8_t a, uint8_t b) {
      uint8_t p = 0;
      while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
      }
      return p;
    };
    for (int x = 0; x < 256; x++) {
      uint8_t inv = 0;
      for (int y = 1; y < 256 && x; y++)
        if (mul((uint8_t)x, (uint8_t)y) == 1) {
          inv = (uint8_t)y;
          break;
        }
      uint8_t r = inv, t = inv;
      for (int i = 0; i < 4; i++) {
        t = (uint8_t)((t << 1) | (t >> 7));
        r ^= t;
      }
      s[x] = r ^ 0x63;
    }
  }
};

const SboxTable &sbox() {
  static const SboxTable t;
  return t;
}

// S[x] for a secret x (key bytes, the state computing H = E_K(0)): every
// entry is read and the wanted one selected by a mask, so the host's cache
// never sees an address that depends on x (the reference keeps its key
// schedule constant-time too, aes_nohw.cc.inc:935-961).
uint8_t sbox_ct(uint8_t x) {
  const uint8_t *S = sbox().s;
  uint32_t r = 0;
  for (uint32_t i = 0; i < 256; i++) {
    const uint32_t eq = ((i ^ x) - 1u) >> 8 & 1u;  // 1 iff i == x
    r |= S[i] & (0u - eq);
  }
  return (uint8_t)r;
}

uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ (0x1b & (0u - (a >> 7)))); }

// FIPS-197 KeyExpansion; returns the number of rounds, 0 on a bad length.
int expand_key(const uint8_t *key, size_t key_len, uint8_t w[240]) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return 0;
  int nk = (int)key_len / 4, nr = nk + 6;
  memcpy(w, key, key_len);
  uint8_t rcon = 1;
  for (int i = nk; i < 4 * (nr + 1); i++) {
    uint8_t t[4];
    memcpy(t, w + 4 * (i - 1), 4);
    if (i % nk == 0) {
      uint8_t t0 = t[0];
      t[0] = sbox_ct(t[1]) ^ rcon;
      t[1] = sbox_ct(t[2]);
      t[2] = sbox_ct(t[3]);
      t[3] = sbox_ct(t0);
      rcon = xtime(rcon);
    } else if (nk == 8 && i % nk == 4) {
      for (auto &b : t) b = sbox_ct(b);
    }
    for (int j = 0; j < 4; j++) w[4 * i + j] = w[4 * (i - nk) + j] ^ t[j];
  }
  return nr;
}

void encrypt_block(const uint8_t *w, int nr, const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; i++) s[i] = in[i] ^ w[i];
  for (int r = 1; r <= nr; r++) {
    uint8_t t[16];
    for (int c = 0; c < 4; c++)
      for (int row = 0; row < 4; row++) t[4 * c + row] = sbox_ct(s[4 * ((c + row) & 3) + row]);
    if (r != nr)
      for (int c = 0; c < 4; c++) {
        uint8_t *a = t + 4 * c;
        uint8_t all = a[0] ^ a[1] ^ a[2] ^ a[3], a0 = a[0];
        a[0] ^= all ^ xtime(a[0] ^ a[1]);
        a[1] ^= all ^ xtime(a[1] ^ a[2]);
        a[2] ^= all ^ xtime(a[2] ^ a[3]);
        a[3] ^= all ^ xtime(a[3] ^ a0);
      }
    for (int i = 0; i < 16; i++) s[i] = t[i] ^ w[16 * r + i];
  }
  memcpy(out, s, 16);
}

// GF(2^128) elements in GCM bit order held as two big-endian 64-bit halves.
struct U128 {
  uint64_t hi, lo;
};

U128 load_u128(const uint8_t b[16]) {
  U128 r{0, 0};
  for (int i = 0; i < 8; i++) {
    r.hi = (r.hi << 8) | b[i];
    r.lo = (r.lo << 8) | b[8 + i];
  }
  return r;
}

void store_u128(U128 v, uint8_t b[16]) {
  for (int i = 7; i >= 0; i--) {
    b[i] = (uint8_t)v.hi;
    b[8 + i] = (uint8_t)v.lo;
    v.hi >>= 8;
    v.lo >>= 8;
  }
}

// Multiply by x: a right shift in GCM's reflected bit order, reducing by
// x^128 + x^7 + x^2 + x + 1 (0xE1 || 0^120).
// (Branch-free: H and its powers are secret.)
U128 mulx(U128 v) {
  const uint64_t carry = 0 - (v.lo & 1);
  v.lo = (v.lo >> 1) | (v.hi << 63);
  v.hi >>= 1;
  v.hi ^= carry & (UINT64_C(0xE1) << 56);
  return v;
}

U128 gf_mul(U128 x, U128 y) {
  U128 z{0, 0};
  for (int i = 0; i < 128; i++) {
    const uint64_t bit = 0 - (i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1);
    z.hi ^= y.hi & bit;
    z.lo ^= y.lo & bit;
    y = mulx(y);
  }
  return z;
}

uint32_t load_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

uint32_t rotl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

}  // namespace

bool gcm_key_setup(const uint8_t *key, size_t key_len, GcmKeyDev *out) {
  uint8_t w[240];
  int nr = expand_key(key, key_len, w);
  if (!nr) {
    secure_zero(w, sizeof(w));
    return false;
  }
  memset(out, 0, sizeof(*out));
  out->nr = (uint32_t)nr;
  out->key_bytes = (uint32_t)key_len;
  for (int r = 0; r <= nr; r++)
    for (int c = 0; c < 4; c++) {
      uint32_t v = load_le32(w + 16 * r + 4 * c);
      out->rk[r][c] = (r == 0 || r == nr) ? v : rotl32(v, 16);
      out->rk_plain[r][c] = v;
    }
  // The bitsliced engine's AddRoundKey masks (GcmKeyDev::bsmask).
  for (int r = 0; r <= nr; r++)
    for (int h = 0; h < 2; h++)
      for (int row = 0; row < 4; row++)
        for (int bit = 0; bit < 8; bit++) {
          const uint32_t lo = (out->rk_plain[r][h] >> (8 * row + bit)) & 1u;
          const uint32_t hi = (out->rk_plain[r][h + 2] >> (8 * row + bit)) & 1u;
          out->bsmask[r][32 * h + 8 * row + bit] = (lo * 0xffffu) | (hi * 0xffff0000u);
        }
  uint8_t hb[16] = {0};
  encrypt_block(w, nr, hb, hb);  // H = E_K(0^128), gcm.cc.inc:270-272
  U128 p = load_u128(hb);
  {
    // H^1 .. H^17 as constant-time multipliers (gf128_ct.h): the reversed
    // domain is the big-endian integer of the block, i.e. hi:lo.
    U128 hk = p;
    for (int k = 1; k <= 17; k++) {
      Gf128 g;
      g.w[3] = (uint32_t)(hk.hi >> 32);
      g.w[2] = (uint32_t)hk.hi;
      g.w[1] = (uint32_t)(hk.lo >> 32);
      g.w[0] = (uint32_t)hk.lo;
      const Gf128 gp = gf_prep(g);
      for (int j = 0; j < 4; j++) out->hpow_ct[k][j] = gp.w[j];
      secure_zero(&g, sizeof(g));
      hk = gf_mul(hk, p);
    }
    secure_zero(&hk, sizeof(hk));
  }
  // The nibble table of H^16 (the bulk kernel expands it into its LDS byte
  // table, gcm.hip build_g8).
  for (int sq = 0; sq < 4; sq++) p = gf_mul(p, p);
  {
    U128 v[128];
    v[0] = p;
    for (int i = 1; i < 128; i++) v[i] = mulx(v[i - 1]);
    for (int k = 0; k < 16; k++)
      for (int half = 0; half < 2; half++)
        for (int val = 0; val < 16; val++) {
          U128 acc{0, 0};
          for (int t = 0; t < 4; t++)
            if ((val >> (3 - t)) & 1) {
              acc.hi ^= v[8 * k + 4 * half + t].hi;
              acc.lo ^= v[8 * k + 4 * half + t].lo;
            }
          uint8_t b[16];
          store_u128(acc, b);
          for (int j = 0; j < 4; j++)
            out->htab16[2 * k + half][val][j] = load_le32(b + 4 * j);
          secure_zero(b, sizeof(b));
        }
    secure_zero(v, sizeof(v));
  }
  // The reference wipes key state on cleanup (OPENSSL_cleanse); so do the
  // host temporaries here.
  secure_zero(w, sizeof(w));
  secure_zero(hb, sizeof(hb));
  secure_zero(&p, sizeof(p));
  return true;
}

void chacha_key_setup(const uint8_t *key, ChaChaKeyDev *out) {
  for (int i = 0; i < 8; i++) out->k[i] = load_le32(key + 4 * i);
}

}  // namespace bssl_amd
