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

#include "internal.h"

namespace bssl_amd {
namespace {

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kRecPerWave = 4;
constexpr int kRecPerTile = kWaves * kRecPerWave;  // 32

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
// LDS.
constexpr int kGhashLdsBytes = kGhashPowers * 8192;  // 40 KiB
constexpr int kAesLdsBytes = 256 * 256;              // 64 KiB

__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) {
  return __builtin_amdgcn_alignbit(v, v, 32 - n);
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *base, uint32_t off) {
  return *reinterpret_cast<const uint32_t *>(base + off);
}

__device__ __forceinline__ uint4 lds_u128(const uint8_t *base, uint32_t off) {
  return *reinterpret_cast<const uint4 *>(base + off);
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// ---------------------------------------------------------------------------
// AES.  State: 4 little-endian column words (byte r of word c = row r).
// Lookup address of T(slot) entry for state byte k: v_perm puts byte k at
// bits 8..15 and the lane/slot constant `lc` (bits 0..7) below it.
template <int K>
__device__ __forceinline__ uint32_t taddr(uint32_t lc, uint32_t s) {
  return __builtin_amdgcn_perm(lc, s, 0x0c0c0004u | (K << 8));
}

// One full round column: rows come from columns (a, b, c, d); rkx is the round
// key word pre-rotated by 16.
__device__ __forceinline__ uint32_t round_col(const uint8_t *T, uint32_t lc0,
                                              uint32_t lc1, uint32_t a,
                                              uint32_t b, uint32_t c,
                                              uint32_t d, uint32_t rkx) {
  uint32_t x0 = lds_u32(T, taddr<0>(lc0, a));
  uint32_t x1 = lds_u32(T, taddr<1>(lc1, b));
  uint32_t x2 = lds_u32(T, taddr<2>(lc0, c));
  uint32_t x3 = lds_u32(T, taddr<3>(lc1, d));
  return x0 ^ x1 ^ rotl(x2 ^ x3 ^ rkx, 16);
}

__device__ __forceinline__ uint32_t last_col(const uint8_t *T, uint32_t lc0,
                                             uint32_t a, uint32_t b,
                                             uint32_t c, uint32_t d,
                                             uint32_t rk) {
  uint32_t x0 = lds_u32(T, taddr<0>(lc0, a));
  uint32_t x1 = lds_u32(T, taddr<1>(lc0, b));
  uint32_t x2 = lds_u32(T, taddr<2>(lc0, c));
  uint32_t x3 = lds_u32(T, taddr<3>(lc0, d));
  // S[x] is byte 1 (and byte 2) of Te0[x].
  uint32_t lo = __builtin_amdgcn_perm(x1, x0, 0x0c0c0501u);
  uint32_t hi = __builtin_amdgcn_perm(x3, x2, 0x06020c0cu);
  return lo ^ hi ^ rk;
}

struct RoundKeys {
  uint32_t w[15][4];
};

template <int NR>
__device__ __forceinline__ uint4 aes_encrypt(uint4 in, const RoundKeys &rk,
                                             const uint8_t *T, uint32_t lc0,
                                             uint32_t lc1) {
  uint32_t s0 = in.x ^ rk.w[0][0], s1 = in.y ^ rk.w[0][1];
  uint32_t s2 = in.z ^ rk.w[0][2], s3 = in.w ^ rk.w[0][3];
#pragma unroll
  for (int r = 1; r < NR; r++) {
    uint32_t t0 = round_col(T, lc0, lc1, s0, s1, s2, s3, rk.w[r][0]);
    uint32_t t1 = round_col(T, lc0, lc1, s1, s2, s3, s0, rk.w[r][1]);
    uint32_t t2 = round_col(T, lc0, lc1, s2, s3, s0, s1, rk.w[r][2]);
    uint32_t t3 = round_col(T, lc0, lc1, s3, s0, s1, s2, rk.w[r][3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  uint4 o;
  o.x = last_col(T, lc0, s0, s1, s2, s3, rk.w[NR][0]);
  o.y = last_col(T, lc0, s1, s2, s3, s0, rk.w[NR][1]);
  o.z = last_col(T, lc0, s2, s3, s0, s1, rk.w[NR][2]);
  o.w = last_col(T, lc0, s3, s0, s1, s2, rk.w[NR][3]);
  return o;
}

// ---------------------------------------------------------------------------
// GHASH: x * H^(2^p) with the nibble tables of power p at `tab` (LDS).
__device__ __forceinline__ uint4 gmul(uint4 x, const uint8_t *tab) {
  uint4 r = make_uint4(0, 0, 0, 0);
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t v = w[k >> 2];
    const int sh = 8 * (k & 3);
    const uint32_t hi = (v >> sh) & 0xf0u;
    const uint32_t lo = (sh >= 4 ? (v >> (sh - 4)) : (v << 4)) & 0xf0u;
    r = xor4(r, lds_u128(tab, (2 * k) * 256 + hi));
    r = xor4(r, lds_u128(tab, (2 * k + 1) * 256 + lo));
  }
  return r;
}

__device__ __forceinline__ uint4 shfl4(uint4 v, int src, int width) {
  return make_uint4(__shfl(v.x, src, width), __shfl(v.y, src, width),
                    __shfl(v.z, src, width), __shfl(v.w, src, width));
}

__device__ __forceinline__ uint4 shfl_down4(uint4 v, int d, int width) {
  return make_uint4(__shfl_down(v.x, d, width), __shfl_down(v.y, d, width),
                    __shfl_down(v.z, d, width), __shfl_down(v.w, d, width));
}

// Combine the 16 per-lane Horner accumulators of a group.  Lane q's
// accumulator must be weighted by H^e with e = (r - 1 - v) mod 16 where v is
// the lane's virtual index (see DESIGN.md "GHASH lane algebra").  `src` is the
// lane whose accumulator goes to position q.  Result valid in every lane.
// Must be called with all 64 lanes active.
__device__ __forceinline__ uint4 group_combine(uint4 acc, int q, int src,
                                               const uint8_t *gtab) {
  uint4 a = shfl4(acc, src, 16);
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int s = 1 << t;
    uint4 m = gmul(a, gtab + t * 8192);
    uint4 o = shfl_down4(a, s, 16);
    if ((q & (2 * s - 1)) == 0) a = xor4(m, o);
  }
  return shfl4(a, 0, 16);
}

// ---------------------------------------------------------------------------
// Record buffers.
__device__ __forceinline__ uint4 load_partial(const uint8_t *p, uint32_t n) {
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < n; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_partial(uint8_t *p, uint4 v, uint32_t n) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t i = 0; i < n; i++) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ uint4 mask_block(uint4 v, uint32_t n) {
  if (n >= 16) return v;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int lo = 4 * i;
    uint32_t m = (n >= (uint32_t)lo + 4) ? 0xffffffffu
                 : (n <= (uint32_t)lo) ? 0u
                                       : ((1u << (8 * (n - lo))) - 1u);
    w[i] &= m;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) {
  return __builtin_amdgcn_perm(0, v, 0x00010203u);
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// Exclusive Horner (sum_k B_k H^(m-1-k)) of the zero-padded 16-byte blocks of
// `len` bytes at p, optionally followed by one extra block; all lanes of the
// group return the value.  All 64 lanes must call it.
__device__ uint4 group_ghash(const uint8_t *p, uint64_t len, bool has_extra,
                             uint4 extra, bool active, int q,
                             const uint8_t *gtab) {
  const uint64_t nb = active ? (len + 15) / 16 + (has_extra ? 1 : 0) : 0;
  const int wmax = wave_max((int)min<uint64_t>(nb, 0x7fffffff));
  if (wmax <= 1) {
    // Single block: no multiplication needed.
    uint4 b0 = make_uint4(0, 0, 0, 0);
    if (nb == 1) b0 = len ? load_partial(p, (uint32_t)min<uint64_t>(len, 16)) : extra;
    return b0;
  }
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t k = q; k < nb; k += 16) {
    uint4 blk;
    if (k * 16 < len) {
      const uint64_t rem = len - k * 16;
      blk = load_partial(p + k * 16, (uint32_t)min<uint64_t>(rem, 16));
    } else {
      blk = extra;
    }
    acc = xor4(gmul(acc, gtab + 4 * 8192), blk);
  }
  const int r = (int)(nb & 15);
  return group_combine(acc, q, (q + r) & 15, gtab);
}

struct RecordMeta {
  uint64_t off, len, ad_off, ad_len;
};

__device__ __forceinline__ RecordMeta record_meta(const BatchDesc &b, uint64_t i) {
  RecordMeta m;
  m.off = b.offsets ? b.offsets[i] : i * b.record_stride;
  m.len = b.lengths ? b.lengths[i] : b.record_len;
  m.ad_off = b.ad_offsets ? b.ad_offsets[i] : i * b.ad_stride;
  m.ad_len = b.ad_lengths ? b.ad_lengths[i] : b.ad_len;
  return m;
}

// ---------------------------------------------------------------------------
// Process the (up to) 4 records of this wave.  `active` is per group.
template <int NR, bool OPEN>
__device__ void process_records(const RoundKeys &rk, const BatchDesc &b,
                                uint64_t rec, bool active, bool bad_key,
                                const uint8_t *gtab, const uint8_t *T,
                                uint32_t lc0, uint32_t lc1) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 15;
  RecordMeta m = {0, 0, 0, 0};
  if (active) m = record_meta(b, rec);
  // gcm.cc.inc:409 message limit 2^36-32; e_aes.cc.inc:790 empty nonce.
  const bool bad = active && (bad_key || b.nonce_len == 0 ||
                              m.len > ((uint64_t(1) << 36) - 32) ||
                              m.ad_len > (uint64_t(1) << 61));
  const bool live = active && !bad;
  const uint8_t *nonce = b.nonces + (live ? rec * b.nonce_len : 0);

  // J0 (gcm.cc.inc:316-338).
  uint4 j0;
  {
    const bool std_iv = b.nonce_len == 12;
    uint4 lenblk = make_uint4(0, 0, 0, bswap32((uint32_t)(b.nonce_len << 3)));
    lenblk.z = bswap32((uint32_t)(b.nonce_len >> 29));
    uint4 y = group_ghash(nonce, std_iv ? 0 : b.nonce_len, true, lenblk,
                          live && !std_iv, q, gtab);
    if (std_iv) {
      j0 = live ? load_partial(nonce, 12) : make_uint4(0, 0, 0, 0);
      j0.w = 0x01000000u;  // be32(1)
    } else {
      j0 = gmul(y, gtab);  // GHASH = H * (exclusive Horner)
    }
  }
  const uint32_t ctr0 = bswap32(j0.w);
  const uint4 ek0 = aes_encrypt<NR>(j0, rk, T, lc0, lc1);

  // AAD (gcm.cc.inc:346-398).
  const uint4 ya = group_ghash(b.ad + (live ? m.ad_off : 0), live ? m.ad_len : 0, false,
                               make_uint4(0, 0, 0, 0), live, q, gtab);

  // Bulk CTR + GHASH (gcm.cc.inc:400-574).
  const uint64_t nb = live ? (m.len + 15) / 16 : 0;
  const uint8_t *src = b.in + m.off;
  uint8_t *dst = b.out + m.off;
  const bool aligned = ((reinterpret_cast<uintptr_t>(src) |
                         reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  uint4 acc = (q == 15 && live) ? ya : make_uint4(0, 0, 0, 0);
  const uint8_t *h16 = gtab + 4 * 8192;
  const int iters = wave_max((int)((nb + 15) / 16));
  for (int it = 0; it < iters; it++) {
    const uint64_t j = (uint64_t)it * 16 + q;
    const uint32_t ctr = ctr0 + 1u + (uint32_t)j;  // inc32 wraps mod 2^32
    const uint4 ks = aes_encrypt<NR>(make_uint4(j0.x, j0.y, j0.z, bswap32(ctr)), rk, T,
                                     lc0, lc1);
    if (j < nb) {
      const uint64_t rem = m.len - j * 16;
      uint4 x, y;
      if (rem >= 16 && aligned) {
        x = *reinterpret_cast<const uint4 *>(src + j * 16);
        y = xor4(x, ks);
        *reinterpret_cast<uint4 *>(dst + j * 16) = y;
      } else {
        const uint32_t n = (uint32_t)min<uint64_t>(rem, 16);
        x = load_partial(src + j * 16, n);
        y = mask_block(xor4(x, ks), n);
        store_partial(dst + j * 16, y, n);
      }
      acc = xor4(gmul(acc, h16), OPEN ? x : y);
    }
  }
  const int r = (int)((nb + 1) & 15);
  const uint4 z = group_combine(acc, q, (q + r + 15) & 15, gtab);

  // Tag (gcm.cc.inc:576-604): ((Z*H) ^ len block) * H ^ E_K(J0).
  const uint64_t abits = m.ad_len << 3, cbits = m.len << 3;
  const uint4 lb = make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                              bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits));
  const uint4 tag = xor4(gmul(xor4(gmul(z, gtab), lb), gtab), ek0);

  uint8_t *tagp = b.tags + rec * b.tag_len;
  bool ok = live;
  if (OPEN && live) {
    const uint32_t tw[4] = {tag.x, tag.y, tag.z, tag.w};
    uint32_t diff = 0;
    for (uint32_t i = 0; i < b.tag_len; i++)
      diff |= ((tw[i >> 2] >> (8 * (i & 3))) & 0xff) ^ tagp[i];
    ok = diff == 0;  // CRYPTO_memcmp, e_aes.cc.inc:860-864
  }
  if (active && q == 0) {
    if (!OPEN) {
      if (ok)
        store_partial(tagp, tag, b.tag_len);
      else
        for (uint32_t i = 0; i < b.tag_len; i++) tagp[i] = 0;
    }
    if (b.status) b.status[rec] = ok ? 1 : 0;
  }
  // Zero the output of a failed record (aead.cc.inc:132-139, 539-547).
  if (active && !ok) {
    for (uint64_t j = q; j * 16 < m.len; j += 16) {
      const uint32_t n = (uint32_t)min<uint64_t>(m.len - j * 16, 16);
      store_partial(dst + j * 16, make_uint4(0, 0, 0, 0), n);
    }
  }
}

template <int NR, bool OPEN>
__global__ __launch_bounds__(kThreads) void gcm_kernel(const GcmKeyDev *__restrict__ keys,
                                                      BatchDesc b) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ghash[kGhashLdsBytes];
  __shared__ __attribute__((aligned(16))) uint8_t s_aes[kAesLdsBytes];
  __shared__ uint32_t s_keys[kRecPerTile];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;

  // AES tables, replicated per bank: entry idx, slot t, lane l at
  // idx*256 + t*128 + l*4.  Slot 1 holds T1 = rotl8(T0).
  for (int e = tid; e < 256 * 64; e += kThreads) {
    const int idx = e >> 6, slot = (e >> 5) & 1;
    const uint32_t v = kTables.te0[idx];
    reinterpret_cast<uint32_t *>(s_aes)[e] = slot ? rotl(v, 8) : v;
  }
  const uint32_t lc0 = (uint32_t)(lane & 31) * 4u;
  const uint32_t lc1 = lc0 + 128u;

  uint32_t loaded = 0xffffffffu;
  RoundKeys rk;
  const uint64_t n = b.num_records;
  for (uint64_t base = (uint64_t)blockIdx.x * kRecPerTile; base < n;
       base += (uint64_t)gridDim.x * kRecPerTile) {
    __syncthreads();
    if (tid < kRecPerTile) {
      const uint64_t i = base + tid;
      s_keys[tid] = i < n ? (b.key_index ? b.key_index[i] : 0u) : 0xffffffffu;
    }
    __syncthreads();
    uint64_t pending = 0;
    for (int t = 0; t < kRecPerTile; t++)
      if (s_keys[t] != 0xffffffffu) pending |= uint64_t(1) << t;
    while (pending) {
      const int first = __builtin_ctzll(pending);
      const uint32_t k = __builtin_amdgcn_readfirstlane(s_keys[first]);
      uint64_t mask = 0;
      for (int t = 0; t < kRecPerTile; t++)
        if (((pending >> t) & 1) && s_keys[t] == k) mask |= uint64_t(1) << t;
      pending &= ~mask;
      const bool bad_key = k >= b.num_keys;
      const uint32_t kk = bad_key ? 0u : k;
      if (kk != loaded) {
        __syncthreads();
        const uint4 *srcp = reinterpret_cast<const uint4 *>(keys[kk].htab);
        for (int e = tid; e < kGhashLdsBytes / 16; e += kThreads)
          reinterpret_cast<uint4 *>(s_ghash)[e] = srcp[e];
        __syncthreads();
        loaded = kk;
#pragma unroll
        for (int r = 0; r <= NR; r++)
#pragma unroll
          for (int c = 0; c < 4; c++) rk.w[r][c] = keys[kk].rk[r][c];
      }
      const int t = wave * kRecPerWave + g;
      const bool active = (mask >> t) & 1;
      process_records<NR, OPEN>(rk, b, base + t, active, bad_key, s_ghash, s_aes, lc0, lc1);
    }
  }
}

int g_num_cus = 0;

template <int NR, bool OPEN>
int launch_nr(const GcmKeyDev *keys, const BatchDesc &b, hipStream_t s) {
  if (!g_num_cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess)
      return 1;
  }
  const uint64_t tiles = (b.num_records + kRecPerTile - 1) / kRecPerTile;
  const unsigned grid = (unsigned)(tiles < (uint64_t)g_num_cus ? tiles : (uint64_t)g_num_cus);
  hipLaunchKernelGGL((gcm_kernel<NR, OPEN>), dim3(grid), dim3(kThreads), 0, s, keys, b);
  return (int)hipGetLastError();
}

}  // namespace

int launch_gcm(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr, void *stream,
               float *timing_ms) {
  if (b.num_records == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timing_ms) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
  }
  int rc;
  switch (nr) {
    case 10: rc = open ? launch_nr<10, true>(keys, b, s) : launch_nr<10, false>(keys, b, s); break;
    case 12: rc = open ? launch_nr<12, true>(keys, b, s) : launch_nr<12, false>(keys, b, s); break;
    case 14: rc = open ? launch_nr<14, true>(keys, b, s) : launch_nr<14, false>(keys, b, s); break;
    default: rc = 1;
  }
  if (timing_ms) {
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    hipEventElapsedTime(timing_ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  return rc;
}

}  // namespace bssl_amd
