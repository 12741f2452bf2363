// gcm_common.h -- device helpers shared by the AES-GCM bulk kernels: the
// T-table engine (gcm.hip) and the table-free bitsliced engine (gcm_bs.hip).
// Record layout and liveness, the record start (J0, the AD hash), GHASH by
// the lane-rotated LDS byte table of H^L, the record end (lane combine, tag,
// check, zero-fill) and the 16-byte block loads/stores.  Reference anchors
// are at each function (crypto/fipsmodule/aes/gcm.cc.inc,
// crypto/fipsmodule/cipher/e_aes.cc.inc, aead.cc.inc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf128_ct.h"
#include "internal.h"
#include "iov_dev.h"

namespace bssl_amd {
namespace {

// The GHASH byte table of H^L: (byte value e at byte position p) x H^L at
// kLdsG8 + e*256 + p*16 (16 positions side by side in one 256-byte row, so 16
// lanes reading 16 different positions never share a bank).
constexpr uint32_t kLdsG8 = 0;
constexpr uint32_t kG8Bytes = 256 * 256;

__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) {
  return __builtin_amdgcn_alignbit(v, v, 32 - n);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32, gfx950
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__device__ __forceinline__ uint4 xor4_3(uint4 a, uint4 b, uint4 c) {
  return make_uint4(xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y), xor3(a.z, b.z, c.z),
                    xor3(a.w, b.w, c.w));
}

// GHASH multiply by H^16 with the lane-rotated byte table (kLdsG8), spread
// over the AES rounds of the same iteration.  Lane q (its index within the
// record's 16 lanes) looks up byte position (t + q) mod 16 in step t, so the
// 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,
// 28-31}, +32) read 16 different 16-byte slots of the 256-byte row: no bank
// conflicts, 16 lookups per block instead of 32 nibble lookups.  The input is
// rotated by q bytes once (r), so step t takes byte t of r with a
// wave-uniform selector; P[k] byte i holds the slot offset ((4k+i+q) mod 16)*16.
struct Gh8 {
  uint32_t r0, r1, r2, r3;  // multiplier input, rotated down by q bytes
  uint4 g;                  // running sum of the looked-up products
};

// r byte t = x byte (t + q) mod 16, q = 4*s + bsh (s1 = s&1, s2 = s&2).
__device__ __forceinline__ void g8_rotate(Gh8 &h, uint4 x, bool s1, bool s2, uint32_t bsh) {
  const uint32_t e0 = s1 ? x.y : x.x, e1 = s1 ? x.z : x.y, e2 = s1 ? x.w : x.z,
                 e3 = s1 ? x.x : x.w;
  const uint32_t d0 = s2 ? e2 : e0, d1 = s2 ? e3 : e1, d2 = s2 ? e0 : e2, d3 = s2 ? e1 : e3;
  h.r0 = __builtin_amdgcn_alignbyte(d1, d0, bsh);
  h.r1 = __builtin_amdgcn_alignbyte(d2, d1, bsh);
  h.r2 = __builtin_amdgcn_alignbyte(d3, d2, bsh);
  h.r3 = __builtin_amdgcn_alignbyte(d0, d3, bsh);
}

template <int T>
__device__ __forceinline__ uint4 g8_load(const Gh8 &h, const uint32_t (&P)[4],
                                         const uint8_t *smem) {
  const uint32_t r = T < 4 ? h.r0 : T < 8 ? h.r1 : T < 12 ? h.r2 : h.r3;
  const uint32_t a =
      __builtin_amdgcn_perm(r, P[T >> 2], 0x0c0c0000u | ((4u + (T & 3)) << 8) | (T & 3));
  return *reinterpret_cast<const uint4 *>(smem + kLdsG8 + a);
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 as_uint4(v4u v) { return make_uint4(v.x, v.y, v.z, v.w); }

// Materializes v here: an empty volatile asm using it keeps hipcc from
// sinking the XORs that produce it past the following asm rounds (which
// would keep every round's 16-byte GHASH reads live at once).
__device__ __forceinline__ void pin4(uint4 &v) {
  asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

// GHASH byte-table selector of step T (see g8_load).
template <int T>
constexpr uint32_t g8_sel() {
  return 0x0c0c0000u | ((4u + (T & 3)) << 8) | (T & 3);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) {
  return __builtin_amdgcn_perm(0, v, 0x00010203u);
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// The per-record reductions of the bulk kernel use readlane / DPP rather than
// LDS shuffles (ds_bpermute goes through the LDS queue, which the AES and
// GHASH lookups of the other waves keep ~84 % busy, and its lane-index
// operands were spilled and reloaded once per unit).

// Maximum over the wave of a value that is uniform within each L-lane group
// (a record's iteration count): one readlane per group.
template <int L>
__device__ __forceinline__ int group_max(int v) {
  int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
  for (int k = 1; k < 64 / L; k++) m = max(m, __builtin_amdgcn_readlane(v, k * L));
  return m;
}

// XOR of a word over the 16 lanes of its row, in every lane of the row:
// rotations by 8 and 4 within the row, then the quad permutations 1032 and
// 2301 (DPP row_ror / quad_perm; XOR is commutative, so rotations reduce as
// well as butterflies do).
__device__ __forceinline__ uint32_t row_xor16(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);   // quad 2301
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);   // quad 1032
  return v;
}

// len = the record's `in` bytes; xlen = extra bytes sealed after them
// (BatchDesc::extra), so the message is len + xlen bytes.
struct RecordMeta {
  uint64_t off, len, ad_off, ad_len;
  uint32_t xlen;
};

// Per-record arrays read without branches when the batch has any: a missing
// array (null pointer, the uniform-layout field applies) is read at kMetaZero
// instead, so the loads are issued together (under per-array null-pointer
// branches hipcc waited for each load before issuing the next).  A batch with
// none of them takes the uniform layout with no loads at all.
__device__ const uint64_t kMetaZero[2] = {0, 0};

template <typename T>
__device__ __forceinline__ T meta_load(const T *arr, uint64_t i) {
  const T *p = arr ? arr + i : reinterpret_cast<const T *>(kMetaZero);
  return *p;
}

__device__ __forceinline__ RecordMeta record_meta(const BatchDesc &b, uint64_t i) {
  RecordMeta m;
  if (!(b.offsets || b.lengths || b.ad_offsets || b.ad_lengths)) {  // uniform layout: no loads
    m.off = i * b.record_stride;
    m.len = b.record_len;
    m.ad_off = i * b.ad_stride;
    m.ad_len = b.ad_len;
    m.xlen = b.extra_len;
    return m;
  }
  const uint64_t off = meta_load(b.offsets, i), len = meta_load(b.lengths, i);
  const uint64_t ado = meta_load(b.ad_offsets, i), adl = meta_load(b.ad_lengths, i);
  m.off = b.offsets ? off : i * b.record_stride;
  m.len = b.lengths ? len : b.record_len;
  m.ad_off = b.ad_offsets ? ado : i * b.ad_stride;
  m.ad_len = b.ad_lengths ? adl : b.ad_len;
  m.xlen = b.extra_len;
  return m;
}

// Bytes [p0, p0 + n) of a record's message: `in` bytes below len, then the
// extra bytes (load), and the same split for the output (store).
__device__ __forceinline__ uint4 load_partial_x(const uint8_t *src, uint64_t len,
                                                const uint8_t *x, uint64_t p0, uint32_t n) {
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t k = p0 + i;
    w[i >> 2] |= (uint32_t)(k < len ? src[k] : x[k - len]) << (8 * (i & 3));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_partial_x(uint8_t *dst, uint64_t len, uint8_t *x,
                                                uint64_t p0, uint4 v, uint32_t n) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t k = p0 + i;
    const uint8_t c = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    if (k < len)
      dst[k] = c;
    else
      x[k - len] = c;
  }
}

// The block of a record that reaches into its extra bytes (one per record at
// most; only in the XT kernels).  Returns the masked output block; `x`
// receives the input block.
__device__ __forceinline__ uint4 crypt_partial_x(const uint8_t *src, uint8_t *dst, uint64_t len,
                                              const uint8_t *xin, uint8_t *xout, uint64_t p0,
                                              uint4 ks, uint32_t n, uint4 &x) {
  x = load_partial_x(src, len, xin, p0, n);
  const uint4 y = mask_block(make_uint4(x.x ^ ks.x, x.y ^ ks.y, x.z ^ ks.z, x.w ^ ks.w), n);
  store_partial_x(dst, len, xout, p0, y, n);
  return y;
}

// 16-byte block loads and stores at any address (u32_any, iov_dev.h).

__device__ __forceinline__ uint4 load_blk_nt(const uint8_t *p) {
  const BSSL_GLOBAL u32_any *ip = (const BSSL_GLOBAL u32_any *)p;
  return make_uint4(__builtin_nontemporal_load(ip), __builtin_nontemporal_load(ip + 1),
                    __builtin_nontemporal_load(ip + 2), __builtin_nontemporal_load(ip + 3));
}

__device__ __forceinline__ void store_blk(uint8_t *p, uint4 y) {
  BSSL_GLOBAL u32_any *o = (BSSL_GLOBAL u32_any *)p;
  o[0] = y.x;
  o[1] = y.y;
  o[2] = y.z;
  o[3] = y.w;
}

__device__ __forceinline__ void store_blk_nt(uint8_t *p, uint4 y) {
  BSSL_GLOBAL u32_any *o = (BSSL_GLOBAL u32_any *)p;
#ifdef BSSL_PLAIN_STORES  // (A/B builds: temporal stores)
  o[0] = y.x;
  o[1] = y.y;
  o[2] = y.z;
  o[3] = y.w;
#else
  __builtin_nontemporal_store(y.x, o);
  __builtin_nontemporal_store(y.y, o + 1);
  __builtin_nontemporal_store(y.z, o + 2);
  __builtin_nontemporal_store(y.w, o + 3);
#endif
}

// Record at processing position i (sched.hip's length order, if any).
__device__ __forceinline__ uint64_t rec_at(const BatchDesc &b, uint64_t i) {
  return b.order ? (uint64_t)b.order[i] : i;  // (one load; no order array: none)
}


// XOR of a word over the L lanes of its group (L = 16: row_xor16; L = 8:
// row_half_mirror then the quad permutations; L = 4: the quad permutations;
// L = 2: the quad permutation 1032),
// in every lane of the group.
template <int L>
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
  static_assert(L == 16 || L == 8 || L == 4 || L == 2, "lanes per record");
  if constexpr (L == 16) return row_xor16(v);
  if constexpr (L == 2)
    return v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);  // quad 1032
  if constexpr (L == 8)
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // half mirror
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);    // quad 2301
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);    // quad 1032
  return v;
}

// Kernel block words (the 16 block bytes as 4 little-endian words) <-> the
// reversed domain of gf128_ct.h (the big-endian integer of the bytes).
__device__ __forceinline__ Gf128 to_gf(uint4 v) {
  Gf128 g;
  g.w[3] = bswap32(v.x);
  g.w[2] = bswap32(v.y);
  g.w[1] = bswap32(v.z);
  g.w[0] = bswap32(v.w);
  return g;
}
__device__ __forceinline__ uint4 from_gf(Gf128 g) {
  return make_uint4(bswap32(g.w[3]), bswap32(g.w[2]), bswap32(g.w[1]), bswap32(g.w[0]));
}
__device__ __forceinline__ Gf128 gf_load(const uint32_t *p) {
  const uint4 v = *reinterpret_cast<const uint4 *>(p);
  Gf128 g;
  g.w[0] = v.x;
  g.w[1] = v.y;
  g.w[2] = v.z;
  g.w[3] = v.w;
  return g;
}
__device__ __forceinline__ Gf128 gf_xor(Gf128 a, Gf128 b) {
  for (int i = 0; i < 4; i++) a.w[i] ^= b.w[i];
  return a;
}

// ---------------------------------------------------------------------------
// Record start inside the bulk kernel (round 4: no prologue kernel, no
// per-record state in HBM): the per-record constant work of
// CRYPTO_gcm128_init_ctx / _aad (gcm.cc.inc:298-398), done by the record's
// L lanes at the start of their unit.

// Whether record `rec` is sealed/opened at all: a valid key index, a nonce
// (e_aes.cc.inc:790), the length limits (gcm.cc.inc:368,409) and the
// tls12/tls13 nonce check (tls_scan.hip, BatchDesc::valid).
__device__ __forceinline__ bool record_live(const BatchDesc &b, uint64_t rec,
                                            const RecordMeta &m) {
  return (!b.key_index || b.key_index[rec] < b.num_keys) && b.nonce_len != 0 &&
         m.len + m.xlen <= ((uint64_t(1) << 36) - 32) && m.ad_len <= (uint64_t(1) << 61) &&
         (!b.valid || b.valid[rec]);
}

// Pre-counter block J0 (gcm.cc.inc:316-338): nonce || be32(1) for 96-bit
// nonces, else GHASH(N || 0^s || [len(N)]_64), computed by every lane of the
// record (constant-time VALU products by H).
__device__ __forceinline__ uint4 record_j0(const BatchDesc &b, uint64_t rec,
                                           const uint32_t (*hp)[4]) {
  const uint8_t *nonce = b.nonces + rec * b.nonce_len;
  if (b.nonce_len == 12) {
    uint4 j0 = load_partial(nonce, 12);
    j0.w = 0x01000000u;  // be32(1)
    return j0;
  }
  const Gf128 h1 = gf_load(hp[1]);
  Gf128 y = {{0, 0, 0, 0}};
  for (uint64_t o = 0; o < b.nonce_len; o += 16)
    y = gf_mul(gf_xor(y, to_gf(load_partial(nonce + o,
                                            (uint32_t)umin64(b.nonce_len - o, 16)))),
               h1);
  const uint64_t bits = b.nonce_len << 3;
  y.w[0] ^= (uint32_t)bits;
  y.w[1] ^= (uint32_t)(bits >> 32);
  return from_gf(gf_mul(y, h1));
}

// Block k (16 bytes, zero-padded) of record rec's AD.
__device__ __forceinline__ uint4 ad_block(const BatchDesc &b, uint64_t rec, const RecordMeta &m,
                                          uint64_t k) {
  const uint64_t o = 16 * k;
  const uint32_t n = (uint32_t)umin64(m.ad_len - o, 16);
  return b.aadvecs ? ivec_load16(b.aadvecs, b.aadvec_start[rec], b.aadvec_start[rec + 1], o, n)
                   : load_partial(b.ad + m.ad_off + o, n);
}

// Exclusive GHASH of the AD, Y_A = sum_k A_k H^(m-1-k) (m AD blocks), in
// every lane of the record's L.  A one-block AD (TLS: 13 bytes) is its own
// hash; longer ADs are shared out like the message: lane q folds blocks
// k = q, q + L, ... by Horner in H^L, weighs its sum by H^(m-1-k_last) and
// the L lanes XOR-reduce (row_xor).  `many`: some record of the wave has a
// multi-block AD (wave-uniform, so the loop below is).
template <int L>
__device__ __forceinline__ uint4 record_ad_hash(const BatchDesc &b, uint64_t rec,
                                                const RecordMeta &m, bool live, bool many,
                                                const uint32_t (*hp)[4]) {
  const uint64_t nad = live ? (m.ad_len + 15) / 16 : 0;
  if (!many) return nad ? ad_block(b, rec, m, 0) : make_uint4(0, 0, 0, 0);
  const uint32_t q = threadIdx.x & (L - 1);
  const Gf128 hl = gf_load(hp[L]);
  Gf128 acc = {{0, 0, 0, 0}};
  uint64_t last = 0;
  const int rounds = group_max<L>((int)((nad + L - 1) / L));
  for (int i = 0; i < rounds; i++) {
    const uint64_t k = q + (uint64_t)L * i;
    if (k < nad) {
      acc = gf_xor(i ? gf_mul(acc, hl) : acc, to_gf(ad_block(b, rec, m, k)));
      last = k;
    }
  }
  const uint32_t e = (uint32_t)(nad - 1 - last) & (L - 1);  // (lanes with no block: acc = 0)
  Gf128 z = e ? gf_mul(acc, gf_load(hp[e])) : acc;
#pragma unroll
  for (int i = 0; i < 4; i++) z.w[i] = row_xor<L>(z.w[i]);
  return from_gf(z);
}

// End of a record (all bulk kernels): combine the 16 lanes' GHASH
// accumulators, form the tag, check it (open), write tag/status, and zero the
// output of a failed record.  Lane algebra: lane q holds the
// virtual elements v = q+1+16i of [Y_A, C_0, ..., C_{nb-1}], Horner'd at
// stride 16, so its accumulator needs weight H^(15-p), p = (q - r + 1) mod 16
// with r = (nb + 1) mod 16 (the lane holding the last element gets H^0).
// Each lane multiplies its accumulator by H^(16-p) -- its weight times the
// tag's first H -- and the 16 products are XOR-reduced:
//   tag = ((Z*H) ^ len block) * H ^ E_K(J0)  (gcm.cc.inc:576-604).
// Both products are constant-time VALU multiplications (gf128_ct.h) by the
// key's prepared powers H^1..H^16 (key->hpow_ct), indexed by lane position
// and record length only; no table is indexed by a secret.
template <bool OPEN, int L>
__device__ __forceinline__ void finish_record(uint4 acc, uint64_t nb, const RecordMeta &m,
                                              uint4 ek0, const BatchDesc &b, uint64_t rec,
                                              bool active, bool live, uint8_t *dst,
                                              const uint32_t (*hp)[4]) {
  const int q = threadIdx.x & (L - 1);
  const int r = (int)((nb + 1) & (L - 1));
  const int p = (q - r + 1) & (L - 1);
  Gf128 z = gf_mul(to_gf(acc), gf_load(hp[L - p]));
#pragma unroll
  for (int i = 0; i < 4; i++) z.w[i] = row_xor<L>(z.w[i]);
  // Length block be64(AD bits) || be64(message bits) in the reversed domain.
  const uint64_t abits = m.ad_len << 3, cbits = (m.len + m.xlen) << 3;
  z.w[0] ^= (uint32_t)cbits;
  z.w[1] ^= (uint32_t)(cbits >> 32);
  z.w[2] ^= (uint32_t)abits;
  z.w[3] ^= (uint32_t)(abits >> 32);
  z = gf_mul(z, gf_load(hp[1]));
  const uint4 tag = xor4(from_gf(z), ek0);

  uint8_t *tagp = batch_tag(b, rec);
  int ok = live;
  if (q == 0) {
    if (OPEN && live) {
      // CRYPTO_memcmp (e_aes.cc.inc:860-864) of the first tag_len bytes: the
      // received tag by dword-aligned loads (one memory round trip; a byte
      // loop cost one round trip per byte), compared as OR of XORs.
      const uint4 t = load_partial(tagp, b.tag_len);
      const uint4 mine = mask_block(tag, b.tag_len);
      ok = ((t.x ^ mine.x) | (t.y ^ mine.y) | (t.z ^ mine.z) | (t.w ^ mine.w)) == 0;
    }
    if (active) {
      if (!OPEN) store_partial(tagp, ok ? tag : make_uint4(0, 0, 0, 0), b.tag_len);
      if (b.status) b.status[rec] = ok ? 1 : 0;
    }
  }
  if (OPEN) ok = __shfl(ok, 0, L);  // (seal: ok = live, the same in every lane)
  // Zero the output of a failed record (aead.cc.inc:132-139, 539-547; an
  // iovec record's chunks, clear_iovec, :310-333).
  if (active && !ok) {
    if (b.iovecs) {
      for (uint64_t c = b.iovec_start[rec]; c < b.iovec_start[rec + 1]; c++) {
        const IovecDev v = b.iovecs[c];
        for (uint64_t i = q; i < v.len; i += L) v.out[i] = 0;
      }
    } else {
      for (uint64_t j = q; j * 16 < m.len; j += L) {
        const uint32_t n = (uint32_t)umin64(m.len - j * 16, 16);
        store_partial(dst + j * 16, make_uint4(0, 0, 0, 0), n);
      }
    }
    if (q == 0)
      for (uint32_t i = 0; i < m.xlen; i++) batch_extra_out(b, rec)[i] = 0;
  }
}


// ---------------------------------------------------------------------------
// A unit's record inputs (one record per L-lane group), issued together at
// the unit's start: layout, liveness, nonce, the first AD block and the
// lane's first plaintext block.  (Loading them one unit ahead, before the
// previous unit's record end, measured slower: the extra live registers
// spilled, configG 687 vs 743 GiB/s; so did claiming the next unit two
// iterations early, 729 vs 758, profiles/r04/.)
struct UnitIn {
  uint64_t rec;
  RecordMeta m;
  uint4 nonce;  // 12-byte nonces: J0 = nonce || be32(1) (words 0..2)
  uint4 ad0;    // AD block 0, zero-padded
  uint4 x0;     // the lane's first plaintext block (full blocks only)
  bool active, live;
};

template <bool XT, bool IOV>
__device__ __forceinline__ void unit_load(UnitIn &u, const BatchDesc &b, uint64_t i, int q,
                                          uint64_t end) {
  u.active = i < end;
  u.rec = u.active ? rec_at(b, i) : 0;
  u.m = {0, 0, 0, 0, 0};
  u.live = false;
  if (u.active) {
    u.m = record_meta(b, u.rec);
    u.live = record_live(b, u.rec, u.m);
  }
  if constexpr (!XT) u.m.xlen = 0;  // (the launcher picks XT iff extra_len != 0)
  // (Left undefined when not loaded, as load_full's blocks.)
  if (u.live && b.nonce_len == 12) u.nonce = load_partial(b.nonces + u.rec * 12, 12);
  u.ad0 = make_uint4(0, 0, 0, 0);
  if (u.live && u.m.ad_len) u.ad0 = ad_block(b, u.rec, u.m, 0);
  if constexpr (!IOV)
    if (u.live && (uint64_t)q < u.m.len / 16) u.x0 = load_blk_nt(b.in + u.m.off + 16 * q);
}

// Byte table of H^16 from the key's nibble tables (power 4): entry (e, p) =
// T[2p][e >> 4] ^ T[2p+1][e & 15] (key_setup.cc layout), at kLdsG8 + e*256 +
// p*16.  Thread tid writes entries tid + i*kThreads; since kThreads is a
// multiple of 256 its p and (e & 15) are fixed and e >> 4 steps by
// kThreads/256, so all of its global loads are issued before the first LDS
// write (one memory latency per key change instead of one per entry).
template <int THREADS>
__device__ __forceinline__ void build_g8(uint8_t *smem, const uint4 *__restrict__ t16, int tid) {
  if constexpr (4096 % THREADS != 0) {  // (any other workgroup size: entry by entry)
    for (int e = tid; e < 4096; e += THREADS) {
      const uint32_t p = (uint32_t)e & 15u, lo = ((uint32_t)e >> 4) & 15u, hi = (uint32_t)e >> 8;
      reinterpret_cast<uint4 *>(smem + kLdsG8)[e] =
          xor4(t16[(2 * p) * 16 + hi], t16[(2 * p + 1) * 16 + lo]);
    }
    return;
  }
  static_assert(THREADS % 256 == 0, "table build split");
  constexpr int kPer = 4096 / THREADS;
  const uint32_t p = (uint32_t)tid & 15u, lo = ((uint32_t)tid >> 4) & 15u;
  const uint32_t hi = (uint32_t)tid >> 8;
  const uint4 b = t16[(2 * p + 1) * 16 + lo];
  uint4 a[kPer];
#pragma unroll
  for (int i = 0; i < kPer; i++) a[i] = t16[(2 * p) * 16 + hi + (uint32_t)i * (THREADS / 256)];
#pragma unroll
  for (int i = 0; i < kPer; i++)
    reinterpret_cast<uint4 *>(smem + kLdsG8)[tid + i * THREADS] = xor4(a[i], b);
}

// Byte table of H^L (L < 16: the short-record kernels, whose GHASH stride is
// L) computed in the kernel from the key's prepared H^L (hpow_ct[L]): the
// 128 basis products (bit `bit` of byte p) x H^L by 128 threads with the
// constant-time VALU product, then entry (e, p) = XOR of the basis elements
// of p for the bits of e (e and p are table indices, public).
// BASIS: LDS offset of a 2 KiB scratch for the basis products.
template <int THREADS, uint32_t BASIS>
__device__ __forceinline__ void build_gpow(uint8_t *smem, const uint32_t *hl, int tid) {
  static_assert(THREADS >= 128 && 4096 % THREADS == 0, "table build split");
  uint4 *basis = reinterpret_cast<uint4 *>(smem + BASIS);
  if (tid < 128) {
    const uint32_t p = (uint32_t)tid >> 3, bit = (uint32_t)tid & 7u;
    uint32_t w[4] = {0, 0, 0, 0};
    w[p >> 2] = 1u << (8 * (p & 3) + bit);
    basis[tid] = from_gf(gf_mul(to_gf(make_uint4(w[0], w[1], w[2], w[3])), gf_load(hl)));
  }
  __syncthreads();
  const uint32_t p = (uint32_t)tid & 15u;
  uint4 bv[8];
#pragma unroll
  for (int k = 0; k < 8; k++) bv[k] = basis[p * 8 + k];
#pragma unroll
  for (int i = 0; i < 4096 / THREADS; i++) {
    const uint32_t e = ((uint32_t)tid >> 4) + (uint32_t)i * (THREADS / 16);
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t msk = 0u - ((e >> k) & 1u);
      v = make_uint4(v.x ^ (bv[k].x & msk), v.y ^ (bv[k].y & msk), v.z ^ (bv[k].z & msk),
                     v.w ^ (bv[k].w & msk));
    }
    reinterpret_cast<uint4 *>(smem + kLdsG8)[tid + i * THREADS] = v;
  }
}

}  // namespace
}  // namespace bssl_amd
