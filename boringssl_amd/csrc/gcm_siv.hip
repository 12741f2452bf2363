// gcm_siv.hip -- AES-GCM-SIV (RFC 8452) seal / open over device-resident
// record batches.
//
// Replaces aead_aes_gcm_siv_sealv / _openv_detached
// (crypto/cipher/e_aesgcmsiv.cc:782-867) and their helpers gcm_siv_keys
// (:750-780), gcm_siv_polyval (:686-736) and gcm_siv_crypt (:571-601).
// Design:
// * 16 lanes per record, 16 records per 256-thread workgroup.
// * Per-record keys: lanes 0..3 (0..5 for AES-256) of a record encrypt
//   le32(i) || nonce under the master key (T-table AES, tables in LDS) and the
//   halves are exchanged by shuffles; lane 0 expands the record's encryption
//   key into the record's LDS slot.
// * POLYVAL through GHASH, as the reference computes it (:604-682):
//   H_g = mulX_GHASH(ByteReverse(H)) and every block byte-reversed -- which in
//   big-endian words is the block's little-endian words in reverse order, so
//   it costs nothing.  Products use Shoup's 4-bit method with one 16-entry
//   table per power of H_g in LDS (M[v] = v(x) * H_g^k) and the 4-bit
//   reduction computed arithmetically: 32 dependent nibble steps, no
//   position-dependent tables (which would be 8 KiB per power per record).
//   Lane q folds the elements j = q, q+16, ... of [AD blocks, message blocks,
//   length block] with Horner's rule in H_g^16, multiplies its sum by
//   H_g^(n - j_last) (tables H, H^2, H^4, H^8, H^16) and the 16 lanes are
//   XOR-reduced.
// * Seal: POLYVAL over the plaintext, tag = AES_K'(POLYVAL ^ nonce, bit 127
//   cleared), then CTR from the tag (byte 15 |= 0x80, little-endian 32-bit
//   counter in bytes 0..3): the plaintext is read twice, as SIV requires.
//   Open: CTR and POLYVAL in one pass (the lane that decrypts a block folds
//   it), then the tag compare; a failed record is zero-filled.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "iov_dev.h"

namespace bssl_amd {
namespace {

// AES tables: T0 and T1 = rotl8(T0), each replicated once per LDS bank (entry
// x of table t for lane l at t[x][t][l & 31], 64 KiB), so every lookup of a
// wave is bank-conflict free whatever the (secret) index -- the
// constant-time argument of gcm.hip's tables; T2/T3 are
// rot16(T0/T1), one rotate per column.  (Rounds 1/2 used four plain 1 KiB
// tables, whose bank conflicts depend on the data.)
// Round-1/2 choices kept: the per-block multiply by H^16 as
// four independent Shoup chains (gmul4d, one reduction per chain) instead of
// one 32-step chain; a record's 16 lanes are the 16 lanes of one
// ds_read_b128 lane group ({0-3,12-15,20-27} / {4-11,16-19,28-31}, +32), so
// the Shoup-table reads of a group all hit one record's 256-byte table:
// distinct nibbles are distinct banks, equal ones the same address.  With
// contiguous lanes a group mixes two records' tables and their reads collide.
// And the Shoup step's 4-bit reduction as shifts of the top nibble (red4_hi)
// instead of four multiplies.  (Counter-window caching of rounds 1-2 in the
// seal keystream pass measured no faster, 502-503 vs 505 GiB/s: the
// keystream pass's lookups are not what binds this kernel.)
constexpr int kL = 16;                // lanes per record
// One persistent 768-thread workgroup per CU (12 waves: the 168-VGPR budget's
// 3 waves per SIMD; LDS 64 KiB of tables + 48 record slots = 137 KiB).  Each
// wave takes 4-record units from a grid-wide counter and keeps 4 record slots
// of its own, so waves never wait for each other (a per-workgroup barrier at
// every record start held 48 records in lock-step).
constexpr int kThreads = 768;
constexpr int kRecs = kThreads / kL;  // record slots per workgroup
constexpr int kPows = 5;              // H, H^2, H^4, H^8, H^16

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
    uint8_t inv = 1, base = (uint8_t)x;  // x^254
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
    // bytes (2s, s, s, 3s): the MixColumns column of a row-0 byte
    t.te0[x] = (uint32_t)cx_mul(s, 2) | ((uint32_t)s << 8) | ((uint32_t)s << 16) |
               ((uint32_t)cx_mul(s, 3) << 24);
  }
  return t;
}

__constant__ Tables kSivTables = make_tables();

struct Lds {
  uint32_t t[256][2][32];      // T0 / T1, replica (lane & 31)
  uint4 rk[kRecs][15];         // each record's encryption round keys
  uint4 m[kRecs][kPows][16];   // each record's Shoup tables
};
static_assert(sizeof(Lds) <= 160 * 1024, "LDS per workgroup");

__device__ __forceinline__ uint32_t rotl(uint32_t v, int n) {
  return __builtin_amdgcn_alignbit(v, v, 32 - n);
}

__device__ __forceinline__ uint32_t t0(const Lds &L, uint32_t x) {
  return L.t[x][0][threadIdx.x & 31];
}
__device__ __forceinline__ uint32_t t1(const Lds &L, uint32_t x) {
  return L.t[x][1][threadIdx.x & 31];
}
__device__ __forceinline__ uint32_t sbox(const Lds &L, uint32_t x) {
  return (t0(L, x) >> 8) & 0xff;
}

// Table T_t[x] (T_t = rotl(T0, 8t)).
__device__ __forceinline__ uint32_t tt(const Lds &L, int t, uint32_t x) {
  return t == 0 ? t0(L, x) : t == 1 ? t1(L, x) : rotl(t == 2 ? t0(L, x) : t1(L, x), 16);
}

// FIPS-197 cipher on little-endian column words, from round R0 on (s = the
// state entering round R0); `rk` in LDS or global memory.
template <int NR, int R0>
__device__ __forceinline__ uint4 aes_enc_from(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                              const uint4 *rk, const Lds &L) {
#pragma unroll
  for (int r = R0; r < NR; r++) {
    const uint4 k = rk[r];
    // T0[a] ^ T1[b] ^ T2[c] ^ T3[d] = T0[a] ^ T1[b] ^ rot16(T0[c] ^ T1[d])
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kk) {
      return t0(L, a & 0xff) ^ t1(L, (b >> 8) & 0xff) ^
             rotl(t0(L, (c >> 16) & 0xff) ^ t1(L, d >> 24), 16) ^ kk;
    };
    const uint32_t t0v = col(s0, s1, s2, s3, k.x), t1 = col(s1, s2, s3, s0, k.y),
                   t2 = col(s2, s3, s0, s1, k.z), t3 = col(s3, s0, s1, s2, k.w);
    s0 = t0v; s1 = t1; s2 = t2; s3 = t3;
  }
  const uint4 k = rk[NR];
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return sbox(L, a & 0xff) | (sbox(L, (b >> 8) & 0xff) << 8) |
           (sbox(L, (c >> 16) & 0xff) << 16) | (sbox(L, d >> 24) << 24);
  };
  return make_uint4(last(s0, s1, s2, s3) ^ k.x, last(s1, s2, s3, s0) ^ k.y,
                    last(s2, s3, s0, s1) ^ k.z, last(s3, s0, s1, s2) ^ k.w);
}

template <int NR>
__device__ __forceinline__ uint4 aes_enc(uint4 in, const uint4 *rk, const Lds &L) {
  return aes_enc_from<NR, 1>(in.x ^ rk[0].x, in.y ^ rk[0].y, in.z ^ rk[0].z, in.w ^ rk[0].w, rk,
                             L);
}

// Counter-mode caching for the SIV keystream (Bernstein-Schwabe, as gcm.hip):
// the counter is word 0 + p (little-endian, e_aesgcmsiv.cc:555-580), so within
// a window of 256 counters only state byte 0 changes.  Round 1 then costs one
// lookup (column 0's T0) and round 2 four (one per column, from round-1
// column 0): 5 lookups instead of 32.  The window constants (27 lookups) are
// rebuilt when the high 24 bits of state word 0 change.
struct CtrWindow {
  uint32_t hi = 0xffffffffu;  // (no 24-bit value equals it)
  uint32_t k0, l0, l1, l2, l3;
  __device__ __forceinline__ void update(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                         const uint4 *rk, const Lds &L) {
    if ((s0 >> 8) == hi) return;
    hi = s0 >> 8;
    const uint4 a = rk[1], c = rk[2];
    k0 = tt(L, 1, (s1 >> 8) & 0xff) ^ tt(L, 2, (s2 >> 16) & 0xff) ^ tt(L, 3, s3 >> 24) ^ a.x;
    const uint32_t t1 = tt(L, 0, s1 & 0xff) ^ tt(L, 1, (s2 >> 8) & 0xff) ^
                        tt(L, 2, (s3 >> 16) & 0xff) ^ tt(L, 3, s0 >> 24) ^ a.y;
    const uint32_t t2 = tt(L, 0, s2 & 0xff) ^ tt(L, 1, (s3 >> 8) & 0xff) ^
                        tt(L, 2, (s0 >> 16) & 0xff) ^ tt(L, 3, s1 >> 24) ^ a.z;
    const uint32_t t3 = tt(L, 0, s3 & 0xff) ^ tt(L, 1, (s0 >> 8) & 0xff) ^
                        tt(L, 2, (s1 >> 16) & 0xff) ^ tt(L, 3, s2 >> 24) ^ a.w;
    l0 = tt(L, 1, (t1 >> 8) & 0xff) ^ tt(L, 2, (t2 >> 16) & 0xff) ^ tt(L, 3, t3 >> 24) ^ c.x;
    l1 = tt(L, 0, t1 & 0xff) ^ tt(L, 1, (t2 >> 8) & 0xff) ^ tt(L, 2, (t3 >> 16) & 0xff) ^ c.y;
    l2 = tt(L, 0, t2 & 0xff) ^ tt(L, 1, (t3 >> 8) & 0xff) ^ tt(L, 3, t1 >> 24) ^ c.z;
    l3 = tt(L, 0, t3 & 0xff) ^ tt(L, 2, (t1 >> 16) & 0xff) ^ tt(L, 3, t2 >> 24) ^ c.w;
  }
  // Keystream block for state word 0 = s0 (in this window).
  template <int NR>
  __device__ __forceinline__ uint4 block(uint32_t s0, const uint4 *rk, const Lds &L) const {
    const uint32_t t0 = k0 ^ tt(L, 0, s0 & 0xff);
    return aes_enc_from<NR, 3>(l0 ^ tt(L, 0, t0 & 0xff), l1 ^ tt(L, 3, t0 >> 24),
                               l2 ^ tt(L, 2, (t0 >> 16) & 0xff), l3 ^ tt(L, 1, (t0 >> 8) & 0xff),
                               rk, L);
  }
};

// ---- GF(2^128) in GCM order, as big-endian words (w0 = bytes 0..3) --------

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// * x (shift right by one, reduce by 0xe1 || 0^120).
__device__ __forceinline__ uint4 mulx(uint4 v) {
  const uint32_t red = (v.w & 1) ? 0xe1000000u : 0u;
  return make_uint4((v.x >> 1) ^ red, (v.y >> 1) | (v.x << 31), (v.z >> 1) | (v.y << 31),
                    (v.w >> 1) | (v.z << 31));
}

// red4(z3 & 0xf) << 16 without the multiplies: with u = z3 << 28 (the four
// bits at the top), clmul(r, 0x1c20) << 16 = r<<28 ^ r<<27 ^ r<<26 ^ r<<21
// = u ^ u>>1 ^ u>>2 ^ u>>7 (0x1c20 = bits 5, 10, 11, 12).
__device__ __forceinline__ uint32_t red4_hi(uint32_t z3) {
  const uint32_t u = z3 << 28;
  return u ^ (u >> 1) ^ (u >> 2) ^ (u >> 7);
}

// X * H^k with M = the 16-entry table of H^k (Shoup 4-bit, nibbles from the
// highest-degree one down).
__device__ __forceinline__ uint4 gmul(uint4 X, const uint4 *M) {
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  const uint32_t w[4] = {X.x, X.y, X.z, X.w};
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    const uint32_t nib = (w[k >> 3] >> (28 - 4 * (k & 7))) & 0xf;
    const uint32_t r = red4_hi(z3);
    z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
    z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
    z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
    z0 = (z0 >> 4) ^ r;
    const uint4 m = M[nib];
    z0 ^= m.x; z1 ^= m.y; z2 ^= m.z; z3 ^= m.w;
    if ((k & 7) == 0) __builtin_amdgcn_sched_barrier(0);
  }
  return make_uint4(z0, z1, z2, z3);
}

// X * x^32: one word down, the 32 bits shifted out of the top reduced by
// x^128 = 1 + x + x^2 + x^7 (as mulx, 32 bits at once).
__device__ __forceinline__ uint4 mulx32(uint4 z) {
  const uint32_t s = z.w;
  return make_uint4(s ^ (s >> 1) ^ (s >> 2) ^ (s >> 7), z.x ^ (s << 31) ^ (s << 30) ^ (s << 25),
                    z.y, z.z);
}


// gmul4 with the reduction deferred: each 8-step chain shifts its 32
// spilled bits into a fifth word instead of reducing 4 bits per step, and
// reduces them once at the end (x^128 = 1 + x + x^2 + x^7, as mulx32; the
// reduced terms stay below degree 39 + 28, so no second reduction).  Per
// step: 4 funnel shifts, 1 shift and 4 XORs.
__device__ __forceinline__ uint4 gmul4d(uint4 X, const uint4 *M) {
  uint32_t z[4][5];
  const uint32_t w[4] = {X.x, X.y, X.z, X.w};
#pragma unroll
  for (int g = 0; g < 4; g++) z[g][0] = z[g][1] = z[g][2] = z[g][3] = z[g][4] = 0;
#pragma unroll
  for (int k = 7; k >= 0; k--) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const uint32_t nib = (w[g] >> (28 - 4 * k)) & 0xf;
      z[g][4] = __builtin_amdgcn_alignbit(z[g][3], z[g][4], 4);
      z[g][3] = __builtin_amdgcn_alignbit(z[g][2], z[g][3], 4);
      z[g][2] = __builtin_amdgcn_alignbit(z[g][1], z[g][2], 4);
      z[g][1] = __builtin_amdgcn_alignbit(z[g][0], z[g][1], 4);
      z[g][0] = z[g][0] >> 4;
      const uint4 m = M[nib];
      z[g][0] ^= m.x; z[g][1] ^= m.y; z[g][2] ^= m.z; z[g][3] ^= m.w;
    }
  }
  uint4 r[4];
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const uint32_t sp = z[g][4];
    r[g] = make_uint4(z[g][0] ^ sp ^ (sp >> 1) ^ (sp >> 2) ^ (sp >> 7),
                      z[g][1] ^ (sp << 31) ^ (sp << 30) ^ (sp << 25), z[g][2], z[g][3]);
  }
  uint4 acc = r[3];
#pragma unroll
  for (int g = 2; g >= 0; g--) acc = xor4(mulx32(acc), r[g]);
  return acc;
}

// Record lanes: lane q of the record in slot `slot` (ds_read_b128 lane groups).
// Lane within the 32-lane half of the record's q-th lane (set B = the
// {4-11,16-19,28-31} group).
__device__ __forceinline__ int group_lane(int setb, int q) {
  return setb ? (q < 8 ? q + 4 : q < 12 ? q + 8 : q + 16) : (q < 4 ? q : q < 8 ? q + 8 : q + 12);
}
struct RecLanes {
  int q, slot, setb, half;  // half = lane & 32
  __device__ int src(int i) const {  // wave lane of the record's lane i
    return half + group_lane(setb, i);
  }
};
__device__ __forceinline__ RecLanes rec_lanes() {
  RecLanes r;
  const int t = threadIdx.x;
  const int l = t & 31;
  r.setb = (l >= 4 && l < 12) || (l >= 16 && l < 20) || l >= 28;
  r.q = r.setb ? (l < 12 ? l - 4 : l < 20 ? l - 8 : l - 16)
               : (l < 4 ? l : l < 16 ? l - 8 : l - 12);
  r.slot = 2 * (t >> 5) + r.setb;
  r.half = t & 32;
  return r;
}
__device__ __forceinline__ uint32_t rshfl(uint32_t v, const RecLanes &R, int i) {
  return __shfl(v, R.src(i), 64);
}
__device__ __forceinline__ uint4 shfl_xor4(uint4 v, const RecLanes &R, int o) {
  const int s = R.src(R.q ^ o);
  return make_uint4(__shfl(v.x, s, 64), __shfl(v.y, s, 64), __shfl(v.z, s, 64),
                    __shfl(v.w, s, 64));
}

// ---- record buffers ----------------------------------------------------------

// Up to 16 bytes at p as little-endian words, zero-padded.
__device__ __forceinline__ uint4 load_block(const uint8_t *p, uint64_t avail) {
  if (avail >= 16 && (reinterpret_cast<uintptr_t>(p) & 15) == 0)
    return *reinterpret_cast<const uint4 *>(p);
  uint32_t w[4] = {0, 0, 0, 0};
  const uint32_t n = avail < 16 ? (uint32_t)avail : 16u;
  for (uint32_t i = 0; i < n; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_block(uint8_t *p, uint4 v, uint64_t avail) {
  if (avail >= 16 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    *reinterpret_cast<uint4 *>(p) = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uint32_t n = avail < 16 ? (uint32_t)avail : 16u;
  for (uint32_t i = 0; i < n; i++) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// Little-endian block words -> GCM-order big-endian words of the byte-reversed
// block (POLYVAL's ByteReverse, e_aesgcmsiv.cc:624-629).
__device__ __forceinline__ uint4 rev(uint4 x) { return make_uint4(x.w, x.z, x.y, x.x); }

#define SIV_OCC __attribute__((amdgpu_waves_per_eu(3)))
__device__ const uint64_t kSivMetaZero[2] = {0, 0};

template <typename T>
__device__ __forceinline__ T siv_meta(const T *arr, uint64_t i, bool active) {
  const T *p = arr && active ? arr + i : reinterpret_cast<const T *>(kSivMetaZero);
  return *p;
}

// One record (16 lanes, the record's slot `slot` of the workgroup's LDS):
// everything a record needs happens inside its wave, so the only
// synchronisation is wave-local (siv_wave_sync).
__device__ __forceinline__ void siv_wave_sync() {
  // LDS writes of some lanes read back by other lanes of the same wave: LDS
  // executes a wave's instructions in order; this keeps the compiler from
  // reordering across the hand-off.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// IOV: iovec records walked in place (BatchDesc::iovecs, iov_dev.h): both
// passes over the message follow the chunks with per-lane walks (stride
// 16 kL bytes).
template <int NR, bool OPEN, bool IOV>
__device__ __forceinline__ void siv_record(const GcmKeyDev *__restrict__ keys, const BatchDesc &b,
                                           Lds &L, const RecLanes &R, uint64_t rec) {
  const int q = R.q;
  const int slot = R.slot;
  const bool active = rec < b.num_records;
  uint64_t off = 0, len = 0, ad_off = 0, ad_len = 0;
  uint32_t kidx = 0;
  // Branch-free: a missing array is read at kSivMetaZero, so these loads and
  // the nonce's are in flight together (under the null-pointer branches hipcc
  // waited for each before issuing the next).
  uint8_t vld = 1;
  if (!(b.offsets || b.lengths || b.ad_offsets || b.ad_lengths || b.key_index || b.valid)) {
    if (active) {  // uniform layout, one key: no per-record loads
      off = rec * b.record_stride;
      len = b.record_len;
      ad_off = rec * b.ad_stride;
      ad_len = b.ad_len;
    }
  } else {
    const uint64_t o = siv_meta(b.offsets, rec, active), l = siv_meta(b.lengths, rec, active);
    const uint64_t ao = siv_meta(b.ad_offsets, rec, active);
    const uint64_t al = siv_meta(b.ad_lengths, rec, active);
    const uint32_t ki = siv_meta(b.key_index, rec, active);
    if (active) {
      off = b.offsets ? o : rec * b.record_stride;
      len = b.lengths ? l : b.record_len;
      ad_off = b.ad_offsets ? ao : rec * b.ad_stride;
      ad_len = b.ad_lengths ? al : b.ad_len;
      kidx = b.key_index ? ki : 0u;
    }
    vld = siv_meta(b.valid, rec, active);
  }
  // e_aesgcmsiv.cc:794-808, 830-846.
  const bool live = active && kidx < b.num_keys && b.nonce_len == 12 && b.tag_len == 16 &&
                    len <= (uint64_t(1) << 36) && ad_len < (uint64_t(1) << 61) &&
                    (!b.valid || vld);
  // (Addressed once the record index is known: any in-range record's nonce
  // is readable when nonce_len is 12.)
  const bool nok = active && b.nonce_len == 12;
  const uint8_t *np = b.nonces + (nok ? rec * 12 : 0);
  uint4 nw = nok ? load_block(np, 12) : make_uint4(0, 0, 0, 0);
  if (!live) nw = make_uint4(0, 0, 0, 0);

  // gcm_siv_keys (e_aesgcmsiv.cc:750-780): AES_K(le32(i) || nonce)[0:8].
  constexpr int kKeyBlocks = NR == 14 ? 6 : 4;
  uint4 km = make_uint4(0, 0, 0, 0);
  if (live && q < kKeyBlocks)
    km = aes_enc<NR>(make_uint4((uint32_t)q, nw.x, nw.y, nw.z),
                     reinterpret_cast<const uint4 *>(keys[kidx].rk_plain), L);
  uint32_t ek[8];
#pragma unroll
  for (int i = 0; i < kKeyBlocks - 2; i++) {
    ek[2 * i] = rshfl(km.x, R, i + 2);
    ek[2 * i + 1] = rshfl(km.y, R, i + 2);
  }
  const uint32_t a0 = rshfl(km.x, R, 0), a1 = rshfl(km.y, R, 0), a2 = rshfl(km.x, R, 1),
                 a3 = rshfl(km.y, R, 1);
  // FIPS-197 KeyExpansion of the record key, little-endian words, lane 0.
  if (q == 0) {
    constexpr int nk = NR - 6;
    uint32_t win[nk];
    uint32_t *out = reinterpret_cast<uint32_t *>(L.rk[slot]);
#pragma unroll
    for (int i = 0; i < nk; i++) {
      win[i] = ek[i];
      out[i] = ek[i];
    }
    uint32_t rcon = 1;
#pragma unroll
    for (int i = nk; i < 4 * (NR + 1); i++) {
      uint32_t t = win[(i - 1) % nk];
      if (i % nk == 0) {
        t = (t >> 8) | (t << 24);  // RotWord
        t = sbox(L, t & 0xff) | (sbox(L, (t >> 8) & 0xff) << 8) |
            (sbox(L, (t >> 16) & 0xff) << 16) | (sbox(L, t >> 24) << 24);
        t ^= rcon;
        rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11b : 0);
      } else if (nk == 8 && i % nk == 4) {
        t = sbox(L, t & 0xff) | (sbox(L, (t >> 8) & 0xff) << 8) |
            (sbox(L, (t >> 16) & 0xff) << 16) | (sbox(L, t >> 24) << 24);
      }
      win[i % nk] ^= t;
      out[i] = win[i % nk];
    }
  }
  // Shoup tables of H_g^(2^p), p = 0..4.  H_g = mulX_GHASH(ByteReverse(H))
  // (e_aesgcmsiv.cc:634-645): the little-endian integer of H shifted right
  // by one, 0xe1 into its top byte if bit 0 was set, read big-endian.
  uint4 hp = make_uint4(((a3 >> 1) ^ ((a0 & 1) ? 0xe1000000u : 0u)), (a2 >> 1) | (a3 << 31),
                        (a1 >> 1) | (a2 << 31), (a0 >> 1) | (a1 << 31));
#pragma unroll 1
  for (int p = 0; p < kPows; p++) {
    const uint4 b8 = hp, b4 = mulx(b8), b2 = mulx(b4), b1 = mulx(b2);
    uint4 e = make_uint4(0, 0, 0, 0);
    if (q & 8) e = xor4(e, b8);
    if (q & 4) e = xor4(e, b4);
    if (q & 2) e = xor4(e, b2);
    if (q & 1) e = xor4(e, b1);
    L.m[slot][p][q] = e;
    siv_wave_sync();
    if (p + 1 < kPows) hp = gmul(hp, L.m[slot][p]);
  }
  const uint4 *rk = L.rk[slot];

  // POLYVAL sequence [AD blocks, message blocks, length block]; lane q takes
  // elements j = q, q + 16, ...
  const uint64_t nA = live ? (ad_len + 15) / 16 : 0, nP = live ? (len + 15) / 16 : 0;
  const uint64_t n = live ? nA + nP + 1 : 0;
  const uint8_t *ad = b.ad + ad_off;
  const uint8_t *src = b.in + off;
  uint8_t *dst = b.out + off;
  uint4 ctr0 = make_uint4(0, 0, 0, 0);
  if (OPEN && live) {
    ctr0 = load_block(batch_tag(b, rec), 16);
    ctr0.w |= 0x80000000u;  // counter[15] |= 0x80 (e_aesgcmsiv.cc:577)
  }
  const uint64_t abits = ad_len * 8, mbits = len * 8;
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint64_t jlast = 0;
  bool any = false;
  IovWalk wl, ws;  // (IOV) loads and stores of the lane's message blocks
  if constexpr (IOV) {
    if (live) {
      iov_walk_init(wl, b, rec);
      iov_walk_init(ws, b, rec);
    }
  }
  for (uint64_t j = q; j < n; j += kL) {
    uint4 blk;
    if (j < nA) {
      if constexpr (IOV)
        blk = ivec_load16(b.aadvecs, b.aadvec_start[rec], b.aadvec_start[rec + 1], 16 * j,
                          (uint32_t)umin64(ad_len - 16 * j, 16));
      else
        blk = load_block(ad + 16 * j, ad_len - 16 * j);
    } else if (j < nA + nP) {
      const uint64_t p = j - nA;
      const uint32_t pn = (uint32_t)umin64(len - 16 * p, 16);
      uint4 x;
      if constexpr (IOV)
        x = iov_walk_load(wl, b, rec, 16 * p, pn, 16 * kL);
      else
        x = load_block(src + 16 * p, len - 16 * p);
      if (OPEN) {
        const uint4 ks = aes_enc<NR>(make_uint4(ctr0.x + (uint32_t)p, ctr0.y, ctr0.z, ctr0.w), rk, L);
        uint4 y = xor4(x, ks);
        if constexpr (IOV)
          iov_walk_store(ws, b, rec, 16 * p, y, pn, 16 * kL);
        else
          store_block(dst + 16 * p, y, len - 16 * p);
        const uint64_t rem = len - 16 * p;  // mask the padding of a partial block
        if (rem < 16) {
          uint32_t w[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint32_t lo = 4 * i;
            w[i] &= rem >= lo + 4 ? 0xffffffffu : rem <= lo ? 0u : ((1u << (8 * (rem - lo))) - 1u);
          }
          y = make_uint4(w[0], w[1], w[2], w[3]);
        }
        blk = y;
      } else {
        blk = x;
      }
    } else {
      blk = make_uint4((uint32_t)abits, (uint32_t)(abits >> 32), (uint32_t)mbits,
                       (uint32_t)(mbits >> 32));
    }
    acc = any ? xor4(gmul4d(acc, L.m[slot][kPows - 1]), rev(blk)) : rev(blk);
    any = true;
    jlast = j;
  }
  // acc * H^(n - jlast), then the sum over the record's lanes.
  if (any) {
    const uint32_t e = (uint32_t)(n - jlast);  // 1..16
    if (e == 16) {
      acc = gmul(acc, L.m[slot][4]);
    } else {
#pragma unroll 1
      for (int t = 0; t < 4; t++)
        if (e & (1u << t)) acc = gmul(acc, L.m[slot][t]);
    }
  }
#pragma unroll
  for (int o = kL / 2; o >= 1; o >>= 1) acc = xor4(acc, shfl_xor4(acc, R, o));
  // POLYVAL result (byte-reversed back), ^ nonce, bit 127 cleared, AES_K'.
  uint4 s = rev(acc);
  s.x ^= nw.x;
  s.y ^= nw.y;
  s.z ^= nw.z;
  s.w &= 0x7fffffffu;
  const uint4 tag = aes_enc<NR>(s, rk, L);

  int ok = live;
  if (OPEN && live) {
    const uint4 t = load_block(batch_tag(b, rec), 16);  // CRYPTO_memcmp, :861-864
    ok = ((t.x ^ tag.x) | (t.y ^ tag.y) | (t.z ^ tag.z) | (t.w ^ tag.w)) == 0;
  }
  if (!OPEN && live) {
    // gcm_siv_crypt from the tag (e_aesgcmsiv.cc:817).
    ctr0 = tag;
    ctr0.w |= 0x80000000u;
    if constexpr (IOV) {
      iov_walk_init(wl, b, rec);
      iov_walk_init(ws, b, rec);
    }
    for (uint64_t p = q; p < nP; p += kL) {
      const uint32_t pn = (uint32_t)umin64(len - 16 * p, 16);
      uint4 x;
      if constexpr (IOV)
        x = iov_walk_load(wl, b, rec, 16 * p, pn, 16 * kL);
      else
        x = load_block(src + 16 * p, len - 16 * p);
      const uint4 ks = aes_enc<NR>(make_uint4(ctr0.x + (uint32_t)p, ctr0.y, ctr0.z, ctr0.w), rk, L);
      if constexpr (IOV)
        iov_walk_store(ws, b, rec, 16 * p, mask_block(xor4(x, ks), pn), pn, 16 * kL);
      else
        store_block(dst + 16 * p, xor4(x, ks), len - 16 * p);
    }
  }
  if (active && q == 0) {
    if (!OPEN) store_block(batch_tag(b, rec), ok ? tag : make_uint4(0, 0, 0, 0), 16);
    if (b.status) b.status[rec] = ok ? 1 : 0;
  }
  // Zero the output of a failed record (aead.cc.inc:132-139, 539-547).
  if (active && !ok) {
    if constexpr (IOV)
      iov_clear(b, rec, q, kL);
    else
      for (uint64_t p = q; 16 * p < len; p += kL)
        store_block(dst + 16 * p, make_uint4(0, 0, 0, 0), len - 16 * p);
  }
  siv_wave_sync();  // the slot's round keys / tables are free for the next record
}

template <int NR, bool OPEN, bool IOV>
__global__ __launch_bounds__(kThreads) SIV_OCC void gcm_siv_kernel(const GcmKeyDev *__restrict__ keys,
                                                           BatchDesc b,
                                                           uint32_t *__restrict__ units) {
  __shared__ Lds L;
  for (int e = threadIdx.x; e < 256 * 64; e += kThreads) {
    const uint32_t v = kSivTables.te0[e >> 6];
    (&L.t[0][0][0])[e] = ((e >> 5) & 1) ? rotl(v, 8) : v;
  }
  __syncthreads();
  const RecLanes R = rec_lanes();
  const int lane = threadIdx.x & 63;
  const int local = R.slot & 3;  // the wave's record slots are 4w .. 4w + 3
  for (;;) {
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(units, 1u);
    u = __builtin_amdgcn_readfirstlane(__shfl(u, 0, 64));
    if ((uint64_t)u * 4 >= b.num_records) break;
    siv_record<NR, OPEN, IOV>(keys, b, L, R, (uint64_t)u * 4 + local);
  }
}

}  // namespace

int launch_gcm_siv(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr, void *stream,
                   const KernelEvents *ev) {
  if (b.num_records == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int num_cus = device_cu_count();
  if (!num_cus) return 1;
  uint32_t *units = nullptr;  // the grid-wide unit counter
  if (hipMallocAsync(reinterpret_cast<void **>(&units), 64, s) != hipSuccess) return 2;
  if (hipMemsetAsync(units, 0, 64, s) != hipSuccess) {
    hipFreeAsync(units, s);
    return 2;
  }
  const uint64_t wanted = (b.num_records + kRecs - 1) / kRecs;
  const unsigned grid = (unsigned)(wanted < (uint64_t)num_cus ? wanted : (uint64_t)num_cus);
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
  const bool iov = b.iovecs != nullptr;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, s, keys, b, units); };
  if (nr == 14) {
    if (open)
      iov ? go(gcm_siv_kernel<14, true, true>) : go(gcm_siv_kernel<14, true, false>);
    else
      iov ? go(gcm_siv_kernel<14, false, true>) : go(gcm_siv_kernel<14, false, false>);
  } else {
    if (open)
      iov ? go(gcm_siv_kernel<10, true, true>) : go(gcm_siv_kernel<10, true, false>);
    else
      iov ? go(gcm_siv_kernel<10, false, true>) : go(gcm_siv_kernel<10, false, false>);
  }
  const int rc = (int)hipGetLastError();
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
  hipFreeAsync(units, s);
  return rc;
}

}  // namespace bssl_amd
