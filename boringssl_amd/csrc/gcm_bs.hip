// gcm_bs.hip -- the table-free AES-GCM engine (gfx950): AES bitsliced on the
// VALU with no lookup table of any kind, GHASH by the conflict-free LDS byte
// table of H^L, the record start and end in the bulk kernel.  DESIGN.md §4.2b.
//
// Replaces, like gcm.hip, aead_aes_gcm_sealv_impl / _openv_detached_impl
// (crypto/fipsmodule/cipher/e_aes.cc.inc:779-867) ->
// CRYPTO_gcm128_{init_ctx,aad,encrypt,decrypt,tag} (crypto/fipsmodule/aes/
// gcm.cc.inc:298-604); its AES is the reference's own constant-time choice,
// a bitsliced cipher (aes_nohw_sub_bytes, crypto/fipsmodule/aes/
// aes_nohw.cc.inc:508; its batched CTR32, :1171-1214), here on 16 blocks per
// lane with two state columns per register (bs16_aes.h).
//
// * Work split.  L lanes per record (64 / L records per wave: one "unit"),
//   lane q encrypts the counter blocks j = 16*L*c + L*n + q of chunk c in its
//   16 bit-slots n, so a wave instruction moves 16*L-byte runs per record,
//   and folds its ciphertext blocks into a GHASH accumulator by Horner's rule
//   at stride L (multiplier H^L, the LDS byte table; gcm_common.h).  Units are
//   claimed from a grid-wide counter.
// * Chunk.  Round 0 of the 16 counter blocks (J0 words XOR the round key, the
//   counter word through one 32x32 bit transpose), rounds 1..NR with the
//   key's precomputed AddRoundKey masks (GcmKeyDev::bsmask, scalar loads), two
//   output transposes into 16 keystream blocks, then one pass over the slots
//   in which the plaintext loads run ahead of the XOR/store and each slot's
//   GHASH multiply (acc * H^L, whose input is known before the block arrives)
//   is issued before waiting for the block.
// * Record start.  J0 and the AD hash by the record's lanes (gcm_common.h).
//   E_K(J0) by a bitsliced batch per 1,024 records (64 lanes x 16 slots, one
//   "group"): the wave that claims the middle unit of group g computes the
//   E_K(J0) of group g + kBsAhead (the first kBsAhead groups by units
//   0..kBsAhead-1) and writes them as epoch-tagged granules to a per-launch
//   scratch (zeroed by the launcher); the record end polls its granules
//   (normally long ready) and, after kBsEk0Polls polls without them, computes
//   its own E_K(J0) (self_ek0), so no record end depends on another wave for
//   more than a bounded time.
// * Record end.  finish_record (gcm_common.h): the lanes' weights H^(L-p), the
//   L-lane XOR, length block, tag, check and zero-fill.
#include <hip/hip_runtime.h>

#include <atomic>
#ifdef BSSL_AMD_BS_PROF
#include <cstdio>
#endif

#include "bs16_aes.h"
#include "gcm_common.h"

namespace bssl_amd {
namespace {
#include "gcm_bs_io.inc"
}  // namespace
}  // namespace bssl_amd

namespace bssl_amd {
namespace {

constexpr int kBsThreads = 1024;          // 16 waves per CU at 128 VGPRs
constexpr uint32_t kBsGroupRecs = 1024;   // records per E_K(J0) batch
#ifndef BS_AHEAD
#define BS_AHEAD 4
#endif
#ifndef BS_EDGE_PRIO
#define BS_EDGE_PRIO 0  // (A/B builds: s_setprio of the record start and end)
#endif
constexpr uint32_t kBsAhead = BS_AHEAD;    // E_K(J0) groups produced ahead (bs_kernel)
constexpr uint32_t kBsLdsBasis = kG8Bytes;  // build_gpow scratch (2 KiB)
constexpr uint32_t kBsLdsState = kBsLdsBasis + 128 * 16;  // parked unit state (bs_unit)
// L2 prefetch of a chunk's record bytes at the start of round NR - BS_PF
// (0: none); the loads land in a scratch line of LDS.
#ifndef BS_PF
#define BS_PF 0
#endif
constexpr uint32_t kBsLdsSink = kBsLdsState + 16 * 4 * kBsThreads;  // 256 B
#define BS_PF_LD(n) "global_load_lds_dword %1, off offset:%" #n "\n\t"
#define BS_PF_ASM                                                                                  \
  "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t" BS_PF_LD(3) BS_PF_LD(4) BS_PF_LD(5)         \
      BS_PF_LD(6) BS_PF_LD(7) BS_PF_LD(8) BS_PF_LD(9) BS_PF_LD(10) BS_PF_LD(11) BS_PF_LD(12)       \
          BS_PF_LD(13) BS_PF_LD(14) BS_PF_LD(15) BS_PF_LD(16) BS_PF_LD(17) BS_PF_LD(18)            \
              "s_mov_b32 m0, %0"
#ifdef BSSL_AMD_BS_PROF
// Diagnostic builds: per-wave phase clocks (s_memtime cycles), summed per
// launch into g_bs_prof and printed by the launcher.
constexpr int kBsProfN = 16;
constexpr uint32_t kBsLdsProf = kBsLdsSink + 256;
constexpr uint32_t kBsLdsBytes = kBsLdsProf + 8 * kBsProfN * (kBsThreads / 64);
__device__ unsigned long long g_bs_prof[kBsProfN];
// Per group (first 4096 of a launch): realtime of production start / end, of
// the first consumer's arrival at its record end, and of the claim of the
// group's first unit.
__device__ unsigned long long g_bs_grp[4096][4];
struct BsClock {
  uint64_t t = __builtin_amdgcn_s_memtime();
  __device__ void lap(uint8_t *smem, int k) {
    const uint64_t n = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0)
      reinterpret_cast<uint64_t *>(smem + kBsLdsProf)[(threadIdx.x >> 6) * kBsProfN + k] += n - t;
    t = n;
  }
};
#define BS_LAP(k) clk.lap(smem, k)
#else
constexpr uint32_t kBsLdsBytes = kBsLdsSink + 256;
#define BS_LAP(k) ((void)0)
#endif
// Launch control words (zeroed by the launcher): the unit counter.
// E_K(J0) of processing position i: four data-tagged 8-byte granules {E word
// k, epoch} at ek0[2i] (words 0 and 2), ek0[2i + 1] (words 1 and 3), two per
// 16-byte write-through (sc1) store, read by sc1 loads until all four carry this launch's epoch (a
// per-launch number): no flag, no ordering, no reliance on a 16-byte store
// landing whole, and a line left in an XCD's L2 by an earlier launch cannot
// pass for this one's (MI355X_MICROARCH.md, inter-workgroup visibility:
// granule hand-off).  (A flag per group written after the values
// raced on the GPU: a tag mismatch in the ragged parity test.)

typedef uint32_t v32u __attribute__((ext_vector_type(32)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The lane's index in its wave from a volatile asm statement: an opaque value
// the compiler recomputes at each use instead of keeping it (and everything
// derived from it) live across the rounds.
__device__ __forceinline__ uint32_t bs_lane() {
  uint32_t v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return v;
}

// 0 or 0xffffffff: bit `k` of w.
__device__ __forceinline__ uint32_t bit_mask(uint32_t w, int k) {
  return (uint32_t)(((int32_t)(w << (31 - k))) >> 31);
}

// 32x32 bit transpose (bit n of m[k] <-> bit k of m[n]): the 16- and 8-bit
// stages are byte permutations (one v_perm_b32 per output word), the 4/2/1-bit
// stages one shift plus one bit-select per output word.
template <int S>
__device__ __forceinline__ void tr_stage(uint32_t m[32]) {
  constexpr uint32_t kLo = S == 4 ? 0x0f0f0f0fu : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    if (k & S) continue;
    const uint32_t a = m[k], b = m[k + S];
    if constexpr (S == 16) {
      m[k] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      m[k + S] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    } else if constexpr (S == 8) {
      m[k] = __builtin_amdgcn_perm(b, a, 0x06020400u);
      m[k + S] = __builtin_amdgcn_perm(b, a, 0x07030501u);
    } else {
      m[k] = (a & kLo) | ((b << S) & ~kLo);
      m[k + S] = (b & ~kLo) | ((a >> S) & kLo);
    }
  }
}

__device__ __forceinline__ void transpose32(uint32_t m[32]) {
  tr_stage<16>(m);
  tr_stage<8>(m);
  tr_stage<4>(m);
  tr_stage<2>(m);
  tr_stage<1>(m);
}

// Keystream words of register pair h: word n (< 16) = column h of slot n,
// word 16 + n = column h + 2 of slot n.
__device__ __forceinline__ v32u bs16_words(const uint32_t (&p)[4][2][8], int h) {
  uint32_t o[32];
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int b = 0; b < 8; b++) o[8 * r + b] = p[r][h][b];
  transpose32(o);
  v32u v;
#pragma unroll
  for (int n = 0; n < 32; n++) v[n] = o[n];
  return v;
}

// The 16 blocks w[n] ^ rk0 as bitsliced state (round 0 of 16 arbitrary
// blocks: the E_K(J0) batches).
__device__ __forceinline__ void bs16_load_blocks(uint32_t (&p)[4][2][8], const uint4 (&w)[16],
                                                 const uint32_t rk0[4]) {
  uint32_t t0[32], t1[32];
#pragma unroll
  for (int n = 0; n < 16; n++) {
    t0[n] = w[n].x ^ rk0[0];
    t0[16 + n] = w[n].z ^ rk0[2];
    t1[n] = w[n].y ^ rk0[1];
    t1[16 + n] = w[n].w ^ rk0[3];
  }
  transpose32(t0);
  transpose32(t1);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    p[k / 8][0][k % 8] = t0[k];
    p[k / 8][1][k % 8] = t1[k];
  }
}

// acc * H^L with the lane-rotated byte table: 16 lookups in four groups of
// four (sched barriers keep at most four lookups' 16 registers in flight
// beside the 64 keystream words of the slot loop).
__device__ __forceinline__ uint4 g8_mul(uint4 x, bool rs1, bool rs2, uint32_t rbs,
                                        const uint32_t (&P)[4], const uint8_t *smem) {
  Gh8 h;
  g8_rotate(h, x, rs1, rs2, rbs);
  uint4 a = xor4(xor4_3(g8_load<0>(h, P, smem), g8_load<1>(h, P, smem), g8_load<2>(h, P, smem)),
                 g8_load<3>(h, P, smem));
  __builtin_amdgcn_sched_barrier(0);
  a = xor4(xor4_3(a, g8_load<4>(h, P, smem), g8_load<5>(h, P, smem)),
           xor4_3(g8_load<6>(h, P, smem), g8_load<7>(h, P, smem), make_uint4(0, 0, 0, 0)));
  __builtin_amdgcn_sched_barrier(0);
  a = xor4(xor4_3(a, g8_load<8>(h, P, smem), g8_load<9>(h, P, smem)),
           xor4(g8_load<10>(h, P, smem), g8_load<11>(h, P, smem)));
  __builtin_amdgcn_sched_barrier(0);
  a = xor4(xor4_3(a, g8_load<12>(h, P, smem), g8_load<13>(h, P, smem)),
           xor4(g8_load<14>(h, P, smem), g8_load<15>(h, P, smem)));
  return a;
}

// ---------------------------------------------------------------------------
// E_K(J0) of records [i0, i0 + 1024) in processing order (one group): lane l
// takes positions i0 + 16 l + s in its slots s.  KS: records carry their own
// keys (keysets) -- one cipher per distinct key among a lane's slots, with
// that key's masks per lane; one-key batches take one cipher with the key's
// wave-uniform masks.  Results to the granules of ek0 (above).
template <int NR, bool KS>
__device__ __forceinline__ void produce_ek0_ks(const GcmKeyDev *__restrict__ keys, const BatchDesc &b,
                                         uint64_t i0, uint64_t end, uint4 *__restrict__ ek0,
                                         uint32_t epoch) {
  const int lane = threadIdx.x & 63;
  const uint64_t base = i0 + 16u * (uint64_t)lane;
  // Top priority while producing: a group's consumers wait for it, and at
  // the kernel's start ~20 productions run beside every wave's first record
  // start (at priority 0 they took 300-470 us there and the first consumers
  // arrived at ~230 us: ~7 % of the groups late by 160 us on average).
  __builtin_amdgcn_s_setprio(3);
  uint4 j0[16];
  uint32_t kidx[16];
  uint32_t todo = 0;
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const uint64_t i = base + s;
    j0[s] = make_uint4(0, 0, 0, 0);
    kidx[s] = 0;
    if (i < end) {
      const uint64_t rec = rec_at(b, i);
      const RecordMeta m = record_meta(b, rec);
      if (record_live(b, rec, m)) {
        kidx[s] = KS ? b.key_index[rec] : 0u;
        if (b.nonce_len == 12) {
          const uint4 nn = load_partial(b.nonces + rec * 12, 12);
          j0[s] = make_uint4(nn.x, nn.y, nn.z, 0x01000000u);
        } else {
          j0[s] = record_j0(b, rec, keys[kidx[s]].hpow_ct);
        }
        todo |= 1u << s;
      }
    }
  }
  while (__ballot(todo != 0)) {
    uint32_t mine = todo;
    uint32_t p[4][2][8];
    if constexpr (KS) {
      const uint32_t k = todo ? kidx[__builtin_ctz(todo)] : 0u;
      mine = 0;
#pragma unroll
      for (int s = 0; s < 16; s++) mine |= (uint32_t)(((todo >> s) & 1u) && kidx[s] == k) << s;
      const uint32_t *rkp = &keys[k].rk_plain[0][0];
      bs16_load_blocks(p, j0, rkp);
      bs16_cipher<NR, false>(p, rkp);
    } else {
      uint32_t rk0[4];
#pragma unroll
      for (int c = 0; c < 4; c++) rk0[c] = keys[0].rk_plain[0][c];
      bs16_load_blocks(p, j0, rk0);
      bs16_cipher_tab<NR>(p, &keys[0].bsmask[0][0]);
    }
    const v32u KA = bs16_words(p, 0), KB = bs16_words(p, 1);
#pragma unroll
    for (int s = 0; s < 16; s++)
      if ((mine >> s) & 1u) {
        const u32x4 g0 = {KA[s], epoch, KA[16 + s], epoch}, g1 = {KB[s], epoch, KB[16 + s], epoch};
        // (s_nop 1: a store of more than 8 bytes reads its data registers a
        // cycle late, and the compiler's hazard check does not see inside
        // inline asm -- without it the next VALU write of those registers
        // went into the granule.)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\tglobal_store_dwordx4 %0, %2, off offset:16 sc1\n\t"
                     "s_nop 1"
                     ::"v"(ek0 + 2 * (base + s)), "v"(g0), "v"(g1)
                     : "memory");
      }
    todo &= ~mine;
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int NR, bool KS>
__device__ __forceinline__ void produce_ek0(const GcmKeyDev *__restrict__ keys, const BatchDesc &b,
                                         uint64_t i0, uint64_t end, uint4 *__restrict__ ek0,
                                         uint32_t epoch) {
  if constexpr (KS) {
    produce_ek0_ks<NR, true>(keys, b, i0, end, ek0, epoch);
    return;
  }
  const int lane = (int)bs_lane();  // (opaque: not hoisted into the kernel prologue)
  const uint64_t base = i0 + 16u * (uint64_t)lane;
  // Top priority while producing (as produce_ek0_ks).
  __builtin_amdgcn_s_setprio(3);
  // The live slots (and, for keysets, their keys).  No J0 array is kept: each
  // cipher pass re-reads its slots' nonces straight into the round-0
  // transpose inputs, so the 64 words of 16 J0 blocks are never live beside
  // the cipher state (kept, they spilled: 162 of the kernel's 178 VGPR
  // spills were here).
  uint32_t todo = 0;
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const uint64_t i = base + s;
    if (i < end) {
      const uint64_t rec = rec_at(b, i);
      if (record_live(b, rec, record_meta(b, rec))) todo |= 1u << s;
    }
  }
  auto key_of = [&](int s) -> uint32_t {  // (KS: a live slot's key)
    return KS ? b.key_index[rec_at(b, base + s)] : 0u;
  };
  do {
    uint32_t mine = todo, k = 0;
    if constexpr (KS) {
      k = todo ? key_of(__builtin_ctz(todo)) : 0u;
      mine = 0;
#pragma unroll
      for (int s = 0; s < 16; s++)
        if ((todo >> s) & 1u) mine |= (uint32_t)(key_of(s) == k) << s;
    }
    const GcmKeyDev *key = keys + k;
    // Round 0, one state pair at a time (pair h: columns h and h + 2 of
    // J0 ^ rk0 through one 32x32 transpose; the nonces are read once per pair).
    uint32_t p[4][2][8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t ra = key->rk_plain[0][h], rb = key->rk_plain[0][h + 2];
      uint32_t t[32];
#pragma unroll
      for (int s = 0; s < 16; s++) {
        uint4 j0 = make_uint4(0, 0, 0, 0);
        if ((mine >> s) & 1u) {
          const uint64_t rec = rec_at(b, base + s);
          if (b.nonce_len == 12) {
            const uint4 nn = load_partial(b.nonces + rec * 12, 12);
            j0 = make_uint4(nn.x, nn.y, nn.z, 0x01000000u);
          } else {
            j0 = record_j0(b, rec, key->hpow_ct);
          }
        }
        t[s] = (h ? j0.y : j0.x) ^ ra;
        t[16 + s] = (h ? j0.w : j0.z) ^ rb;
      }
      transpose32(t);
#pragma unroll
      for (int q = 0; q < 32; q++) p[q / 8][h][q % 8] = t[q];
    }
    if constexpr (KS)
      bs16_cipher<NR, false>(p, &key->rk_plain[0][0]);
    else
      bs16_cipher_tab<NR>(p, &key->bsmask[0][0]);
    // Granule quad 0 = {E word 0, epoch, E word 2, epoch} comes from pair 0
    // of the state alone and quad 1 = {E word 1, epoch, word 3, epoch} from
    // pair 1, so each half is stored as soon as its transpose is done and the
    // two never hold 64 registers together.
    auto store_half = [&](const v32u &K, int half) {
#pragma unroll
      for (int s = 0; s < 16; s++)
        if ((mine >> s) & 1u) {
          const u32x4 g = {K[s], epoch, K[16 + s], epoch};
          // (s_nop 1: a store of more than 8 bytes reads its data registers a
          // cycle late, and the compiler's hazard check does not see inside
          // inline asm -- without it the next VALU write of those registers
          // went into the granule.)
          asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1\n\ts_nop 1"
                       ::"v"(ek0 + 2 * (base + s)), "v"(g), "i"(16 * half)
                       : "memory");
        }
    };
    store_half(bs16_words(p, 0), 0);
    store_half(bs16_words(p, 1), 1);
    todo &= ~mine;
  } while (KS && __ballot(todo != 0));
  __builtin_amdgcn_s_setprio(0);
}

// E_K(J0) of processing position i (active lanes): sc1 loads of its two
// granules until both carry `epoch` (the wave loops until every active lane
// has its value) or `max_polls` retries have passed.  Returns whether every
// active lane got its value (wave-uniform); `polls`: the retries.
__device__ __forceinline__ uint4 load_ek0(const uint4 *ek0, uint64_t i, bool active, uint32_t epoch,
                                          uint32_t max_polls, uint32_t &polls, bool &got) {
  u32x4 g0 = {0, 0, 0, 0}, g1 = {0, 0, 0, 0};
  polls = 0;
  for (;;) {
    bool ok = true;
    if (active) {
      asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %2, off offset:16 sc1\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(g0), "=&v"(g1)
                   : "v"(ek0 + 2 * i)
                   : "memory");
      ok = g0.y == epoch && g0.w == epoch && g1.y == epoch && g1.w == epoch;
    }
    got = __ballot(!ok) == 0;
    if (got || polls >= max_polls) break;
    __builtin_amdgcn_s_sleep(4);
    polls++;
  }
  return make_uint4(g0.x, g1.x, g0.z, g1.z);  // (quad 0: words 0, 2; quad 1: words 1, 3)
}

// Polls of a record end before it computes its own E_K(J0): each is an L2
// round trip plus a short sleep, so the bound is ~1 ms -- far above the
// producer's lead in a normal launch (the values are ready ~200 us before the
// record ends that read them), far below any watchdog.
#ifndef BS_SELF_EK0
#define BS_SELF_EK0 1  // (A/B builds: 0 = round 5's unbounded wait, no fallback)
#endif
constexpr uint32_t kBsEk0Polls = BS_SELF_EK0 ? 1024u : 0xffffffffu;

// The wave's own E_K(J0) of the lane's record (live lanes; the others get
// E_K(0^128), unused): one bitsliced batch with the record's J0 in slot 0 of
// every lane.  The fallback of a record end whose granules did not arrive
// (load_ek0 returned false), and with production switched off
// (BSSL_AMD_test_set_bs_ek0_producers) the path of every record end.
template <int NR>
__device__ __forceinline__ uint4 self_ek0(const GcmKeyDev *__restrict__ key, const BatchDesc &b,
                                       uint64_t rec, bool live) {
  uint4 w[16];
#pragma unroll
  for (int s = 0; s < 16; s++) w[s] = make_uint4(0, 0, 0, 0);
  if (live) {
    if (b.nonce_len == 12) {
      const uint4 nn = load_partial(b.nonces + rec * 12, 12);
      w[0] = make_uint4(nn.x, nn.y, nn.z, 0x01000000u);
    } else {
      w[0] = record_j0(b, rec, key->hpow_ct);
    }
  }
  uint32_t rk0[4];
#pragma unroll
  for (int c = 0; c < 4; c++) rk0[c] = key->rk_plain[0][c];
  uint32_t p[4][2][8];
  bs16_load_blocks(p, w, rk0);
  bs16_cipher_tab<NR>(p, &key->bsmask[0][0]);
  const v32u KA = bs16_words(p, 0), KB = bs16_words(p, 1);
  return make_uint4(KA[0], KB[0], KA[16], KB[16]);
}

// iovec records: the chunk cursors of a lane (gcm.hip process_records' form:
// chunk index + stream start, and running pointers / bytes left in the chunk
// between chunk boundaries).  Input and output chunks have the same lengths,
// so both runs advance together.
struct BsIovCur {
  uint64_t ld_c, ld_cs, st_c, st_cs;
  const uint8_t *ld_ptr;
  uint8_t *st_ptr;
  int32_t left;  // bytes left in the current chunk run (-1: none yet)
};

// One block of an iovec record that is not a whole block inside the current
// chunk run (a chunk boundary, a straddle, the record's last block, the first
// block): walk the chunk table for the load and the store, re-anchor the runs.
// Out of line: inlined into each of the 16 slots of the unrolled pass it held
// the 64 keystream registers through 16 copies of the walk and spilled
// 8 KiB per lane; as a call the walks' registers are its own.  Returns the
// hashed block (OPEN: the input, else the output).
// (The batch's fields by value: a reference to the kernel's by-value
// descriptor would make the compiler copy it to the stack.)
template <int L, bool OPEN>
__device__ __noinline__ uint4 bs_iov_slow(const IovecDev *iovecs, const uint64_t *iovec_start,
                                          uint64_t rlen, BsIovCur &cur, uint64_t rec, uint32_t j,
                                          uint4 ks) {
  BatchDesc b;  // (the iovec helpers read only b.iovecs)
  b.iovecs = iovecs;
  const uint64_t pb = (uint64_t)j * 16;
  const uint64_t c_end = iovec_start[rec + 1];
  const uint32_t nbytes = (uint32_t)umin64(rlen - pb, 16);
  uint4 x;
  {
    IovCur k;
    iov_at(k, b, cur.ld_c, cur.ld_cs);
    iov_seek(k, b, pb, c_end);
    if (nbytes == 16 && pb + 16 <= k.ce)
      x = load16_any(k.in + (pb - k.cs));
    else if (!iov_load2(b, k, pb, nbytes, c_end, x))
      x = iov_gather(b, k, pb, nbytes, c_end);
    cur.ld_c = k.c;
    cur.ld_cs = k.cs;
    cur.ld_ptr = k.in + (pb - k.cs) + 16 * L;
    cur.left = (int32_t)umin64(k.ce - pb, 1u << 30) - 16 * L;
  }
  const uint4 y = mask_block(xor4(x, ks), nbytes);
  {
    IovCur k;
    iov_at(k, b, cur.st_c, cur.st_cs);
    iov_seek(k, b, pb, c_end);
    if (nbytes == 16 && pb + 16 <= k.ce)
      store16_any(k.out + (pb - k.cs), y);
    else if (!iov_store2(b, k, pb, y, nbytes, c_end))
      iov_scatter(b, k, pb, y, nbytes, c_end);
    cur.st_c = k.c;
    cur.st_cs = k.cs;
    cur.st_ptr = k.out + (pb - k.cs) + 16 * L;
  }
  return OPEN ? x : y;
}

// Where a record end gets its E_K(J0): the epoch-tagged granules of the
// batched production (polled, with the bounded-wait fallback).  The mixed
// engine (gcm_mix.hip) passes its own source.
struct BsEk0Granules {
  const uint4 *ek0;
  uint32_t epoch, max_polls;
  template <int NR>
  __device__ __forceinline__ uint4 get(uint64_t pos, bool act_live, const GcmKeyDev *key,
                                       const BatchDesc &b, uint64_t rec, uint32_t &polls) const {
    bool got;
    uint4 e0 = load_ek0(ek0, pos, act_live, epoch, max_polls, polls, got);
#if BS_SELF_EK0
    if (!got) e0 = self_ek0<NR>(key, b, rec, act_live);  // (wave-uniform)
#endif
    return e0;
  }
};

// ---------------------------------------------------------------------------
// Per-lane unit state parked in LDS while the rounds hold the registers
// (word k of thread t at kBsLdsState + (k * kBsThreads + t) * 4: consecutive
// lanes on consecutive banks).  The rounds need ~105 VGPRs of the 128; these
// values would otherwise stay live across them and spill.
enum : int {
  kSc0, kSw1, kSc1,  // round-1 S-box outputs of the pair-0 groups (packed, bs_unit) and
                     // J0 word 1 XOR round key 0
  kScb,              // counter word of the lane's slot 0 of chunk 0: bswap(J0.w) + 1 + q
  kSnb, kSnfull,     // the record's blocks and full blocks (this lane's record)
  kSoff, kSoffHi,    // the record's offset in in / out
  kSacc0, kSacc1, kSacc2, kSacc3,
  kSflags,           // bit 0 active, bit 1 live
  kSrec, kSrecHi,
  kSwords
};

// The 64 / L records of one unit, L lanes each: the lane's record is at
// processing position first + r for r = lane / L (wave-uniform `first`; bit r
// of the wave-uniform `amask`: the unit has a record there).  The lane's own
// position and flag are recomputed from the lane index where needed.
// PARK / PTHREADS: LDS offset of the parked unit state and the threads it is
// laid out for (the bitsliced kernels: kBsLdsState for all 1,024 threads; the
// mixed engine: its bitsliced waves only); `slot`: the wave's parking slot
// (wave-uniform, its index in the workgroup, taken once at the kernel start
// so that no thread index stays live across the units).  EK0: the record ends' E_K(J0)
// source (BsEk0Granules).
template <int NR, bool OPEN, bool XT, bool IOV, int L, uint32_t PARK = kBsLdsState,
          int PTHREADS = kBsThreads, class EK0 = BsEk0Granules>
__device__ __forceinline__ void bs_unit(const GcmKeyDev *__restrict__ key, const BatchDesc &b,
                                        uint64_t first, uint64_t amask, uint8_t *smem,
                                        const EK0 &ek0src, uint32_t slot) {
  static_assert(L == 16 || L == 8 || L == 4 || L == 2, "lanes per record");
  static_assert(!(IOV && XT), "iovec records carry no extra bytes");
#ifdef BSSL_AMD_BS_PROF
  BsClock clk;
#endif
  // Lane-derived values are recomputed where they are used from an opaque
  // lane index (v_mbcnt in a volatile asm statement): kept live across the
  // rounds they spilled to scratch, and every chunk paid the scratch round
  // trips.  The unit state goes through inline-asm LDS accesses (the compiler
  // must neither forward the stored values in registers across the rounds nor
  // turn them into flat accesses).  Word k of thread t is at kBsLdsState +
  // (k / 4) * 16 * kBsThreads + 16 * t + 4 * (k % 4): quads of consecutive
  // words per lane, read by one ds_read_b128 (16-byte lane stride: no bank
  // conflicts).
#if BS_PF > 0
  const uint32_t lsink =
      (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t *)smem) +
      kBsLdsSink;
#endif
  const uint32_t lbase =
      (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t *)smem) +
      PARK + 16u * 64u * slot;
  auto addr = [&]() -> uint32_t {
    uint32_t a;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\t"
                 "v_lshl_add_u32 %0, %0, 4, %1"
                 : "=&v"(a)
                 : "s"(lbase));
    return a;
  };
  auto get = [&](int k) -> uint32_t {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v)
                 : "v"(addr()), "i"((k >> 2) * 16 * PTHREADS + 4 * (k & 3)));
    return v;
  };
  auto put4 = [&](int k, uint4 v) {  // words k..k+3 (k % 4 == 0)
    const u32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1 offset:%2\n\ts_nop 1" ::"v"(addr()), "v"(w),
                 "i"((k >> 2) * 16 * PTHREADS));
  };
  auto get4 = [&](int k) -> uint4 {  // words k..k+3 (k % 4 == 0)
    u32x4 w;
    asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(w)
                 : "v"(addr()), "i"((k >> 2) * 16 * PTHREADS));
    return make_uint4(w.x, w.y, w.z, w.w);
  };
  const int q = (int)(bs_lane() & (L - 1));
  int nchunks;
  // IOV: chunk cursors (as gcm.hip process_records: chunk index + stream
  // start; between chunk boundaries only the running pointers move).
  BsIovCur iov = {0, 0, 0, 0, nullptr, nullptr, -1};
#if BS_EDGE_PRIO
  __builtin_amdgcn_s_setprio(BS_EDGE_PRIO);  // (A/B: the record start's loads and products)
#endif
  {
    const uint32_t r = bs_lane() / L;
    const uint64_t i = first + r;
    const bool active = (amask >> r) & 1u;
    const uint64_t rec = active ? rec_at(b, i) : 0;
    RecordMeta m = {0, 0, 0, 0, 0};
    if (active) m = record_meta(b, rec);
    if constexpr (!XT) m.xlen = 0;
    const bool live = active && record_live(b, rec, m);
    // J0 (gcm.cc.inc:316-338) and the AD hash (:347-398), in the record's lanes.
    uint4 j0 = make_uint4(0, 0, 0, 0);
    if (live) {
      if (b.nonce_len == 12) {
        const uint4 nn = load_partial(b.nonces + rec * 12, 12);
        j0 = make_uint4(nn.x, nn.y, nn.z, 0x01000000u);
      } else {
        j0 = record_j0(b, rec, key->hpow_ct);
      }
    }
    const bool many_ad = __ballot(live && m.ad_len > 16) != 0;
    uint4 acc = record_ad_hash<L>(b, rec, m, live, many_ad, key->hpow_ct);
    if (q != L - 1 || !live) acc = make_uint4(0, 0, 0, 0);
    // (< 2^32: the GCM length limit holds for a live record)
    const uint32_t nb = live ? (uint32_t)((m.len + m.xlen + 15) / 16) : 0u;
    const uint32_t nfull = live && !IOV ? (uint32_t)(m.len / 16) : 0u;
    nchunks = __builtin_amdgcn_readfirstlane(wave_max((int)((nb + 16 * L - 1) / (16 * L))));
    // Counter-mode caching: the pair-0 groups (columns 0 and 2 of J0 ^ rk0)
    // are the same in every slot of every chunk, so their round-1 SubBytes
    // is done once here.  Each of the 32 output planes is 0 / 0xffff per
    // half: packed as bits k (low half) and 16 + k (high half) of two words.
    {
      const uint32_t w0 = j0.x ^ key->rk_plain[0][0], w2 = j0.z ^ key->rk_plain[0][2];
      uint32_t pk[2] = {0, 0};
#pragma unroll
      for (int r = 0; r < 4; r++) {
        uint32_t g[8], o[8];
#pragma unroll
        for (int bb = 0; bb < 8; bb++)
          g[bb] = (bit_mask(w0, 8 * r + bb) & 0xffffu) | (bit_mask(w2, 8 * r + bb) & 0xffff0000u);
        sbox_planes(g, o);
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
          const int k = 8 * (r & 1) + bb;
          pk[r >> 1] |= ((o[bb] & 1u) << k) | (((o[bb] >> 16) & 1u) << (16 + k));
        }
      }
      put4(kSc0, make_uint4(pk[0], j0.y ^ key->rk_plain[0][1], pk[1],
                            bswap32(j0.w) + 1u + (uint32_t)q));
    }
    put4(kSnb, make_uint4(nb, nfull, (uint32_t)m.off, (uint32_t)(m.off >> 32)));
    put4(kSacc0, acc);
    put4(kSflags, make_uint4((active ? 1u : 0u) | (live ? 2u : 0u), (uint32_t)rec,
                             (uint32_t)(rec >> 32), 0u));
    if constexpr (IOV) {
      if (live) iov.ld_c = iov.st_c = b.iovec_start[rec];
    }
  }
  const uint32_t *__restrict__ mk = &key->bsmask[0][0];
#if BS_EDGE_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  BS_LAP(0);
#pragma unroll 1
  for (int c = 0; c < nchunks; c++) {
    uint32_t p[4][2][8];
    const uint4 st = get4(kSc0);  // round-1 cache words, w1, counter base
    {
      // Round 0.  Pair 0 = columns 0 and 2 of J0 ^ rk0 (the same in every
      // slot: 0 / 0xffff per half); pair 1 = column 1 (low half, constant)
      // and the counter words of column 3 (high half), out of one transpose:
      // t[n] = column 1, t[16 + n] = word 3 of slot n.
      const uint32_t w1 = st.y;
      const uint32_t rk3 = key->rk_plain[0][3];
      const uint32_t cb = st.w + (uint32_t)(16 * L) * (uint32_t)c;  // inc32: mod 2^32
      uint32_t t[32];
#pragma unroll
      for (int n = 0; n < 16; n++) {
        t[n] = w1;
        t[16 + n] = bswap32(cb + (uint32_t)L * (uint32_t)n) ^ rk3;
      }
      transpose32(t);
#pragma unroll
      for (int k = 0; k < 32; k++) p[k / 8][1][k % 8] = t[k];
    }
    {
      // Round 1 of the pair-0 groups from the per-record cache: plane k of
      // packed word W is W << (15 - k) with each 16-bit half shifted right
      // arithmetically by 15 (v_pk_ashrrev_i16).
      typedef short s16x2 __attribute__((ext_vector_type(2)));
      const uint32_t pk[2] = {st.x, st.z};
      uint32_t c1[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
          const int k = 8 * (r & 1) + bb;
          s16x2 v = __builtin_bit_cast(s16x2, pk[r >> 1] << (15 - k));
          v = v >> (short)15;
          c1[r][bb] = __builtin_bit_cast(uint32_t, v);
        }
#if BS_PF > 0
      // Prefetch of the chunk's record bytes into L2 a few rounds before the
      // output pass reads them (LDS-DMA dword loads into a shared scratch line
      // of LDS: no VGPR destination, nothing waits for them; the output pass's
      // counted waits only get stricter): full chunks only, so every address is
      // inside the lane's record.
      auto pf = [&](int rd) {
        if (rd != NR - BS_PF) return;
        const uint4 rs = get4(kSnb);
        const uint32_t jc = (uint32_t)(16 * L) * (uint32_t)c + (bs_lane() & (L - 1));
        if (jc + (uint32_t)(16 * L) * 15u < rs.y) {
          const uint8_t *s0 = b.in + ((uint64_t)rs.z | ((uint64_t)rs.w << 32)) + (uint64_t)jc * 16;
          uint32_t keep;
          asm volatile(BS_PF_ASM
                       : "=&s"(keep)
                       : "v"(s0), "s"(lsink), "i"(0), "i"(16 * L), "i"(32 * L), "i"(48 * L),
                         "i"(64 * L), "i"(80 * L), "i"(96 * L), "i"(112 * L), "i"(128 * L),
                         "i"(144 * L), "i"(160 * L), "i"(176 * L), "i"(192 * L), "i"(208 * L),
                         "i"(224 * L), "i"(240 * L)
                       : "memory");
        }
      };
      bs16_cipher_ctr<NR>(p, c1, mk, pf);
#else
      bs16_cipher_ctr<NR>(p, c1, mk);
#endif
    }
    BS_LAP(1);
    // Pass 1 (memory): out = in ^ keystream for the lane's full blocks, the
    // plaintext loads running kAhead slots ahead (slot n of the lane is 16*L*n
    // bytes past slot 0: immediate offsets); the hashed block (the ciphertext:
    // the output when sealing, the input when opening) replaces the keystream
    // in KA/KB.  Pass 2 (LDS): acc = acc * H^L ^ C over the lane's blocks.
    // Both passes are unrolled, so every index is static and each slot's
    // registers die with it.  A lane's other block (the record's partial last
    // block and extra bytes, j in [nfull, nb): its last element, at most one
    // per lane) parks its keystream in kt and is sealed and hashed last.
    // (Scheduling barriers: the scheduler would otherwise interleave the two
    // transposes and hoist the plaintext loads above them, which needs more
    // than the 128 registers.)
    uint32_t KA[32], KB[32];
    __builtin_amdgcn_sched_barrier(0);
    {
      const v32u ka = bs16_words(p, 0);
#pragma unroll
      for (int k = 0; k < 32; k++) {
        KA[k] = ka[k];
        asm volatile("" : "+v"(KA[k]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const v32u kb = bs16_words(p, 1);
#pragma unroll
      for (int k = 0; k < 32; k++) {
        KB[k] = kb[k];
        asm volatile("" : "+v"(KB[k]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    BS_LAP(2);
    const uint32_t jc = (uint32_t)(16 * L) * (uint32_t)c + (bs_lane() & (L - 1));
    const uint4 rs = get4(kSnb);
    const uint32_t nb = rs.x, nfull = rs.y;
    const uint64_t off = (uint64_t)rs.z | ((uint64_t)rs.w << 32);
    const uint8_t *src = b.in + off;
    uint8_t *dst = b.out + off;
    const uint8_t *s0 = src + (uint64_t)jc * 16;
    uint8_t *d0 = dst + (uint64_t)jc * 16;
    // The output pass (not iovec records): one inline-asm statement
    // (gcm_bs_io.inc) -- plaintext loads D slots ahead, each slot's GHASH
    // multiply issued while its block is in flight, stores and the hash fold
    // predicated on the lane's full blocks (a prefix of its slots: nv), fixed
    // scratch registers.  (The compiler's schedule of the same work hoisted
    // every load and spilled.)  A lane's other block in this chunk (the
    // record's partial last block or extra bytes: slot tl) gets its keystream
    // kept in kt and is sealed after the pass.
    if constexpr (!IOV) {
      const int gq = (int)(bs_lane() & 15);
      uint32_t P[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) v |= (((4u * k + e + gq) & 15u) << 4) << (8 * e);
        P[k] = v;
      }
      const int nv = jc < nfull ? (int)min((nfull - jc + L - 1) / L, 16u) : 0;
      const int tl = (nv < 16 && jc + (uint32_t)L * (uint32_t)nv < nb) ? nv : -1;
      const uint4 av = get4(kSacc0);
      uint32_t accv[4] = {av.x, av.y, av.z, av.w};
      uint32_t kt[4] = {0, 0, 0, 0};
      // (rs1 / rs2 of g8_rotate as lane masks: bits 2 and 3 of the lane's
      // index in its 16-lane row)
      constexpr uint64_t kM1 = 0xf0f0f0f0f0f0f0f0ull, kM2 = 0xff00ff00ff00ff00ull;
      const uint64_t a0 = reinterpret_cast<uint64_t>(s0), a1 = reinterpret_cast<uint64_t>(d0);
      const uint32_t rb = (uint32_t)gq & 3u;
      const bool any_tail = __ballot(tl >= 0) != 0;
      const bool full = !any_tail && __ballot(nv < 16) == 0;
#define BS_IO(SUFFIX) bs_chunk_io_##SUFFIX(KA, KB, accv, kt, a0, a1, kM1, kM2, rb, nv, tl, P)
#if defined(BSSL_AMD_BS_ABLATE)  // diagnostic builds (wrong output): 1 no GHASH, 2 no I/O, 3 neither
      if constexpr (BSSL_AMD_BS_ABLATE == 1) BS_IO(seal_L16_noghash);
      else if constexpr (BSSL_AMD_BS_ABLATE == 2) BS_IO(seal_L16_nomem);
      else if constexpr (BSSL_AMD_BS_ABLATE == 3) BS_IO(seal_L16_none);
      else if constexpr (BSSL_AMD_BS_ABLATE == 4) {
#pragma unroll
        for (int k = 0; k < 32; k++) accv[k & 3] ^= KA[k] ^ KB[k];
      }
      if constexpr (false)
#endif
      if constexpr (L == 16) {
        if (full) { if constexpr (OPEN) BS_IO(open_full_L16); else BS_IO(seal_full_L16); }
        else if (any_tail) { if constexpr (OPEN) BS_IO(open_tail_L16); else BS_IO(seal_tail_L16); }
        else { if constexpr (OPEN) BS_IO(open_L16); else BS_IO(seal_L16); }
      } else if constexpr (L == 8) {
        if (full) { if constexpr (OPEN) BS_IO(open_full_L8); else BS_IO(seal_full_L8); }
        else if (any_tail) { if constexpr (OPEN) BS_IO(open_tail_L8); else BS_IO(seal_tail_L8); }
        else { if constexpr (OPEN) BS_IO(open_L8); else BS_IO(seal_L8); }
      } else if constexpr (L == 4) {
        if (full) { if constexpr (OPEN) BS_IO(open_full_L4); else BS_IO(seal_full_L4); }
        else if (any_tail) { if constexpr (OPEN) BS_IO(open_tail_L4); else BS_IO(seal_tail_L4); }
        else { if constexpr (OPEN) BS_IO(open_L4); else BS_IO(seal_L4); }
      } else {
        if (full) { if constexpr (OPEN) BS_IO(open_full_L2); else BS_IO(seal_full_L2); }
        else if (any_tail) { if constexpr (OPEN) BS_IO(open_tail_L2); else BS_IO(seal_tail_L2); }
        else { if constexpr (OPEN) BS_IO(open_L2); else BS_IO(seal_L2); }
      }
#undef BS_IO
      BS_LAP(3);
      if (tl >= 0) {
        // (The record's buffers re-derived from the parked offset: kept live
        // across the pass, the two pointers spilled once per chunk.)
        const uint32_t jt = (uint32_t)(16 * L) * (uint32_t)c + (bs_lane() & (L - 1)) +
                            (uint32_t)L * (uint32_t)tl;
        const uint4 rt = get4(kSnb);
        const uint64_t offt = (uint64_t)rt.z | ((uint64_t)rt.w << 32);
        const uint8_t *src = b.in + offt;
        uint8_t *dst = b.out + offt;
        const uint64_t rec = (uint64_t)get(kSrec) | ((uint64_t)get(kSrecHi) << 32);
        const RecordMeta m = record_meta(b, rec);
        const uint32_t xlen = XT ? m.xlen : 0u;
        const uint4 hm = g8_mul(make_uint4(accv[0], accv[1], accv[2], accv[3]), (gq >> 2) & 1,
                                (gq >> 3) & 1, rb, P, smem);
        const uint32_t nbytes = (uint32_t)umin64(m.len + xlen - (uint64_t)jt * 16, 16);
        const uint4 ktv = make_uint4(kt[0], kt[1], kt[2], kt[3]);
        uint4 x, y;
        if constexpr (XT) {
          y = crypt_partial_x(src, dst, m.len, batch_extra_in(b, rec), batch_extra_out(b, rec),
                              (uint64_t)jt * 16, ktv, nbytes, x);
        } else {
          x = load_partial(src + (uint64_t)jt * 16, nbytes);
          y = mask_block(xor4(x, ktv), nbytes);
          store_partial(dst + (uint64_t)jt * 16, y, nbytes);
        }
        const uint4 c = OPEN ? x : y;
        accv[0] = hm.x ^ c.x;
        accv[1] = hm.y ^ c.y;
        accv[2] = hm.z ^ c.z;
        accv[3] = hm.w ^ c.w;
      }
      put4(kSacc0, make_uint4(accv[0], accv[1], accv[2], accv[3]));
      BS_LAP(4);
      continue;
    }
    // iovec records (the contiguous path continued above): pass 1 walks the
    // chunks with the load / store cursors, pass 2 hashes.  A record's
    // partial last block is handled inside pass 1 (iov_load2 / iov_gather).
    if constexpr (IOV) {
      int nv = 0;  // the lane's blocks of this chunk (hashed in pass 2)
      // (the record's bytes: its total, parked as its block count and full
      // blocks would not tell a partial last block; re-read per chunk)
      uint64_t nbytes_total = 0;
      {
        const uint64_t rec = (uint64_t)get(kSrec) | ((uint64_t)get(kSrecHi) << 32);
        if (nb) nbytes_total = b.lengths ? b.lengths[rec] : b.record_len;
      }
#pragma unroll
      for (int n = 0; n < 16; n++) {
        const uint32_t j = jc + (uint32_t)L * (uint32_t)n;
        const uint4 ks = make_uint4(KA[n], KB[n], KA[16 + n], KB[16 + n]);
        uint4 cv = make_uint4(0, 0, 0, 0);
        if (j < nb) {
          // A whole block inside the current chunk run: one load and one
          // store at the running pointers; anything else out of line.
          // (Temporal accesses, as the T-table engine's iovec walk.)
          if (iov.left >= 16 && (j + 1) * 16 <= nbytes_total) {
            const uint4 x = load16_any(iov.ld_ptr);
            const uint4 y = xor4(x, ks);
            store16_any(iov.st_ptr, y);
            iov.ld_ptr += 16 * L;
            iov.st_ptr += 16 * L;
            iov.left -= 16 * L;
            cv = OPEN ? x : y;
          } else {
            const uint64_t rec = (uint64_t)get(kSrec) | ((uint64_t)get(kSrecHi) << 32);
            cv = bs_iov_slow<L, OPEN>(b.iovecs, b.iovec_start, nbytes_total, iov, rec, j, ks);
          }
          nv = n + 1;
        }
        KA[n] = cv.x;
        KB[n] = cv.y;
        KA[16 + n] = cv.z;
        KB[16 + n] = cv.w;
      }
      // (Pass 2 starts here: the pins keep the compiler from hoisting its
      // lookups into pass 1, whose registers they would need.)
#pragma unroll
      for (int k = 0; k < 32; k++) asm volatile("" : "+v"(KA[k]), "+v"(KB[k]));
      const int gq = (int)(bs_lane() & 15);  // (GHASH lane constants, gcm_common.h Gh8)
      const bool rs1 = (gq >> 2) & 1, rs2 = (gq >> 3) & 1;
      const uint32_t rbs = (uint32_t)gq & 3u;
      uint32_t P[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) v |= (((4u * k + e + gq) & 15u) << 4) << (8 * e);
        P[k] = v;
      }
      uint4 acc = get4(kSacc0);
#pragma unroll
      for (int n = 0; n < 16; n++) {
        const uint4 hm = g8_mul(acc, rs1, rs2, rbs, P, smem);
        if (n < nv) acc = xor4(hm, make_uint4(KA[n], KB[n], KA[16 + n], KB[16 + n]));
      }
      put4(kSacc0, acc);
    }
  }
  // Record end.
#if BS_EDGE_PRIO
  __builtin_amdgcn_s_setprio(BS_EDGE_PRIO);
#endif
  const uint4 rq = get4(kSflags);
  const uint32_t fl = rq.x;
  const bool act = fl & 1u, live = (fl >> 1) & 1u;
  const uint64_t rec = (uint64_t)rq.y | ((uint64_t)rq.z << 32);
  RecordMeta m = {0, 0, 0, 0, 0};
  if (act) m = record_meta(b, rec);
  if constexpr (!XT) m.xlen = 0;
  const uint32_t nb = get(kSnb);
  const uint4 acc = get4(kSacc0);
  BS_LAP(5);
#ifdef BSSL_AMD_BS_PROF
  if ((threadIdx.x & 63) == 0 && first / kBsGroupRecs < 4096)
    atomicMin(&g_bs_grp[first / kBsGroupRecs][2], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
  uint32_t polls = 0;
  // (Live records only: the producer skips the others, whose output
  // finish_record zero-fills.)
  const uint4 e0 = ek0src.template get<NR>(first + bs_lane() / L, act && live, key, b, rec, polls);
  BS_LAP(8);
#ifdef BSSL_AMD_BS_PROF
  if ((threadIdx.x & 63) == 0) {
    uint64_t *w = reinterpret_cast<uint64_t *>(smem + kBsLdsProf) + (threadIdx.x >> 6) * kBsProfN;
    w[10] += polls;
    w[11] += 1;
    if (polls) {
      w[15] += 1;
      // where the waiting units are: position in the batch (first 16 groups,
      // last 16 groups, the rest) -- diagnostic buckets in slots 12..14
      const uint64_t gi = first / kBsGroupRecs, ng = (b.num_records + kBsGroupRecs - 1) / kBsGroupRecs;
      w[gi < 16 ? 12 : gi + 16 >= ng ? 13 : 14] += 1;
    }
  }
#else
  (void)polls;
#endif
  BS_LAP(9);
  finish_record<OPEN, L>(acc, nb, m, e0, b, rec, act, live, b.out + m.off, key->hpow_ct);
  BS_LAP(6);
#if BS_EDGE_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}

// One-key bulk kernel: one workgroup of 16 waves per CU; each wave takes the
// next unit of 64 / L records from the grid-wide counter (ctl[0]).  Before
// its unit, the claimant of a group's producer unit computes that group's
// E_K(J0) (produce_ek0).
template <int NR, bool OPEN, bool XT, bool IOV, int L>
__global__ __launch_bounds__(kBsThreads) void gcm_bs_kernel(const GcmKeyDev *__restrict__ keys,
                                                             BatchDesc b, uint32_t *__restrict__ ctl,
                                                             uint4 *__restrict__ ek0,
                                                             uint32_t epoch, uint32_t produce) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBsLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);  // (an SGPR)
#ifdef BSSL_AMD_BS_PROF
  if (lane < kBsProfN) reinterpret_cast<uint64_t *>(smem + kBsLdsProf)[(tid >> 6) * kBsProfN + lane] = 0;
  uint64_t t_prod = 0;
#endif
  if constexpr (L == 16)
    build_g8<kBsThreads>(smem, reinterpret_cast<const uint4 *>(keys[0].htab16), tid);
  else
    build_gpow<kBsThreads, kBsLdsBasis>(smem, keys[0].hpow_ct[L], tid);
  __syncthreads();
  constexpr uint32_t kRec = 64 / L;
  constexpr uint32_t kGroupUnits = kBsGroupRecs / kRec;
  // Processing positions of this launch (BatchDesc::split_lo/_hi: a length
  // class of a ragged batch); E_K(J0) groups count from lo.
  uint64_t lo = 0, n = b.num_records;
  if (b.split_lo) lo = *b.split_lo;
  if (b.split_hi) n = *b.split_hi;
  for (;;) {
    uint32_t u = 0;
    if (bs_lane() == 0) u = atomicAdd(ctl, 1u);
    u = __builtin_amdgcn_readfirstlane(u);
    const uint64_t first = lo + (uint64_t)u * kRec;
    if (first >= n) break;
    // Producer units: unit u < kBsAhead for group u (in parallel at the
    // start), the middle unit of group g for g + kBsAhead (with the producer
    // half a group ahead, a tenth of the units waited ~90 us for their
    // group's values at the record end).
    const uint32_t g = u / kGroupUnits;
    uint32_t pg = 0xffffffffu;
    if (u < kBsAhead && u < kGroupUnits / 2) pg = u;
    if (u % kGroupUnits == kGroupUnits / 2) pg = g + kBsAhead;
    if (produce && pg != 0xffffffffu && lo + (uint64_t)pg * kBsGroupRecs < n) {
#ifdef BSSL_AMD_BS_PROF
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#endif
      produce_ek0<NR, false>(keys, b, lo + (uint64_t)pg * kBsGroupRecs, n, ek0, epoch);
#ifdef BSSL_AMD_BS_PROF
      t_prod += __builtin_amdgcn_s_memtime() - t0;
      if (lane == 0 && pg < 4096) {
        g_bs_grp[pg][0] = r0;
        g_bs_grp[pg][1] = __builtin_amdgcn_s_memrealtime();
      }
#endif
    }
    const uint64_t amask = n - first >= kRec ? (kRec == 64 ? ~0ull : (1ull << kRec) - 1)
                                             : (1ull << (n - first)) - 1;
#ifdef BSSL_AMD_BS_PROF
    if (lane == 0 && u % kGroupUnits == 0 && g < 4096) g_bs_grp[g][3] = __builtin_amdgcn_s_memrealtime();
#endif
    bs_unit<NR, OPEN, XT, IOV, L>(keys, b, first, amask, smem,
                                  BsEk0Granules{ek0, epoch, kBsEk0Polls}, wave);
  }
#ifdef BSSL_AMD_BS_PROF
  if (lane == 0) {
    uint64_t *w = reinterpret_cast<uint64_t *>(smem + kBsLdsProf) + (tid >> 6) * kBsProfN;
    w[7] = t_prod;
    for (int k = 0; k < kBsProfN; k++) atomicAdd(&g_bs_prof[k], (unsigned long long)w[k]);
  }
#endif
}

// Keyset batches (key_index per record): records in tiles of 16 units; a
// tile whose records use several keys runs one pass per distinct key (the
// LDS byte table is per key).  E_K(J0) groups as in the one-key kernel, per
// record key (produce_ek0<KS = true>), claimed by the tile that holds the
// group's producer position.
template <int NR, bool OPEN, bool XT>
__global__ __launch_bounds__(kBsThreads) void gcm_bs_keyset_kernel(
    const GcmKeyDev *__restrict__ keys, BatchDesc b, uint32_t *__restrict__ ctl,
    uint4 *__restrict__ ek0, uint32_t epoch, uint32_t produce) {
  constexpr int kRecPerTile = 16 * 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBsLdsBytes + 64 * 16 + 16];
  uint32_t *s_pass_key = reinterpret_cast<uint32_t *>(smem + kBsLdsBytes);
  uint64_t *s_pass_mask = reinterpret_cast<uint64_t *>(smem + kBsLdsBytes + 64 * 4);
  int *s_npass = reinterpret_cast<int *>(smem + kBsLdsBytes + 64 * 12);
  uint64_t *s_base = reinterpret_cast<uint64_t *>(smem + kBsLdsBytes + 64 * 12 + 8);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t loaded = 0xffffffffu;
  const uint64_t n = b.num_records;
  for (;;) {
    // Tiles from the grid-wide counter (ctl[0]); wave 0 plans the tile.
    __syncthreads();
    if (wave == 0) {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(ctl, 1u);
      t = __builtin_amdgcn_readfirstlane(t);
      const uint64_t base = (uint64_t)t * kRecPerTile;
      const uint64_t i = base + lane;
      uint32_t k = (base < n && i < n) ? b.key_index[rec_at(b, i)] : 0xffffffffu;
      if (k != 0xffffffffu && k >= b.num_keys) k = 0;  // (not live: zeroed output)
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
      if (lane == 0) {
        *s_npass = base < n ? np : -1;
        *s_base = base;
      }
      // Group producers: tile t < kBsAhead for group t, the middle tile of
      // group g for g + kBsAhead (as the one-key kernel).
      if (base < n) {
        constexpr uint32_t kGroupTiles = kBsGroupRecs / kRecPerTile;
        const uint32_t g = t / kGroupTiles;
        uint32_t pg = 0xffffffffu;
        if (t < kBsAhead && t < kGroupTiles / 2) pg = t;
        if (t % kGroupTiles == kGroupTiles / 2) pg = g + kBsAhead;
        if (produce && pg != 0xffffffffu && (uint64_t)pg * kBsGroupRecs < n)
          produce_ek0<NR, true>(keys, b, (uint64_t)pg * kBsGroupRecs, n, ek0, epoch);
      }
    }
    __syncthreads();
    const int npass = *s_npass;
    if (npass < 0) break;
    const uint64_t base = *s_base;
    for (int pi = 0; pi < npass; pi++) {
      const uint32_t k = __builtin_amdgcn_readfirstlane(s_pass_key[pi]);
      const uint64_t mask = s_pass_mask[pi];
      if (k != loaded) {
        __syncthreads();
        build_g8<kBsThreads>(smem, reinterpret_cast<const uint4 *>(keys[k].htab16), tid);
        __syncthreads();
        loaded = k;
      }
      bs_unit<NR, OPEN, XT, false, 16>(keys + k, b, base + 4 * wave, (mask >> (4 * wave)) & 15u,
                                       smem, BsEk0Granules{ek0, epoch, kBsEk0Polls},
                                       (uint32_t)wave);
    }
  }
}

}  // namespace

// Table-free launcher (launch_gcm with the bitsliced engine selected).
// Lanes per record: 16 for records of 4 KiB or more (8 in a ragged batch), 2 for shorter ones
// (a chunk covers 16 * L blocks of a record: a 1350-byte record of 85
// blocks fills 3 chunks of 32 slots at L = 2, against one of 256 at L = 16;
// the per-record start and end are spread over the record's L lanes, and at
// L = 2 each lane has eight times the blocks).  A ragged batch in length
// order is two launches, the records of 4 KiB or more at 16 lanes and the
// shorter ones at 2 (the class cursor of the length sort, as gcm.hip).
#ifndef BS_LONG_L
#define BS_LONG_L 16
#endif
#ifndef BS_SHORT_L
#define BS_SHORT_L 2
#endif
// Lanes per record: 16 for uniform batches of records of 4 KiB or more, 8 for
// the long class of a ragged batch (4 KiB to 16 KiB and beyond: fewer empty
// slots in a record's last chunk; config 4 644 -> 677 GiB/s, while config 2
// lost 3 % at 8, same box, gpurun_out r5s21), 2 below 4 KiB (config G at 4:
// 544 against 676).
constexpr int kBsLongL = BS_LONG_L, kBsShortL = BS_SHORT_L;  // (A/B builds: -DBS_LONG_L=8 ...)
constexpr int kBsRaggedL = 8;

#ifndef BSSL_AMD_MIX_TU  // (gcm_mix.hip includes this file for bs_unit)
namespace {
std::atomic<bool> g_bs_producers{true};
}  // namespace

bool set_bs_ek0_producers(bool on) { return g_bs_producers.exchange(on); }

int launch_gcm_bs(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr, hipStream_t s,
                  const KernelEvents *ev) {
  const int num_cus = device_cu_count();
  if (!num_cus) return 1;
  const uint64_t n = b.num_records;
  // Two control blocks (one per launch of a split batch): the unit counters;
  // then the E_K(J0) granules of every processing position.  All of it is
  // zeroed: a granule's tag is the launch's epoch (never 0), and a pool
  // allocation recycled from any earlier use (this library's counters,
  // flags, histograms) cannot hold a value the poll would take for this
  // launch's.  n * 32 bytes: ~0.25 % of a 16 KiB-record batch.
  static std::atomic<uint32_t> s_epoch{0};
  uint32_t epoch = s_epoch.fetch_add(1, std::memory_order_relaxed) + 1;
  if (!epoch) epoch = s_epoch.fetch_add(1, std::memory_order_relaxed) + 1;
  const uint32_t produce = g_bs_producers.load(std::memory_order_relaxed) ? 1u : 0u;
  const size_t ctl_bytes = 256;
  const size_t scratch_bytes = 2 * ctl_bytes + n * 32;
  uint8_t *scratch = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&scratch), scratch_bytes, s) != hipSuccess)
    return 2;
  uint32_t *ctl = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *ctl2 = reinterpret_cast<uint32_t *>(scratch + ctl_bytes);
  uint4 *ek0 = reinterpret_cast<uint4 *>(scratch + 2 * ctl_bytes);
  if (hipMemsetAsync(scratch, 0, scratch_bytes, s) != hipSuccess) {
    hipFreeAsync(scratch, s);
    return 2;
  }
  BatchDesc bo = b;  // with the processing order of a ragged batch
  uint32_t *order = nullptr;
  if (wants_length_order(b)) {
    if (hipMallocAsync(reinterpret_cast<void **>(&order), (n + 128) * sizeof(uint32_t), s) !=
        hipSuccess) {
      hipFreeAsync(scratch, s);
      return 2;
    }
    const int orc = build_length_order(b.lengths, n, order, order + n, s);
    if (orc) {
      hipFreeAsync(order, s);
      hipFreeAsync(scratch, s);
      return orc;
    }
    bo.order = order;
  }
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
  const unsigned grid = (unsigned)((n + 3) / 4 < (uint64_t)num_cus ? (n + 3) / 4 : (uint64_t)num_cus);
  auto go = [&](auto kern, const BatchDesc &d, uint32_t *c) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBsThreads), 0, s, keys, d, c, ek0, epoch, produce);
  };
  // Length classes (one-key, not iovec): short uniform records take L = 2;
  // a ragged batch in length order splits at 4 KiB.
  const bool split = !b.key_index && !b.iovecs && order;
  const bool short_uniform = !b.key_index && !b.iovecs && !b.lengths && b.record_len < 4096;
  BatchDesc bl = bo, bs = bo;
  if (split) bl.split_hi = bs.split_lo = order + n + kSplitWord;
#define BSSL_BS_ONEKEY(NR_, OPEN_, XT_)                                              \
  do {                                                                               \
    if (split) {                                                                     \
      go(gcm_bs_kernel<NR_, OPEN_, XT_, false, kBsRaggedL>, bl, ctl);                \
      go(gcm_bs_kernel<NR_, OPEN_, XT_, false, kBsShortL>, bs, ctl2);                \
    } else if (short_uniform) {                                                      \
      go(gcm_bs_kernel<NR_, OPEN_, XT_, false, kBsShortL>, bo, ctl);                 \
    } else {                                                                         \
      go(gcm_bs_kernel<NR_, OPEN_, XT_, false, kBsLongL>, bo, ctl);                  \
    }                                                                                \
  } while (0)
#define BSSL_BS_LAUNCH(NR_, OPEN_)                                                   \
  do {                                                                               \
    if (b.key_index) {                                                               \
      if (b.extra_len) go(gcm_bs_keyset_kernel<NR_, OPEN_, true>, bo, ctl);          \
      else go(gcm_bs_keyset_kernel<NR_, OPEN_, false>, bo, ctl);                     \
    } else if (b.iovecs) {                                                           \
      go(gcm_bs_kernel<NR_, OPEN_, false, true, 16>, bo, ctl);                       \
    } else if (b.extra_len) {                                                        \
      BSSL_BS_ONEKEY(NR_, OPEN_, true);                                              \
    } else {                                                                         \
      BSSL_BS_ONEKEY(NR_, OPEN_, false);                                             \
    }                                                                                \
  } while (0)
  switch (nr * 2 + (open ? 1 : 0)) {
#ifdef BSSL_BS_QUICK  // (development builds: AES-128 seal only)
    case 20: go(gcm_bs_kernel<10, false, false, false, 16>, bo, ctl); break;
#else
    case 20: BSSL_BS_LAUNCH(10, false); break;
    case 21: BSSL_BS_LAUNCH(10, true); break;
    case 24: BSSL_BS_LAUNCH(12, false); break;
    case 25: BSSL_BS_LAUNCH(12, true); break;
    case 28: BSSL_BS_LAUNCH(14, false); break;
    case 29: BSSL_BS_LAUNCH(14, true); break;
#endif
    default: break;
  }
#undef BSSL_BS_LAUNCH
#undef BSSL_BS_ONEKEY
  const int rc = (int)hipGetLastError();
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
#ifdef BSSL_AMD_BS_PROF
  {
    unsigned long long h[kBsProfN];
    hipStreamSynchronize(s);
    hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bs_prof), sizeof(h));
    const unsigned long long z[kBsProfN] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_bs_prof), z, sizeof(z));
    static unsigned long long gr[4096][4];
    hipMemcpyFromSymbol(gr, HIP_SYMBOL(g_bs_grp), sizeof(gr));
    const uint64_t ng = (n + kBsGroupRecs - 1) / kBsGroupRecs < 4096 ? (n + kBsGroupRecs - 1) / kBsGroupRecs : 4096;
    uint64_t late = 0, late_sum = 0, prod_sum = 0, lead_sum = 0, maxlate = 0, nprod = 0;
    for (uint64_t g = 0; g < ng; g++) {
      if (!gr[g][1] || gr[g][2] == ~0ull) continue;
      nprod++;
      prod_sum += gr[g][1] - gr[g][0];
      lead_sum += gr[g][3] > gr[g][0] ? gr[g][3] - gr[g][0] : 0;
      if (gr[g][2] < gr[g][1]) {
        late++;
        late_sum += gr[g][1] - gr[g][2];
        if (gr[g][1] - gr[g][2] > maxlate) maxlate = gr[g][1] - gr[g][2];
      }
    }
    fprintf(stderr, "bs_grp groups %llu late %llu late_avg_us %.1f late_max_us %.1f prod_avg_us %.1f "
            "claim_after_prod_start_avg_us %.1f\n", (unsigned long long)nprod, (unsigned long long)late,
            late ? late_sum / 100.0 / late : 0.0, maxlate / 100.0, nprod ? prod_sum / 100.0 / nprod : 0.0,
            nprod ? lead_sum / 100.0 / nprod : 0.0);
    for (uint64_t g = 0; g < ng && g < 48; g++)
      if (gr[g][1] && gr[g][2] != ~0ull && gr[g][2] < gr[g][1])
        fprintf(stderr, "bs_grp late g=%llu prod %.1f..%.1f us, first arrival %.1f, first claim %.1f\n",
                (unsigned long long)g, (gr[g][0] - gr[0][3]) / 100.0, (gr[g][1] - gr[0][3]) / 100.0,
                (gr[g][2] - gr[0][3]) / 100.0, (gr[g][3] - gr[0][3]) / 100.0);
    static unsigned long long init[4096][4];
    for (auto &row : init) row[0] = row[1] = row[3] = 0, row[2] = ~0ull;
    hipMemcpyToSymbol(HIP_SYMBOL(g_bs_grp), init, sizeof(init));
    fprintf(stderr,
            "bs_prof n=%llu start %llu rounds %llu transp %llu out %llu tail %llu endmeta %llu "
            "finish %llu produce %llu flagwait %llu ek0load %llu polls %llu units %llu "
            "polled_first16 %llu polled_last16 %llu polled_mid %llu polled_units %llu\n",
            (unsigned long long)n, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9],
            h[10], h[11], h[12], h[13], h[14], h[15]);
  }
#endif
  if (order) hipFreeAsync(order, s);
  hipFreeAsync(scratch, s);
  return rc;
}
#endif  // BSSL_AMD_MIX_TU

}  // namespace bssl_amd
