// gcm_mix.hip -- the mixed-role AES-GCM kernel (round 6):
// NB bitsliced waves (gcm_bs.hip bs_unit: AES on the VALU, no table) and
// 16 - NB T-table waves (gcm.hip process_records: AES by LDS lookups) in one
// workgroup per CU, taking 4-record units (16 lanes per record) from one
// grid-wide counter.  The T-table engine is LDS-bound (82 % LDS, 45 % VALU
// busy on config 2) and the bitsliced one VALU-bound (63 % VALU, little LDS),
// so waves of both kinds on one CU could fill both units -- the reference's
// stitched kernels interleave AES and GHASH for the same reason
// (aes-gcm-avx512-x86_64.pl:845).  Opt-in and experimental: selected by
// BSSL_AMD_GCM_MODE=mix2|mix4|mix6 for one-key uniform batches of records of
// 4 KiB or more (AES-128; other batches take the T-table engine).  Both roles
// share the LDS GHASH byte table of H^16 at address 0; the T-tables follow at
// 64 KiB; the bitsliced waves park their unit state after them and compute
// each record's E_K(J0) at its end with the T-tables' quad form (ek0_quad),
// so no batched E_K(J0) production is needed.  DESIGN.md §9.1.
#define BSSL_AMD_MIX_TU 1
#include "gcm.hip"
#include "gcm_bs.hip"

namespace bssl_amd {
namespace {

// E_K(J0) at a bitsliced record end from the T-tables in LDS: lane c of each
// quad computes column c of the record's block (ek0_quad), quad_gather joins
// them (all 16 lanes of a record hold the same J0).
template <int NR>
struct MixEk0 {
  const uint8_t *smem;
  const RoundKeys *rk;
  uint32_t lc0, lc1;
  template <int NR2>
  __device__ __forceinline__ uint4 get(uint64_t, bool act_live, const GcmKeyDev *key,
                                       const BatchDesc &b, uint64_t rec, uint32_t &polls) const {
    static_assert(NR2 == NR, "rounds");
    polls = 0;
    uint4 j0 = make_uint4(0, 0, 0, 0);
    if (act_live) {
      if (b.nonce_len == 12) {
        const uint4 nn = load_partial(b.nonces + rec * 12, 12);
        j0 = make_uint4(nn.x, nn.y, nn.z, 0x01000000u);
      } else {
        j0 = record_j0(b, rec, key->hpow_ct);
      }
    }
    const RoundKeys &k = *rk;
    return quad_gather(ek0_quad<NR, 0>(j0.x ^ k.w[0][0], j0.y ^ k.w[0][1], j0.z ^ k.w[0][2],
                                       j0.w ^ k.w[0][3], k, smem, lc0, lc1));
  }
};

constexpr uint32_t kMixPark = (kLdsBytes + 15u) & ~15u;  // after gcm.hip's tables

template <int NR, bool OPEN, int NB>
__global__ __launch_bounds__(1024) void gcm_mix_kernel(const GcmKeyDev *__restrict__ keys,
                                                        BatchDesc b, uint32_t *__restrict__ ctl) {
  static_assert(NB > 0 && NB < 16, "bitsliced waves");
  __shared__ __attribute__((aligned(16))) uint8_t smem[kMixPark + 16 * 4 * 64 * NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  fill_aes_tables<1024>(smem, tid);
  build_g8<1024>(smem, reinterpret_cast<const uint4 *>(keys[0].htab16), tid);
  __syncthreads();
  const uint32_t lc0 = kLdsAes + (uint32_t)(lane & 31) * 4u;
  const uint32_t lc1 = lc0 + 128u;
  RoundKeys rk;
#pragma unroll
  for (int r = 0; r <= NR; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) rk.w[r][c] = keys[0].rk[r][c];
  const uint64_t n = b.num_records;
#ifndef MIX_TT_PRIO
#define MIX_TT_PRIO 3
#endif
  // The T-table waves issue at priority 3, above the bitsliced waves (whose
  // output pass runs at 2): at equal priority the older bitsliced waves took
  // the VALU slots the T-table waves' LDS stream waits on (mix4 874 -> 1,036
  // GiB/s, LDS busy 0.24 -> 0.52; profiles/r06/s6).
  if (MIX_TT_PRIO && wave >= NB) __builtin_amdgcn_s_setprio(MIX_TT_PRIO);
  for (;;) {
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(ctl, 1u);
    u = __builtin_amdgcn_readfirstlane(u);
    const uint64_t first = (uint64_t)u * 4;
    if (first >= n) break;
    if (wave < NB) {
      const uint64_t amask = n - first >= 4 ? 15ull : (1ull << (n - first)) - 1;
      bs_unit<NR, OPEN, false, false, 16, kMixPark, NB * 64>(
          keys, b, first, amask, smem, MixEk0<NR>{smem, &rk, lc0, lc1},
          __builtin_amdgcn_readfirstlane((uint32_t)wave));
    } else {
      UnitIn in;
      unit_load<false, false>(in, b, first + lane / 16, lane & 15, n);
      process_records<NR, OPEN, false, 16, false, false>(rk, b, in, smem, keys, lc0, lc1);
    }
  }
}

}  // namespace

bool gcm_mix_eligible(const BatchDesc &b, int nr) {
  return nr == 10 && !b.key_index && !b.iovecs && !b.extra_len && !b.lengths && !b.offsets &&
         !b.ad_lengths && !b.ad_offsets && b.record_len >= 4096 && b.num_records > 1;
}

int launch_gcm_mix(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nb, hipStream_t s,
                   const KernelEvents *ev) {
  const int num_cus = device_cu_count();
  if (!num_cus) return 1;
  uint32_t *ctl = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&ctl), 64, s) != hipSuccess) return 2;
  if (hipMemsetAsync(ctl, 0, 64, s) != hipSuccess) {
    hipFreeAsync(ctl, s);
    return 2;
  }
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->start), s);
  const uint64_t units = (b.num_records + 3) / 4;
  const unsigned grid = (unsigned)(units < (uint64_t)num_cus ? units : (uint64_t)num_cus);
#define BSSL_MIX(NB_)                                                                     \
  do {                                                                                    \
    if (open)                                                                             \
      hipLaunchKernelGGL((gcm_mix_kernel<10, true, NB_>), dim3(grid), dim3(1024), 0, s,   \
                         keys, b, ctl);                                                   \
    else                                                                                  \
      hipLaunchKernelGGL((gcm_mix_kernel<10, false, NB_>), dim3(grid), dim3(1024), 0, s,  \
                         keys, b, ctl);                                                   \
  } while (0)
  switch (nb) {
    case 2: BSSL_MIX(2); break;
    case 6: BSSL_MIX(6); break;
    default: BSSL_MIX(4); break;
  }
#undef BSSL_MIX
  const int rc = (int)hipGetLastError();
  if (ev) hipEventRecord(reinterpret_cast<hipEvent_t>(ev->stop), s);
  hipFreeAsync(ctl, s);
  return rc;
}

}  // namespace bssl_amd
