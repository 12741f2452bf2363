/* synth.h -- the synthetic record-batch workload (host side).
 *
 * TEST/BENCH INFRASTRUCTURE.  Defines the deterministic inputs shared by the
 * oracle, the reference harness (oracle/ref/ref_tool.cc) and the device-side
 * generator in boringssl_amd/csrc/synth.hip (a separate implementation of the
 * same definitions).  SURVEY.md section 8(d) fixes the shape of each config;
 * the generator below is counter-based (splitmix64 of a record/word index) so
 * that any record can be produced independently on the GPU.
 *
 *   key k     : byte b = byte (b%8) of SPLITMIX(SYNTH_KEY_SEED + 16*k + b/8)
 *   fixed IV  : byte b = byte (b%8) of SPLITMIX(SYNTH_IV_SEED + b/8), b < 12
 *   nonce i   : fixed IV XOR (0^4 || be64(i))       (TLS 1.3 style)
 *   AD i      : be64(i) || 0x17 || 0x03 0x03 || be16(len_i)   (13 bytes)
 *   PT i      : byte b = byte (b%8) of SPLITMIX(SYNTH_PT_SEED ^ (i<<32) ^ (b/8))
 *   mixed len : 64 + SPLITMIX(SYNTH_LEN_SEED + i) % 16321   (64..16384)
 */
#ifndef BSSL_AMD_SYNTH_H
#define BSSL_AMD_SYNTH_H
#include <stddef.h>
#include <stdint.h>

#define SYNTH_KEY_SEED UINT64_C(0xB055)
#define SYNTH_IV_SEED UINT64_C(0x1D5EED)
#define SYNTH_PT_SEED UINT64_C(1)
#define SYNTH_LEN_SEED UINT64_C(42)
#define SYNTH_RECORD_ALIGN 16

static inline uint64_t synth_splitmix(uint64_t x) {
  uint64_t z = x + UINT64_C(0x9E3779B97F4A7C15);
  z = (z ^ (z >> 30)) * UINT64_C(0xBF58476D1CE4E5B9);
  z = (z ^ (z >> 27)) * UINT64_C(0x94D049BB133111EB);
  return z ^ (z >> 31);
}

#ifdef __cplusplus
extern "C" {
#endif
void synth_key(uint64_t k, size_t key_len, uint8_t *out);
void synth_nonce(uint64_t i, uint8_t out[12]);
void synth_ad(uint64_t i, uint64_t len, uint8_t out[13]);
void synth_pt(uint64_t i, uint64_t len, uint8_t *out);
uint64_t synth_mixed_len(uint64_t i);
/* Fill `n` records laid out at offsets[i] (lengths lens[i]) with PT, nonces
 * and ADs (AD stride 13).  Uses OpenMP. */
void synth_fill(uint64_t first_record, size_t n, const uint64_t *offsets,
                const uint64_t *lens, uint8_t *pt, uint8_t *nonces,
                uint8_t *ads, int threads);
#ifdef __cplusplus
}
#endif
#endif
