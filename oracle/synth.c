/* synth.c -- host implementation of the synthetic workload (see synth.h). */
#include "synth.h"

void synth_key(uint64_t k, size_t key_len, uint8_t *out) {
  for (size_t b = 0; b < key_len; b++)
    out[b] = (uint8_t)(synth_splitmix(SYNTH_KEY_SEED + 16 * k + b / 8) >> (8 * (b % 8)));
}

void synth_nonce(uint64_t i, uint8_t out[12]) {
  for (int b = 0; b < 12; b++)
    out[b] = (uint8_t)(synth_splitmix(SYNTH_IV_SEED + (uint64_t)b / 8) >> (8 * (b % 8)));
  for (int b = 0; b < 8; b++) out[4 + b] ^= (uint8_t)(i >> (8 * (7 - b)));
}

void synth_ad(uint64_t i, uint64_t len, uint8_t out[13]) {
  for (int b = 0; b < 8; b++) out[b] = (uint8_t)(i >> (8 * (7 - b)));
  out[8] = 0x17;
  out[9] = 0x03;
  out[10] = 0x03;
  out[11] = (uint8_t)(len >> 8);
  out[12] = (uint8_t)len;
}

void synth_pt(uint64_t i, uint64_t len, uint8_t *out) {
  uint64_t w = 0;
  for (; w + 1 <= len / 8; w++) {
    uint64_t v = synth_splitmix(SYNTH_PT_SEED ^ (i << 32) ^ w);
    for (int b = 0; b < 8; b++) out[8 * w + b] = (uint8_t)(v >> (8 * b));
  }
  if (len % 8) {
    uint64_t v = synth_splitmix(SYNTH_PT_SEED ^ (i << 32) ^ w);
    for (uint64_t b = 0; b < len % 8; b++) out[8 * w + b] = (uint8_t)(v >> (8 * b));
  }
}

uint64_t synth_mixed_len(uint64_t i) {
  return 64 + synth_splitmix(SYNTH_LEN_SEED + i) % 16321;
}

void synth_fill(uint64_t first_record, size_t n, const uint64_t *offsets,
                const uint64_t *lens, uint8_t *pt, uint8_t *nonces,
                uint8_t *ads, int threads) {
  long long nn = (long long)n;
  (void)threads;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
  for (long long j = 0; j < nn; j++) {
    uint64_t i = first_record + (uint64_t)j;
    if (pt) synth_pt(i, lens[j], pt + offsets[j]);
    if (nonces) synth_nonce(i, nonces + 12 * (size_t)j);
    if (ads) synth_ad(i, lens[j], ads + 13 * (size_t)j);
  }
}
