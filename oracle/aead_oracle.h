/* aead_oracle.h -- CPU restatement of the reference bulk-AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (boringssl_amd/, include/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * The oracle is pinned against the reference's own known-answer files
 * (crypto/cipher/test/{aes_128_gcm,aes_256_gcm,chacha20_poly1305}_tests.txt,
 * third_party/wycheproof_testvectors/{aes_gcm,chacha20_poly1305}_test.txt,
 * crypto/fipsmodule/aes/aes_tests.txt, crypto/poly1305/poly1305_tests.txt),
 * converted to the JSON fixtures under tests/golden/ by tests/golden/make_golden.py, and against
 * the reference library itself compiled into oracle/_ref/ (oracle/ref/Makefile).
 */
#ifndef BSSL_AMD_AEAD_ORACLE_H
#define BSSL_AMD_AEAD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORACLE_AES_GCM = 0,          /* key 16/24/32 bytes */
  ORACLE_CHACHA20_POLY1305 = 1, /* key 32 bytes, nonce 12 bytes */
  ORACLE_XCHACHA20_POLY1305 = 2, /* key 32 bytes, nonce 24 bytes */
  ORACLE_AES_GCM_SIV = 3          /* key 16/32 bytes, nonce 12 bytes, tag 16 */
};

/* AES (FIPS-197) single block, key 16/24/32 bytes. */
void oracle_aes_encrypt_block(const uint8_t *key, size_t key_len,
                              const uint8_t in[16], uint8_t out[16]);

/* GHASH multiply X <- X*H in GF(2^128), GCM bit order. */
void oracle_gf128_mul(uint8_t x[16], const uint8_t h[16]);

/* AES-GCM seal/open.  Returns 1 on success, 0 on error / auth failure.
 * Mirrors aead_aes_gcm_sealv_impl / _openv_detached_impl
 * (crypto/fipsmodule/cipher/e_aes.cc.inc:779-867). */
int oracle_aes_gcm_seal(const uint8_t *key, size_t key_len,
                        const uint8_t *nonce, size_t nonce_len,
                        const uint8_t *in, size_t in_len, const uint8_t *ad,
                        size_t ad_len, uint8_t *out, uint8_t *tag,
                        size_t tag_len);
int oracle_aes_gcm_open(const uint8_t *key, size_t key_len,
                        const uint8_t *nonce, size_t nonce_len,
                        const uint8_t *in, size_t in_len, const uint8_t *ad,
                        size_t ad_len, const uint8_t *tag, size_t tag_len,
                        uint8_t *out);

/* ChaCha20 (RFC 8439, 32-bit counter) and Poly1305 one-shot. */
void oracle_chacha20(uint8_t *out, const uint8_t *in, size_t len,
                     const uint8_t key[32], const uint8_t nonce[12],
                     uint32_t counter);
void oracle_poly1305(uint8_t tag[16], const uint8_t *msg, size_t len,
                     const uint8_t key[32]);

/* ChaCha20-Poly1305 AEAD (crypto/cipher/e_chacha20poly1305.cc:84-333). */
int oracle_chacha20_poly1305_seal(const uint8_t key[32], const uint8_t *nonce,
                                  size_t nonce_len, const uint8_t *in,
                                  size_t in_len, const uint8_t *ad,
                                  size_t ad_len, uint8_t *out, uint8_t *tag,
                                  size_t tag_len);
int oracle_chacha20_poly1305_open(const uint8_t key[32], const uint8_t *nonce,
                                  size_t nonce_len, const uint8_t *in,
                                  size_t in_len, const uint8_t *ad,
                                  size_t ad_len, const uint8_t *tag,
                                  size_t tag_len, uint8_t *out);

/* AES-GCM-SIV (RFC 8452; crypto/cipher/e_aesgcmsiv.cc:533-867). */
int oracle_aes_gcm_siv_seal(const uint8_t *key, size_t key_len, const uint8_t *nonce,
                            size_t nonce_len, const uint8_t *in, size_t in_len,
                            const uint8_t *ad, size_t ad_len, uint8_t *out, uint8_t *tag,
                            size_t tag_len);
int oracle_aes_gcm_siv_open(const uint8_t *key, size_t key_len, const uint8_t *nonce,
                            size_t nonce_len, const uint8_t *in, size_t in_len,
                            const uint8_t *ad, size_t ad_len, const uint8_t *tag,
                            size_t tag_len, uint8_t *out);

/* HChaCha20 and XChaCha20-Poly1305 (crypto/chacha/chacha.cc:43-63,
 * crypto/cipher/e_chacha20poly1305.cc:233-256, 310-330). */
void oracle_hchacha20(uint8_t out[32], const uint8_t key[32],
                      const uint8_t nonce[16]);
int oracle_xchacha20_poly1305_seal(const uint8_t key[32], const uint8_t *nonce,
                                   size_t nonce_len, const uint8_t *in,
                                   size_t in_len, const uint8_t *ad,
                                   size_t ad_len, uint8_t *out, uint8_t *tag,
                                   size_t tag_len);
int oracle_xchacha20_poly1305_open(const uint8_t key[32], const uint8_t *nonce,
                                   size_t nonce_len, const uint8_t *in,
                                   size_t in_len, const uint8_t *ad,
                                   size_t ad_len, const uint8_t *tag,
                                   size_t tag_len, uint8_t *out);

/* Batch form used by the parity tests and the cpu_baseline leg.  Record i:
 * key = keys + key_len * (key_index ? key_index[i] : 0), input at
 * in + offsets[i] (length lens[i]), nonce at nonces + i*nonce_len, AD at
 * ad + ad_offsets[i] (length ad_lens[i]).  Writes out + offsets[i] and
 * tags + i*tag_len.  For open (`seal` = 0) `tags` is read and `status[i]`
 * receives 1/0.  Runs on `threads` OpenMP threads.  Returns number of
 * records that failed. */
size_t oracle_batch(int aead, int seal, const uint8_t *keys, size_t key_len,
                    const uint32_t *key_index, size_t n, const uint8_t *in,
                    uint8_t *out, const uint64_t *offsets,
                    const uint64_t *lens, const uint8_t *nonces,
                    size_t nonce_len, const uint8_t *ad,
                    const uint64_t *ad_offsets, const uint64_t *ad_lens,
                    uint8_t *tags, size_t tag_len, uint8_t *status,
                    int threads);

#ifdef __cplusplus
}
#endif

#endif
