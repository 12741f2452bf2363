/* bssl_amd/test_hooks.h -- test-only entry points of libbssl_amd.so.
 *
 * Not part of the EVP_AEAD surface (include/bssl_amd/aead.h): these expose
 * internal layouts and diagnostic switches so the parity tests can check the
 * key-setup paths against each other and exercise fallback paths that a
 * normal run never takes.  A production caller has no reason to use them. */
#ifndef BSSL_AMD_TEST_HOOKS_H
#define BSSL_AMD_TEST_HOOKS_H

#include "bssl_amd/aead.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The per-key AES-GCM device tables (internal layout, sizeof GcmKeyDev bytes
 * per key) of n keys of key_len bytes, built on the host (on_device = 0, the
 * EVP_AEAD_CTX_init path) or by the device key-setup kernel (1, the keyset
 * path) and copied to `out`.  Returns n, 0 on error; with out == NULL
 * returns the per-key table size.  The two paths must agree byte for byte
 * (tests/test_key_setup.py). */
BSSL_AMD_EXPORT size_t BSSL_AMD_gcm_key_tables(const uint8_t *keys, size_t key_len, size_t n,
                                               int on_device, uint8_t *out);

/* The table-free AES-GCM engine hands each record's E_K(J0) from the wave
 * that computes a batch of them to the record's end (gcm_bs.hip).  A record
 * end that has not received its value after a bounded wait computes it
 * itself.  on = 0 switches the batched production off for later launches of
 * this process, so every record end takes that fallback (one parity run
 * exercises it); 1 restores the default.  Returns the previous setting. */
BSSL_AMD_EXPORT int BSSL_AMD_test_set_bs_ek0_producers(int on);

/* The experimental mixed-role AES-GCM engine (gcm_mix.hip; also selected by
 * BSSL_AMD_GCM_MODE=mix2|mix4|mix6): bitsliced_waves (2, 4 or 6) of each
 * workgroup's 16 waves run the table-free engine, the others the T-table
 * engine, on one unit counter, for one-key uniform AES-128-GCM batches of
 * records of 4 KiB or more (other batches take the T-table engine).  Returns
 * the previous engine (restore it with BSSL_AMD_set_aes_gcm_engine), -1 for
 * another wave count. */
BSSL_AMD_EXPORT int BSSL_AMD_test_set_gcm_mix(int bitsliced_waves);

#ifdef __cplusplus
}
#endif

#endif /* BSSL_AMD_TEST_HOOKS_H */
