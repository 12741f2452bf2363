/* bssl_amd/tls.h -- TLS record protection over device batches: the record
 * layer that calls the AEAD path.
 *
 * BSSL_AMD_TLS_AEAD is one direction of a TLS 1.2 / 1.3 connection with an
 * AEAD cipher suite -- the analogue of the reference's SSLAEADContext
 * (ssl/internal.h; ssl/ssl_aead_ctx.cc:44-123, 207-409) -- and a batch of
 * records is what do_seal_record / tls_open_record (ssl/tls_record.cc:266-317,
 * 183-236) do per record, with write/read sequence numbers seq, seq+1, ...
 *
 * Record layout (scatter, as SealScatter's out_prefix / out / out_suffix):
 *   prefix[i]  prefix_len bytes: the 5-byte record header, then for TLS 1.2
 *              AES-GCM the 8-byte explicit nonce
 *   body       record i's plaintext / ciphertext at in/out + offsets[i]
 *              (or i * record_stride), lengths[i] (or record_len) bytes
 *   suffix[i]  suffix_len bytes: for TLS 1.3 the sealed inner content type,
 *              then the 16-byte tag
 * so header ++ prefix-rest ++ body ++ suffix is the wire record.  TLS 1.3
 * records are sealed without padding; open expects unpadded records (the
 * inner type is the byte after the body) and returns it in types[i].
 */
#ifndef BSSL_AMD_TLS_H
#define BSSL_AMD_TLS_H

#include "bssl_amd/aead.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BSSL_AMD_TLS1_2_VERSION 0x0303
#define BSSL_AMD_TLS1_3_VERSION 0x0304

typedef struct bssl_amd_tls_aead_st BSSL_AMD_TLS_AEAD;

/* SSLAEADContext::Create for an AEAD cipher suite (mac_key empty):
 * `aead` is EVP_aead_aes_128_gcm(), EVP_aead_aes_256_gcm() or
 * EVP_aead_chacha20_poly1305(); AES-GCM seal contexts use the reference's
 * nonce-checking tls12 / tls13 variants (ssl_cipher_get_evp_aead,
 * ssl/ssl_cipher.cc).  fixed_iv: 4 bytes for TLS 1.2 AES-GCM, 12 otherwise.
 * `seq` is the sequence number of the first record (TLS 1.3 traffic keys
 * start at 0, which the tls13 AEAD's nonce check relies on, e_aes.cc.inc:
 * 1181-1185).  Returns NULL on error. */
BSSL_AMD_EXPORT BSSL_AMD_TLS_AEAD *BSSL_AMD_TLS_AEAD_new(
    enum evp_aead_direction_t direction, uint16_t version, const EVP_AEAD *aead,
    const uint8_t *key, size_t key_len, const uint8_t *fixed_iv, size_t fixed_iv_len,
    uint64_t seq);
BSSL_AMD_EXPORT void BSSL_AMD_TLS_AEAD_free(BSSL_AMD_TLS_AEAD *t);
BSSL_AMD_EXPORT size_t BSSL_AMD_TLS_AEAD_prefix_len(const BSSL_AMD_TLS_AEAD *t);
BSSL_AMD_EXPORT size_t BSSL_AMD_TLS_AEAD_suffix_len(const BSSL_AMD_TLS_AEAD *t);
/* The sequence number the next record will use. */
BSSL_AMD_EXPORT uint64_t BSSL_AMD_TLS_AEAD_sequence(const BSSL_AMD_TLS_AEAD *t);

typedef struct {
  size_t num_records;
  const uint8_t *in; /* device */
  uint8_t *out;      /* device, may equal in */
  const uint64_t *offsets; /* device, or NULL: i * record_stride */
  const uint64_t *lengths; /* device, or NULL: record_len */
  uint64_t record_stride;
  uint64_t record_len;
  /* Seal: the content type of record i (device, or NULL: `type` for all).
   * Open: receives the inner type (TLS 1.3) or the header type (TLS 1.2). */
  uint8_t *types;
  uint8_t type;
  uint8_t *prefix; /* device, prefix_len bytes per record */
  uint8_t *suffix; /* device, suffix_len bytes per record */
  uint8_t *status; /* device, 1 byte per record (1 = sealed / authentic), or NULL */
} BSSL_AMD_TLS_RECORDS;

/* Seal (open) num_records records with sequence numbers sequence() ..
 * sequence() + n - 1 and advance the sequence by n.  A record that fails
 * (plaintext > 2^14 bytes, a rejected nonce, a bad tag) has status 0 and
 * zeroed outputs; it still consumes its sequence number.  Returns 0 (nothing
 * launched, error queued) when the sequence number would wrap
 * (tls_record.cc:305-308) or on argument errors.  Synchronises the stream
 * for AES-GCM seal (the nonce state, see EVP_AEAD_CTX_seal_batch_device). */
BSSL_AMD_EXPORT int BSSL_AMD_TLS_AEAD_seal_records_device(BSSL_AMD_TLS_AEAD *t,
                                                          const BSSL_AMD_TLS_RECORDS *r,
                                                          void *hip_stream);
BSSL_AMD_EXPORT int BSSL_AMD_TLS_AEAD_open_records_device(BSSL_AMD_TLS_AEAD *t,
                                                          const BSSL_AMD_TLS_RECORDS *r,
                                                          void *hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* BSSL_AMD_TLS_H */
