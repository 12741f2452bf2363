/* bssl_amd/aead.h -- MI355X bulk-AEAD record engine, C ABI.
 *
 * Part 1 re-declares BoringSSL's EVP_AEAD surface (include/openssl/aead.h of
 * the reference) with the same names, argument meaning, return convention
 * (1 = success, 0 = failure), zero-on-error behaviour and CIPHER_R_* reason
 * codes, so a caller of the reference binds to this library unchanged.  Each
 * declaration cites the reference declaration it replaces.  Single-record
 * calls take HOST pointers (as in the reference) and run on the GPU (copy in,
 * one-record batch, copy out); there is no CPU implementation behind them.
 *
 * Part 2 is the batch extension that is the hot path: N independent
 * `EVP_AEAD_CTX_seal_scatter`-equivalent records (aead.cc.inc:163-209) whose
 * buffers are already resident in device memory, launched on a caller-given
 * HIP stream.  It has no reference counterpart; its per-record semantics are
 * exactly those of the single-record calls.
 *
 * Plain C types only (pointers, sizes); a HIP stream is passed as void*.
 */
#ifndef BSSL_AMD_AEAD_H
#define BSSL_AMD_AEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSSL_AMD_EXPORT __attribute__((visibility("default")))

/* ---- Part 1: EVP_AEAD surface (reference include/openssl/aead.h) -------- */

typedef struct evp_aead_st EVP_AEAD;             /* base.h:306 */
typedef struct evp_aead_ctx_st EVP_AEAD_CTX;     /* base.h:305 */
typedef struct engine_st ENGINE;                 /* base.h:321, unused */
typedef struct crypto_ivec_st CRYPTO_IVEC;       /* aead.h:402 */
typedef struct crypto_iovec_st CRYPTO_IOVEC;     /* aead.h:409 */

/* aead.h:222-237: caller-owned context with 560 bytes of opaque state.  Here
 * the state holds a handle to the device-resident key schedule. */
union evp_aead_ctx_st_state {
  uint8_t opaque[560];
  uint64_t alignment;
};
struct evp_aead_ctx_st {
  const EVP_AEAD *aead;
  union evp_aead_ctx_st_state state;
  uint8_t tag_len;
};

struct crypto_ivec_st {   /* aead.h:402-405 */
  const uint8_t *in;
  size_t len;
};
struct crypto_iovec_st {  /* aead.h:409-414 */
  uint8_t *out;
  const uint8_t *in;
  size_t len;
};

#define EVP_AEAD_MAX_KEY_LENGTH 80       /* aead.h:239 */
#define EVP_AEAD_MAX_NONCE_LENGTH 24     /* aead.h:243 */
#define EVP_AEAD_MAX_OVERHEAD 64         /* aead.h:247 */
#define EVP_AEAD_MAX_OPEN_OVERHEAD 320   /* aead.h:253 */
#define EVP_AEAD_DEFAULT_TAG_LENGTH 0    /* aead.h:258 */

enum evp_aead_direction_t {              /* aead.h:592-595 */
  evp_aead_open,
  evp_aead_seal
};

/* AEAD algorithms (aead.h:100-126, 583-586). */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_128_gcm(void);        /* aead.h:100 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_192_gcm(void);        /* aead.h:113 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_256_gcm(void);        /* aead.h:122 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_chacha20_poly1305(void);  /* aead.h:126 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_xchacha20_poly1305(void); /* aead.h:130 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_128_gcm_siv(void);    /* aead.h:142 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_256_gcm_siv(void);    /* aead.h:145 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_128_gcm_tls12(void);  /* aead.h:583 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_256_gcm_tls12(void);  /* aead.h:584 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_128_gcm_tls13(void);  /* aead.h:585 */
BSSL_AMD_EXPORT const EVP_AEAD *EVP_aead_aes_256_gcm_tls13(void);  /* aead.h:586 */

/* Utility functions (aead.h:204-217). */
BSSL_AMD_EXPORT size_t EVP_AEAD_key_length(const EVP_AEAD *aead);
BSSL_AMD_EXPORT size_t EVP_AEAD_nonce_length(const EVP_AEAD *aead);
BSSL_AMD_EXPORT size_t EVP_AEAD_max_overhead(const EVP_AEAD *aead);
BSSL_AMD_EXPORT size_t EVP_AEAD_max_tag_len(const EVP_AEAD *aead);

/* Context lifecycle (aead.h:264-292, 599-606). */
BSSL_AMD_EXPORT void EVP_AEAD_CTX_zero(EVP_AEAD_CTX *ctx);
BSSL_AMD_EXPORT EVP_AEAD_CTX *EVP_AEAD_CTX_new(const EVP_AEAD *aead,
                                               const uint8_t *key,
                                               size_t key_len, size_t tag_len);
BSSL_AMD_EXPORT void EVP_AEAD_CTX_free(EVP_AEAD_CTX *ctx);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_init(EVP_AEAD_CTX *ctx, const EVP_AEAD *aead,
                                      const uint8_t *key, size_t key_len,
                                      size_t tag_len, ENGINE *impl);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_init_with_direction(
    EVP_AEAD_CTX *ctx, const EVP_AEAD *aead, const uint8_t *key,
    size_t key_len, size_t tag_len, enum evp_aead_direction_t dir);
BSSL_AMD_EXPORT void EVP_AEAD_CTX_cleanup(EVP_AEAD_CTX *ctx);
BSSL_AMD_EXPORT const EVP_AEAD *EVP_AEAD_CTX_aead(const EVP_AEAD_CTX *ctx); /* aead.h:533 */

/* Seal/open with host buffers (aead.h:314-399, 447-530). */
BSSL_AMD_EXPORT int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX *ctx, uint8_t *out,
                                      size_t *out_len, size_t max_out_len,
                                      const uint8_t *nonce, size_t nonce_len,
                                      const uint8_t *in, size_t in_len,
                                      const uint8_t *ad, size_t ad_len);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_open(const EVP_AEAD_CTX *ctx, uint8_t *out,
                                      size_t *out_len, size_t max_out_len,
                                      const uint8_t *nonce, size_t nonce_len,
                                      const uint8_t *in, size_t in_len,
                                      const uint8_t *ad, size_t ad_len);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_seal_scatter(
    const EVP_AEAD_CTX *ctx, uint8_t *out, uint8_t *out_tag,
    size_t *out_tag_len, size_t max_out_tag_len, const uint8_t *nonce,
    size_t nonce_len, const uint8_t *in, size_t in_len,
    const uint8_t *extra_in, size_t extra_in_len, const uint8_t *ad,
    size_t ad_len);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_open_gather(
    const EVP_AEAD_CTX *ctx, uint8_t *out, const uint8_t *nonce,
    size_t nonce_len, const uint8_t *in, size_t in_len, const uint8_t *in_tag,
    size_t in_tag_len, const uint8_t *ad, size_t ad_len);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_sealv(const EVP_AEAD_CTX *ctx,
                                       const CRYPTO_IOVEC *iovec,
                                       size_t num_iovec, uint8_t *out_tag,
                                       size_t *out_tag_len,
                                       size_t max_out_tag_len,
                                       const uint8_t *nonce, size_t nonce_len,
                                       const CRYPTO_IVEC *aadvec,
                                       size_t num_aadvec);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_openv(const EVP_AEAD_CTX *ctx,
                                       const CRYPTO_IOVEC *iovec,
                                       size_t num_iovec,
                                       size_t *out_total_bytes,
                                       const uint8_t *nonce, size_t nonce_len,
                                       const CRYPTO_IVEC *aadvec,
                                       size_t num_aadvec);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_openv_detached(
    const EVP_AEAD_CTX *ctx, const CRYPTO_IOVEC *iovec, size_t num_iovec,
    const uint8_t *nonce, size_t nonce_len, const uint8_t *in_tag,
    size_t in_tag_len, const CRYPTO_IVEC *aadvec, size_t num_aadvec);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_tag_len(const EVP_AEAD_CTX *ctx,
                                         size_t *out_tag_len, size_t in_len,
                                         size_t extra_in_len);  /* aead.h:623 */
BSSL_AMD_EXPORT int EVP_AEAD_CTX_get_iv(const EVP_AEAD_CTX *ctx,
                                        const uint8_t **out_iv,
                                        size_t *out_len);        /* aead.h:608 */

/* Error queue (reference include/openssl/err.h:52-67, 362; thread-local,
 * ERR_NUM_ERRORS deep).  Packed codes are ERR_PACK(lib, reason). */
#define ERR_LIB_CIPHER 30
#define ERR_R_OVERFLOW (5 | 64)
#define ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED (2 | 64)
#define ERR_R_INTERNAL_ERROR (4 | 64)
#define ERR_R_MALLOC_FAILURE (1 | 64)
static inline int ERR_GET_LIB(uint32_t e) { return (int)((e >> 24) & 0xff); }
static inline int ERR_GET_REASON(uint32_t e) { return (int)(e & 0xfff); }
BSSL_AMD_EXPORT uint32_t ERR_get_error(void);
BSSL_AMD_EXPORT uint32_t ERR_peek_error(void);
BSSL_AMD_EXPORT uint32_t ERR_peek_last_error(void);
BSSL_AMD_EXPORT void ERR_clear_error(void);

/* Reason codes, include/openssl/cipher.h:792-817 (same numbers). */
#define CIPHER_R_BAD_DECRYPT 101
#define CIPHER_R_BAD_KEY_LENGTH 102
#define CIPHER_R_BUFFER_TOO_SMALL 103
#define CIPHER_R_CTRL_NOT_IMPLEMENTED 104
#define CIPHER_R_INVALID_NONCE_SIZE 111
#define CIPHER_R_INVALID_OPERATION 112  /* cipher.h:804 */
#define CIPHER_R_NO_DIRECTION_SET 124
#define CIPHER_R_OUTPUT_ALIASES_INPUT 115
#define CIPHER_R_TAG_TOO_LARGE 116
#define CIPHER_R_TOO_LARGE 117
#define CIPHER_R_UNSUPPORTED_KEY_SIZE 120
#define CIPHER_R_UNSUPPORTED_NONCE_SIZE 121
#define CIPHER_R_UNSUPPORTED_TAG_SIZE 122
#define CIPHER_R_INVALID_NONCE 125

/* ---- Part 2: device-resident record batches (new) ----------------------- */

/* A batch of independent records.  Every pointer is a DEVICE pointer.
 * Record i: input in + offsets[i] (or i*record_stride when offsets == NULL)
 * of lengths[i] bytes (or record_len when lengths == NULL); output to the same
 * offset of `out` (out == in is in-place); nonce at nonces + i*nonce_len; AD
 * at ad + ad_offsets[i] (or i*ad_stride) of ad_lengths[i] (or ad_len) bytes;
 * tag at tags + i*tag_len (tag_len = the context's tag length).  status[i]
 * (optional) receives 1 on success, 0 on failure (authentication failure on
 * open, or a per-record limit exceeded: GCM 2^36-32 bytes gcm.cc.inc:409,
 * ChaCha20-Poly1305 2^38-64 bytes e_chacha20poly1305.cc:138); a failed
 * record's output (and, for seal, tag) is zero-filled, as the reference does
 * for a failed single call (aead.cc.inc:132-139, 539-547). */
typedef struct bssl_amd_batch_st {
  size_t num_records;
  const uint8_t *in;
  uint8_t *out;
  const uint64_t *offsets;
  const uint64_t *lengths;
  uint64_t record_stride;
  uint64_t record_len;
  const uint8_t *nonces;
  size_t nonce_len;
  const uint8_t *ad;
  const uint64_t *ad_offsets;
  const uint64_t *ad_lengths;
  uint64_t ad_stride;
  uint64_t ad_len;
  uint8_t *tags;
  uint8_t *status;
  /* Keysets only: key_index[i] selects the key of record i.  Records with
   * equal key_index should be contiguous for speed (any order is correct). */
  const uint32_t *key_index;
} BSSL_AMD_BATCH;

/* Seal / open every record of `batch` with the key of `ctx` (key_index is
 * ignored), enqueued on `hip_stream` (NULL = default stream).  Returns 1 if
 * the batch was launched (per-record results in status/tags), 0 on an
 * argument error (pushed to the error queue).  Asynchronous with respect to
 * the host.
 *
 * For the stateful EVP_aead_aes_*_gcm_tls12 / _tls13 contexts a sealed batch
 * is N calls in record order, each with the reference's monotonic-nonce check
 * (e_aes.cc.inc:1071-1100, 1162-1202; nonce_len must be 12): a record whose
 * nonce fails it gets status 0 and zeroed output/tag, and the context's nonce
 * state advances as after the N calls.  These seal calls synchronise
 * `hip_stream` (the state lives in the host-side context).  Keysets reject
 * the tls variants (CIPHER_R_CTRL_NOT_IMPLEMENTED). */
BSSL_AMD_EXPORT int EVP_AEAD_CTX_seal_batch_device(const EVP_AEAD_CTX *ctx,
                                                   const BSSL_AMD_BATCH *batch,
                                                   void *hip_stream);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_open_batch_device(const EVP_AEAD_CTX *ctx,
                                                   const BSSL_AMD_BATCH *batch,
                                                   void *hip_stream);

/* A batch of non-contiguous records: the device form of N
 * EVP_AEAD_CTX_sealv / _openv_detached calls (aead.cc.inc:316-361, 531-584).
 * Every pointer is a DEVICE pointer, including the ones inside the CRYPTO_IOVEC
 * / CRYPTO_IVEC arrays.  Record i is the concatenation of
 * iovecs[iovec_start[i] .. iovec_start[i+1]) (each chunk's output goes to its
 * `out`, which may equal its `in`), its AD the concatenation of
 * aadvecs[aadvec_start[i] .. aadvec_start[i+1]) (aadvecs NULL = no AD);
 * nonce at nonces + i*nonce_len; tag at tags + i*tag_len (written by seal,
 * read by open).  status[i] (optional) as for BSSL_AMD_BATCH; a failed
 * record's chunks (and, for seal, tag) are zero-filled (clear_iovec,
 * aead.cc.inc:310-333).  The bulk kernels walk each record's chunks in place
 * (no staging copy, no gather/scatter pass); the call only enqueues work on
 * `hip_stream` (one small kernel for the per-record totals, then the bulk
 * kernels) and never synchronises it.  Chunks of one batch must not partially
 * overlap (aead.cc.inc:281-308; not checked on the device). */
typedef struct bssl_amd_iov_batch_st {
  size_t num_records;
  const CRYPTO_IOVEC *iovecs;
  const uint64_t *iovec_start;  /* num_records + 1 entries */
  const CRYPTO_IVEC *aadvecs;
  const uint64_t *aadvec_start; /* num_records + 1 entries */
  const uint8_t *nonces;
  size_t nonce_len;
  uint8_t *tags;
  uint8_t *status;
} BSSL_AMD_IOV_BATCH;

BSSL_AMD_EXPORT int EVP_AEAD_CTX_sealv_batch_device(const EVP_AEAD_CTX *ctx,
                                                    const BSSL_AMD_IOV_BATCH *batch,
                                                    void *hip_stream);
BSSL_AMD_EXPORT int EVP_AEAD_CTX_openv_detached_batch_device(const EVP_AEAD_CTX *ctx,
                                                             const BSSL_AMD_IOV_BATCH *batch,
                                                             void *hip_stream);

/* Many keys of one AEAD (the multi-session case): key material for all keys
 * is expanded once and kept resident in device memory. */
typedef struct bssl_amd_keyset_st BSSL_AMD_KEYSET;
BSSL_AMD_EXPORT BSSL_AMD_KEYSET *BSSL_AMD_KEYSET_new(const EVP_AEAD *aead,
                                                     const uint8_t *keys,
                                                     size_t num_keys,
                                                     size_t tag_len);
BSSL_AMD_EXPORT void BSSL_AMD_KEYSET_free(BSSL_AMD_KEYSET *ks);
BSSL_AMD_EXPORT size_t BSSL_AMD_KEYSET_num_keys(const BSSL_AMD_KEYSET *ks);
BSSL_AMD_EXPORT int BSSL_AMD_KEYSET_seal_batch_device(
    const BSSL_AMD_KEYSET *ks, const BSSL_AMD_BATCH *batch, void *hip_stream);
BSSL_AMD_EXPORT int BSSL_AMD_KEYSET_open_batch_device(
    const BSSL_AMD_KEYSET *ks, const BSSL_AMD_BATCH *batch, void *hip_stream);

/* Device selection for the calling host thread (one process or thread per
 * GPU).  Returns 1 on success. */
BSSL_AMD_EXPORT int BSSL_AMD_set_device(int device);
BSSL_AMD_EXPORT int BSSL_AMD_device_count(void);

/* ---- Bench / test support (not part of the EVP surface) ----------------- */

/* Fills a device batch with the synthetic workload of SURVEY.md 8(d)
 * (definition in oracle/synth.h; this is an independent device-side
 * implementation): PT of records first..first+n-1 at offsets/lengths, 12-byte
 * nonces and 13-byte ADs (stride 13). */
BSSL_AMD_EXPORT int BSSL_AMD_synth_fill_device(uint64_t first_record, size_t n,
                                               const uint64_t *offsets,
                                               const uint64_t *lengths,
                                               uint8_t *pt, uint8_t *nonces,
                                               uint8_t *ads, void *hip_stream);

/* Kernel-level timing for this host thread.  While enabled, every batch
 * launch records HIP events on its stream around its bulk kernel (no host
 * synchronisation).  BSSL_AMD_collect_kernel_times waits for the recorded
 * launches, writes up to `max` durations (ms) in launch order and returns how
 * many launches were pending.  last_kernel_ms / _name describe the most
 * recent one. */
BSSL_AMD_EXPORT void BSSL_AMD_set_kernel_timing(int enable);
BSSL_AMD_EXPORT size_t BSSL_AMD_collect_kernel_times(double *out_ms, size_t max);
BSSL_AMD_EXPORT double BSSL_AMD_last_kernel_ms(void);
BSSL_AMD_EXPORT const char *BSSL_AMD_last_kernel_name(void);

/* AES engine of the AES-GCM bulk path (process-wide; both produce the same
 * bytes as the reference).  BSSL_AMD_AES_GCM_ENGINE_BITSLICED: AES bitsliced
 * on the VALU with no lookup table (the reference's own constant-time
 * approach, aes_nohw.cc.inc:508); BSSL_AMD_AES_GCM_ENGINE_TABLE: AES by
 * bank-replicated T-tables in LDS.  The initial value comes from the
 * environment variable BSSL_AMD_GCM_MODE ("bs" or "table"), read once.
 * Returns the previous engine, or -1 (and changes nothing) for an unknown
 * value.  Batches already enqueued keep the engine they were launched with. */
#define BSSL_AMD_AES_GCM_ENGINE_TABLE 0
#define BSSL_AMD_AES_GCM_ENGINE_BITSLICED 1
BSSL_AMD_EXPORT int BSSL_AMD_set_aes_gcm_engine(int engine);
BSSL_AMD_EXPORT int BSSL_AMD_aes_gcm_engine(void);

/* Test-only entry points (the internal key-table layout, diagnostic switches)
 * are declared in bssl_amd/test_hooks.h, not here. */

#ifdef __cplusplus
}
#endif

#endif /* BSSL_AMD_AEAD_H */
