// internal.h -- definitions shared by the host C-ABI layer and the HIP kernels.
//
// Device data layout (all resident in HBM, 16-byte aligned):
//
//   GcmKeyDev   one per AES-GCM key (12,816 bytes): the AES round keys
//               (T-table and plain forms, and the bitsliced engine's per-round
//               AddRoundKey masks), the GHASH nibble table of H^16 and the
//               powers H^1..H^17 as multipliers of the constant-time VALU
//               product (gf128_ct.h).
//               Equivalent of the reference's GCM128_KEY
//               (crypto/fipsmodule/aes/internal.h:325-334), re-laid-out for the
//               LDS-table GHASH of gcm.hip.
//   ChaChaKeyDev one per ChaCha20-Poly1305 key (32 bytes).
//   BatchDesc   the record-batch descriptor passed by value to the kernels.
#ifndef BSSL_AMD_INTERNAL_H
#define BSSL_AMD_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>

namespace bssl_amd {

struct alignas(16) GcmKeyDev {
  // Round keys as little-endian words of the FIPS-197 schedule bytes; the
  // middle rounds (1..nr-1) are stored rotated left by 16 bits, which is how
  // the T-table round of gcm.hip consumes them.
  uint32_t rk[15][4];
  uint32_t nr;
  uint32_t key_bytes;
  uint32_t pad[2];
  // The same schedule unrotated (bitsliced kernel: bit masks per round).
  uint32_t rk_plain[15][4];
  // H^k for k = 1..17 (index 0 unused) in the reversed domain of gf128_ct.h,
  // prepared as multipliers (gf_prep): the constant-time VALU products of the
  // record-end combine, the tag and the AD / J0 hashes (H^17: the one-record
  // kernel folds the tag's last x H into the lane weights).
  uint32_t hpow_ct[18][4];
  // htab16[pos][v] = (element with nibble `pos` equal to v) * H^16, as 4
  // little-endian words of the 16 GCM-order bytes.  Nibble position
  // pos = 2*k + 0 is the high nibble of byte k, 2*k + 1 the low nibble.
  // (Rounds 1-2 also held H, H^2, H^4, H^8, H^32 for the record-end tree,
  // which is now the constant-time VALU product.)
  uint32_t htab16[32][16][4];
  // AddRoundKey of the bitsliced engine (gcm_bs.hip, bs16_aes.h): bsmask[r][i]
  // with i = 32*h + 8*row + bit is the mask XORed into state register (row, h,
  // bit) in round r -- 0xffff in the low half when that bit of round-key
  // column h is set, 0xffff0000 when that bit of column h + 2 is (the engine
  // holds columns h and h + 2 in the two halves of a register).  Read by
  // scalar loads, 64 per round, so no SALU work derives them in the rounds.
  uint32_t bsmask[15][64];
};
static_assert(sizeof(GcmKeyDev) == 240 + 16 + 240 + 18 * 16 + 8192 + 15 * 256, "layout");

struct alignas(16) ChaChaKeyDev {
  uint32_t k[8];
};

enum AeadKind : int {
  kAeadAesGcm = 0,
  kAeadChaChaPoly = 1,
  kAeadXChaChaPoly = 2,
  kAeadAesGcmSiv = 3
};

// Device chunk descriptors of iovec records: CRYPTO_IOVEC / CRYPTO_IVEC
// (reference include/openssl/aead.h:400-414) on the device.
struct IovecDev {
  uint8_t *out;
  const uint8_t *in;
  uint64_t len;
};
struct IvecDev {
  const uint8_t *in;
  uint64_t len;
};

// Record-batch descriptor (device pointers), see BSSL_AMD_BATCH.
struct BatchDesc {
  const uint8_t *in;
  uint8_t *out;
  const uint64_t *offsets;
  const uint64_t *lengths;
  uint64_t record_stride;
  uint64_t record_len;
  const uint8_t *nonces;
  uint64_t nonce_len;
  const uint8_t *ad;
  const uint64_t *ad_offsets;
  const uint64_t *ad_lengths;
  uint64_t ad_stride;
  uint64_t ad_len;
  uint8_t *tags;
  uint8_t *status;
  const uint32_t *key_index;
  uint64_t num_records;
  uint32_t tag_len;
  uint32_t num_keys;
  // Processing order (device, num_records entries) or null for 0..n-1; set by
  // the launchers for ragged batches (sched.hip), never by callers.
  const uint32_t *order;
  // With `order`: the processing positions one launch covers, [*split_lo,
  // *split_hi) (null: 0 and num_records) -- length classes of a ragged batch
  // (records of 4 KiB or more, the shorter ones, ...), which take kernels with
  // different lanes per record (gcm.hip).
  const uint32_t *split_lo;
  const uint32_t *split_hi;
  // Per-record precondition flags (device, 1 = the record may be sealed) or
  // null: the tls12/tls13 nonce checks of tls_scan.hip.  A record with flag 0
  // fails like a reference call that returned 0 (zeroed output, status 0).
  const uint8_t *valid;
  // Extra trailing message bytes (the reference's `extra_in` of seal_scatter,
  // aead.cc.inc:163-209; the TLS 1.3 inner content type): extra_len bytes per
  // record, read at extra + i*extra_stride and sealed (opened) after the
  // record's `in` bytes; their output goes to extra_out + i*extra_out_stride.
  // Tags are at tags + i*tag_stride (0 = tag_len).  Set by the TLS record
  // layer only; the public batch leaves them 0/null.
  const uint8_t *extra;
  uint8_t *extra_out;
  uint32_t extra_len;
  uint32_t extra_stride;
  uint32_t extra_out_stride;
  uint32_t tag_stride;
  // iovec records walked in place by the AES-GCM kernels (iovec.hip,
  // EVP_AEAD_CTX_sealv_batch_device): when `iovecs` is set, record i's message
  // is the concatenation of iovecs[iovec_start[i] .. iovec_start[i+1]) and its
  // AD that of aadvecs[aadvec_start[i] ..] (or none); `lengths` / `ad_lengths`
  // hold the totals and in / out / offsets / ad are unused.  Null otherwise.
  const IovecDev *iovecs;
  const uint64_t *iovec_start;
  const IvecDev *aadvecs;
  const uint64_t *aadvec_start;
  // Single-record host calls (aead_api.cc one_record): when set, the
  // one-record kernels write done_seq here (mapped host memory) after every
  // other store of the record has completed, so the host can return as soon
  // as it sees the value instead of waiting for the stream.  Null otherwise
  // (the other kernels ignore it).
  uint32_t *done;
  uint32_t done_seq;
  // ... and the record's 12-byte nonce (inl bit 0) and its AD of at most 16
  // bytes, zero-padded (inl bit 1), passed by value, so the one-record kernels
  // start the cipher while the record itself is still in flight.  0 otherwise.
  uint32_t inl;
  uint32_t inl_nonce[3];
  uint32_t inl_ad[4];
};

// Tag / extra addresses of record i.
inline __host__ __device__ uint8_t *batch_tag(const BatchDesc &b, uint64_t i) {
  return b.tags + i * (b.tag_stride ? b.tag_stride : b.tag_len);
}
inline __host__ __device__ const uint8_t *batch_extra_in(const BatchDesc &b, uint64_t i) {
  return b.extra + i * b.extra_stride;
}
inline __host__ __device__ uint8_t *batch_extra_out(const BatchDesc &b, uint64_t i) {
  return b.extra_out + i * b.extra_out_stride;
}

// HIP events recorded on the launch stream immediately before and after the
// dominant (bulk) kernel of a batch, for kernel-level timing.
struct KernelEvents {
  void *start;
  void *stop;
};

// Kernel launchers (gcm.hip / chacha.hip).  Return 0 on success or a HIP
// error code.  `ev` (optional) brackets the bulk kernel.
// `engine`: the AES-GCM engine for this batch (GcmEngine; the caller reads
// gcm_engine() once per batch).
int launch_gcm(const GcmKeyDev *keys, const BatchDesc &b, bool open,
               int nr, void *stream, const KernelEvents *ev, int engine);
// AES-GCM engine of the bulk path: the bitsliced table-free engine
// (gcm_bs.hip) or the LDS T-table engine (gcm.hip).  Process-wide; the
// initial value comes from BSSL_AMD_GCM_MODE ("bs" / "bs16" or "table"),
// read once; BSSL_AMD_set_aes_gcm_engine changes it.
enum GcmEngine : int { kGcmEngineTable = 0, kGcmEngineBitsliced = 1, kGcmEngineMix = 2 };
int gcm_engine();
int set_gcm_engine(int engine);  // returns the previous engine, or -1 (bad value)
int launch_gcm_bs(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr,
                  hipStream_t stream, const KernelEvents *ev);
// The experimental mixed-role engine (gcm_mix.hip; BSSL_AMD_GCM_MODE=mixN,
// N bitsliced waves of 16): eligible batches and the launcher.
int gcm_mix_waves();
int set_gcm_mix(int nb);  // selects the mixed engine with nb bitsliced waves (2, 4, 6)
bool gcm_mix_eligible(const BatchDesc &b, int nr);
int launch_gcm_mix(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nb, hipStream_t s,
                   const KernelEvents *ev);
// Test switch of the table-free engine's batched E_K(J0) production (on by
// default; off: every record end computes its own after the bounded wait).
// Returns the previous setting.
bool set_bs_ek0_producers(bool on);
// Builds `order` (n entries) grouping records by length class, longest first;
// `scratch` holds 128 uint32.  Returns 0 or a HIP error code.
int build_length_order(const uint64_t *lengths, uint64_t n, uint32_t *order, uint32_t *scratch,
                       void *stream);
// The length classes of build_length_order (sched.hip uses these): class
// c = kSchedClasses - 1 - len / kSchedClassBytes (the longest records, of
// (kSchedClasses - 1) * kSchedClassBytes bytes or more, in class 0); scratch
// holds the class histogram, then the class cursors, which end the scatter at
// the end of their class.
constexpr int kSchedClasses = 64;
constexpr uint64_t kSchedClassBytes = 256;
// The scratch word that then holds the number of records of min_len bytes or
// more (a multiple of kSchedClassBytes): the cursor of the last class whose
// records are that long.
constexpr int split_word_for(uint64_t min_len) {
  return kSchedClasses + (kSchedClasses - 1 - (int)(min_len / kSchedClassBytes));
}
// Processing positions [0, scratch[kSplitWord]) hold the records of 4096
// bytes or more, the rest the shorter ones ...
constexpr int kSplitWord = split_word_for(4096);
// ... and [0, scratch[kSplitWord2k]) the records of 2048 bytes or more.
constexpr int kSplitWord2k = split_word_for(2048);
static_assert(kSplitWord == 64 + 47 && kSplitWord2k == 64 + 55, "length classes of sched.hip");
// Whether a batch is worth reordering (ragged and large enough).
inline bool wants_length_order(const BatchDesc &b) {
  return b.lengths && b.num_records >= 4096 && b.num_records < (uint64_t(1) << 32);
}
// AES-GCM-SIV (gcm_siv.hip); uses GcmKeyDev::rk_plain of the master key.
int launch_gcm_siv(const GcmKeyDev *keys, const BatchDesc &b, bool open, int nr, void *stream,
                   const KernelEvents *ev);
// xchacha: XChaCha20-Poly1305 (24-byte nonces, per-record HChaCha20 subkey).
int launch_chacha(const ChaChaKeyDev *keys, const BatchDesc &b, bool open, bool xchacha,
                  void *stream, const KernelEvents *ev);
// Whether launch_gcm / launch_chacha would run this batch on a one-record
// kernel, the only kernels that write the completion word BatchDesc::done.
bool gcm_takes_one_record_kernel(const BatchDesc &b, int engine);
bool chacha_takes_one_record_kernel(const BatchDesc &b);
// tls12 / tls13 nonce checks over a batch of seal calls (tls_scan.hip):
// writes valid[i] (device) and advances the context's nonce state in place
// (min_next_nonce, mask); synchronises `stream`.  and_into: valid[i] &= the
// check instead of =.  Returns 0 or an error code.
int tls_nonce_scan(const uint8_t *nonces, uint64_t n, int tls, uint64_t *min_next,
                   uint64_t *mask, uint8_t *valid, int and_into, void *stream);
// TLS record layer (tls_records.hip): per-record nonce, header/prefix, AD and
// inner type of a batch of records with sequence numbers seq .. seq + n - 1.
struct TlsPrepare {
  uint64_t n;
  const uint64_t *lengths;  // or record_len for all
  uint64_t record_len;
  const uint8_t *types;     // or `type` for all
  uint8_t type;
  uint8_t fixed_iv[12];
  uint64_t seq;
  int xor_nonce;            // fixed_iv XOR seq (TLS 1.3, TLS 1.2 ChaCha) vs fixed || seq
  int tls13;
  uint16_t record_version;  // header and TLS 1.2 AD version (0x0303)
  uint32_t explicit_len;    // 8 for TLS 1.2 AES-GCM, else 0
  uint32_t extra_len;       // 1 for TLS 1.3 (inner type), else 0
  uint32_t tag_len;
  uint32_t prefix_len;      // 5 + explicit_len
  uint32_t ad_stride;       // 13 (TLS 1.2) or 5 (TLS 1.3)
  int open;                 // records are received: header/explicit nonce read from prefix
  uint8_t *nonces, *prefix, *ad, *extra, *valid;
};
int launch_tls_prepare(const TlsPrepare &p, void *stream);
// Batches of non-contiguous records (iovec.hip).
struct IovBatchDesc {
  uint64_t num_records;
  const IovecDev *iovecs;
  const uint64_t *iovec_start;   // num_records + 1 entries
  const IvecDev *aadvecs;        // or null (no AD)
  const uint64_t *aadvec_start;  // num_records + 1 entries
  const uint8_t *nonces;
  uint64_t nonce_len;
  uint8_t *tags;
  uint8_t *status;
};
// Runs the bulk kernels over an iovec batch (a BatchDesc with `iovecs` set,
// whose tag_len / key fields the runner fills in).  Returns 0 or an error.
struct IovRunner {
  virtual int operator()(BatchDesc &d) const = 0;
};
// Per-record totals -> run; no staging, no stream synchronisation.
int iov_batch_run(const IovBatchDesc &b, const IovRunner &run, void *stream);
int launch_synth(uint64_t first, size_t n, const uint64_t *offsets,
                 const uint64_t *lengths, uint8_t *pt, uint8_t *nonces,
                 uint8_t *ads, void *stream);

// Compute units of the current device, cached per device ordinal (launch
// grids of the persistent kernels; 0 on error).
inline int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  if (dev < 64) {
    const int v = cache[dev].load(std::memory_order_relaxed);
    if (v) return v;
  }
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// Wipes key material that goes out of scope (reference: OPENSSL_cleanse).
void secure_zero(void *p, size_t n);

// Key setup (key_setup.cc, key_sched.h): one key on the host, or n keys by
// the device kernel into device memory (synchronous on `s`; 0 or an error).
bool gcm_key_setup(const uint8_t *key, size_t key_len, GcmKeyDev *out);
int gcm_key_setup_device(const uint8_t *keys, size_t key_len, size_t n, GcmKeyDev *out,
                         hipStream_t s);
void chacha_key_setup(const uint8_t *key, ChaChaKeyDev *out);
// Key counts from which make_keys builds AES-GCM tables on the device.
constexpr size_t kDeviceKeySetupMin = 64;

}  // namespace bssl_amd

#endif
