// aead_api.cc -- the C ABI of include/bssl_amd/aead.h.
//
// Mirrors the reference's AEAD dispatch layer
// (crypto/fipsmodule/cipher/aead.cc.inc): argument and alias checks, the
// zero-on-error cleanup of every entry point, the per-AEAD vtable limits
// (e_aes.cc.inc:733-924, 1040-1230; e_chacha20poly1305.cc:45-400) and the
// CIPHER_R_* error queue.  All record arithmetic runs in the HIP kernels
// (gcm.hip, chacha.hip): single-record calls upload their host buffers, run a
// one-record batch and download the result.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "bssl_amd/aead.h"
#include "bssl_amd/tls.h"
#include "bssl_amd/test_hooks.h"
#include "internal.h"

using namespace bssl_amd;

// ---------------------------------------------------------------------------
// Error queue (reference crypto/err/err.cc semantics: thread-local,
// ERR_NUM_ERRORS = 16 deep, oldest dropped on overflow).
namespace {
constexpr int kNumErrors = 16;
thread_local uint32_t t_err[kNumErrors];
thread_local int t_err_top = 0, t_err_bottom = 0;

void put_error(int reason) {
  t_err_top = (t_err_top + 1) % kNumErrors;
  if (t_err_top == t_err_bottom) t_err_bottom = (t_err_bottom + 1) % kNumErrors;
  t_err[t_err_top] = ((uint32_t)(ERR_LIB_CIPHER & 0xff) << 24) | ((uint32_t)reason & 0xfff);
}
}  // namespace

#define PUT_ERROR(reason) put_error(reason)

extern "C" uint32_t ERR_get_error(void) {
  if (t_err_top == t_err_bottom) return 0;
  t_err_bottom = (t_err_bottom + 1) % kNumErrors;
  uint32_t e = t_err[t_err_bottom];
  t_err[t_err_bottom] = 0;
  return e;
}

extern "C" uint32_t ERR_peek_error(void) {
  if (t_err_top == t_err_bottom) return 0;
  return t_err[(t_err_bottom + 1) % kNumErrors];
}

extern "C" uint32_t ERR_peek_last_error(void) {
  if (t_err_top == t_err_bottom) return 0;
  return t_err[t_err_top];
}

extern "C" void ERR_clear_error(void) {
  t_err_top = t_err_bottom = 0;
  memset(t_err, 0, sizeof(t_err));
}

// ---------------------------------------------------------------------------
// AEAD method objects (the reference's struct evp_aead_st vtable,
// crypto/fipsmodule/cipher/internal.h:40-78, reduced to the parameters the
// GPU path needs).
struct evp_aead_st {
  uint8_t key_len;
  uint8_t nonce_len;
  uint8_t overhead;
  uint8_t max_tag_len;
  AeadKind kind;
  int tls;  // 0, 12 or 13: the tls12 / tls13 monotonic-nonce variants
};

namespace {
const evp_aead_st kAes128Gcm = {16, 12, 16, 16, kAeadAesGcm, 0};
const evp_aead_st kAes192Gcm = {24, 12, 16, 16, kAeadAesGcm, 0};
const evp_aead_st kAes256Gcm = {32, 12, 16, 16, kAeadAesGcm, 0};
const evp_aead_st kChaChaPoly = {32, 12, 16, 16, kAeadChaChaPoly, 0};
const evp_aead_st kXChaChaPoly = {32, 24, 16, 16, kAeadXChaChaPoly, 0};  // e_chacha20poly1305.cc:385-399
const evp_aead_st kAes128GcmSiv = {16, 12, 16, 16, kAeadAesGcmSiv, 0};  // e_aesgcmsiv.cc:869-899
const evp_aead_st kAes256GcmSiv = {32, 12, 16, 16, kAeadAesGcmSiv, 0};
const evp_aead_st kAes128GcmTls12 = {16, 12, 16, 16, kAeadAesGcm, 12};
const evp_aead_st kAes256GcmTls12 = {32, 12, 16, 16, kAeadAesGcm, 12};
const evp_aead_st kAes128GcmTls13 = {16, 12, 16, 16, kAeadAesGcm, 13};
const evp_aead_st kAes256GcmTls13 = {32, 12, 16, 16, kAeadAesGcm, 13};

// Device-resident key material for one or more keys.
struct KeyMaterial {
  const EVP_AEAD *aead;
  int device;  // the HIP device the key material lives on
  size_t num_keys;
  int nr;
  void *dev;  // GcmKeyDev[num_keys] or ChaChaKeyDev[num_keys]
  size_t bytes;
};

// Makes `dev` the calling thread's current HIP device for the guard's scope
// and restores the previous one (host-buffer calls may come from any thread,
// as the reference's EVP_AEAD_CTX allows, aead.h:298-299).
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) return;
    ok = prev == dev || hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (ok) hipSetDevice(prev);
  }
};

// Device-batch calls take device pointers and a stream of the caller's
// current device; they must be made on the device that holds the keys.
bool on_key_device(const KeyMaterial *km) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != km->device) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return false;
  }
  return true;
}

// State kept in EVP_AEAD_CTX.state (560 bytes, reference aead.h:222-235).
struct CtxState {
  KeyMaterial *km;
  uint64_t min_next_nonce;  // tls12/tls13 (e_aes.cc.inc:1041-1044, 1130-1134)
  uint64_t mask;
};
static_assert(sizeof(CtxState) <= sizeof(((EVP_AEAD_CTX *)nullptr)->state), "state");

CtxState *state_of(const EVP_AEAD_CTX *ctx) {
  return reinterpret_cast<CtxState *>(const_cast<uint8_t *>(ctx->state.opaque));
}

// Key material of num_keys keys on the current device.  AES-GCM(-SIV) key
// sets of kDeviceKeySetupMin keys or more are expanded by the device kernel
// straight into device memory (gcm_key_setup_device); smaller ones -- the
// single key of EVP_AEAD_CTX_init -- on the host and copied (a kernel launch
// and synchronisation cost more than the host's few microseconds per key).
// device_setup: -1 by that rule, 0 host, 1 device (BSSL_AMD_gcm_key_tables).
KeyMaterial *make_keys(const EVP_AEAD *aead, const uint8_t *keys, size_t num_keys,
                       int device_setup = -1) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  KeyMaterial *km = new (std::nothrow) KeyMaterial{aead, dev, num_keys, 0, nullptr, 0};
  if (!km) return nullptr;
  const bool gcm = aead->kind == kAeadAesGcm || aead->kind == kAeadAesGcmSiv;
  if (gcm && num_keys && (device_setup == 1 || (device_setup < 0 && num_keys >= kDeviceKeySetupMin))) {
    const size_t bytes = num_keys * sizeof(GcmKeyDev);
    if (hipMalloc(&km->dev, bytes) != hipSuccess) {
      delete km;
      return nullptr;
    }
    km->bytes = bytes;
    if (gcm_key_setup_device(keys, aead->key_len, num_keys, reinterpret_cast<GcmKeyDev *>(km->dev),
                             nullptr) != 0) {
      // The kernel may have written tables before the failure: wipe them as
      // free_keys does before the memory goes back.
      hipMemset(km->dev, 0, bytes);
      hipDeviceSynchronize();
      hipFree(km->dev);
      delete km;
      return nullptr;
    }
    km->nr = (int)aead->key_len / 4 + 6;
    return km;
  }
  size_t bytes;
  std::vector<uint8_t> host;
  struct Wipe {  // the expanded keys in host memory are wiped on every path
    std::vector<uint8_t> &v;
    ~Wipe() { secure_zero(v.data(), v.size()); }
  } wipe{host};
  if (aead->kind == kAeadAesGcm || aead->kind == kAeadAesGcmSiv) {
    bytes = num_keys * sizeof(GcmKeyDev);
    host.resize(bytes);
    GcmKeyDev *h = reinterpret_cast<GcmKeyDev *>(host.data());
    for (size_t i = 0; i < num_keys; i++) {
      if (!gcm_key_setup(keys + i * aead->key_len, aead->key_len, &h[i])) {
        delete km;
        return nullptr;
      }
    }
    km->nr = (int)h[0].nr;
  } else {
    bytes = num_keys * sizeof(ChaChaKeyDev);
    host.resize(bytes);
    ChaChaKeyDev *h = reinterpret_cast<ChaChaKeyDev *>(host.data());
    for (size_t i = 0; i < num_keys; i++) chacha_key_setup(keys + i * aead->key_len, &h[i]);
  }
  if (hipMalloc(&km->dev, bytes) != hipSuccess) {
    delete km;
    return nullptr;
  }
  km->bytes = bytes;
  if (hipMemcpy(km->dev, host.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(km->dev);
    delete km;
    return nullptr;
  }
  return km;
}

void free_keys(KeyMaterial *km) {
  if (!km) return;
  if (km->dev) {
    DeviceGuard g(km->device);
    // Batches may still be reading the keys on any stream of the device,
    // including non-blocking ones the null-stream memset does not order
    // against (seal/open_batch_device are asynchronous to the host): drain the
    // device first, then wipe the device copy (OPENSSL_cleanse) and free it.
    hipDeviceSynchronize();
    hipMemset(km->dev, 0, km->bytes);
    hipDeviceSynchronize();
    hipFree(km->dev);
  }
  delete km;
}

// Kernel timing: when enabled, every batch launch records a pair of HIP
// events around its bulk kernel (no host synchronisation);
// BSSL_AMD_collect_kernel_times() waits for them and reports the durations.
struct TimingState {
  bool enabled = false;
  std::vector<KernelEvents> free_pairs, pending;
  double last_ms = 0;
  const char *last_name = "";
  ~TimingState() {
    for (auto &e : free_pairs) {
      hipEventDestroy(reinterpret_cast<hipEvent_t>(e.start));
      hipEventDestroy(reinterpret_cast<hipEvent_t>(e.stop));
    }
  }
};
thread_local TimingState t_timing;

const KernelEvents *timing_pair() {
  if (!t_timing.enabled) return nullptr;
  KernelEvents e;
  if (!t_timing.free_pairs.empty()) {
    e = t_timing.free_pairs.back();
    t_timing.free_pairs.pop_back();
  } else {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return nullptr;
    if (hipEventCreate(&b) != hipSuccess) {
      hipEventDestroy(a);
      return nullptr;
    }
    e = KernelEvents{a, b};
  }
  t_timing.pending.push_back(e);
  return &t_timing.pending.back();
}

// Name of the dominant kernel of an AES-GCM launch on `engine` (the timing
// records and bench.py's profile lookup key on it).
const char *gcm_kernel_name(int engine) {
  return engine == kGcmEngineBitsliced ? "gcm_bs_kernel"
         : engine == kGcmEngineMix        ? "gcm_mix_kernel"
                                          : "gcm_kernel";
}

// Launch the bulk kernels of the AEAD over a filled-in descriptor.  Returns 0
// or a HIP error code.  `gcm_eng`: the AES-GCM engine the caller already read
// for this batch (-1: read it here), so one batch never sees two engines.
int launch_desc(const KeyMaterial *km, const BatchDesc &d, bool open, void *stream,
                int gcm_eng = -1) {
  int rc;
  const KernelEvents *ev = timing_pair();
  if (km->aead->kind == kAeadAesGcm) {
    const int eng = gcm_eng >= 0 ? gcm_eng : gcm_engine();
    rc = launch_gcm(static_cast<const GcmKeyDev *>(km->dev), d, open, km->nr, stream, ev, eng);
    t_timing.last_name = gcm_kernel_name(eng);
  } else if (km->aead->kind == kAeadAesGcmSiv) {
    rc = launch_gcm_siv(static_cast<const GcmKeyDev *>(km->dev), d, open, km->nr, stream, ev);
    t_timing.last_name = "gcm_siv_kernel";
  } else {
    rc = launch_chacha(static_cast<const ChaChaKeyDev *>(km->dev), d, open,
                       km->aead->kind == kAeadXChaChaPoly, stream, ev);
    t_timing.last_name = "chacha_poly_kernel";
  }
  return rc;
}

// Launch a batch over device buffers.  Returns 1 on success.
// `one`: the single-record extras of one_record (completion word, inline
// nonce / AD; BatchDesc::done, ::inl), or null.
int run_batch(const KeyMaterial *km, size_t tag_len, const BSSL_AMD_BATCH *batch, bool open,
              bool use_key_index, void *stream, const uint8_t *valid = nullptr,
              const BatchDesc *one = nullptr, bool *done_armed = nullptr) {
  BatchDesc d;
  memset(&d, 0, sizeof(d));
  d.in = batch->in;
  d.out = batch->out;
  d.offsets = batch->offsets;
  d.lengths = batch->lengths;
  d.record_stride = batch->record_stride;
  d.record_len = batch->record_len;
  d.nonces = batch->nonces;
  d.nonce_len = batch->nonce_len;
  d.ad = batch->ad;
  d.ad_offsets = batch->ad_offsets;
  d.ad_lengths = batch->ad_lengths;
  d.ad_stride = batch->ad_stride;
  d.ad_len = batch->ad_len;
  d.tags = batch->tags;
  d.status = batch->status;
  d.key_index = use_key_index ? batch->key_index : nullptr;
  d.num_records = batch->num_records;
  d.tag_len = (uint32_t)tag_len;
  d.num_keys = (uint32_t)km->num_keys;
  d.order = nullptr;
  d.valid = valid;
  d.extra = nullptr;
  d.extra_out = nullptr;
  d.extra_len = d.extra_stride = d.extra_out_stride = d.tag_stride = 0;
  // The AES-GCM engine is read once per batch: the completion-word decision
  // below and the launch must agree on it.
  const int gcm_eng = km->aead->kind == kAeadAesGcm ? gcm_engine() : -1;
  if (one) {
    // The completion word only when a one-record kernel will write it
    // (*done_armed tells one_record whether to spin on it).
    const AeadKind k = km->aead->kind;
    const bool writes = k == kAeadAesGcm ? gcm_takes_one_record_kernel(d, gcm_eng)
                        : k == kAeadAesGcmSiv ? false
                                              : chacha_takes_one_record_kernel(d);
    d.done = writes ? one->done : nullptr;
    if (done_armed) *done_armed = d.done != nullptr;
    d.done_seq = one->done_seq;
    d.inl = one->inl;
    memcpy(d.inl_nonce, one->inl_nonce, sizeof(d.inl_nonce));
    memcpy(d.inl_ad, one->inl_ad, sizeof(d.inl_ad));
  }
  if (launch_desc(km, d, open, stream, gcm_eng) != 0) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  return 1;
}

bool check_batch(const EVP_AEAD *aead, const BSSL_AMD_BATCH *b) {
  if (!b) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return false;
  }
  if (b->num_records == 0) return true;
  if (!b->in || !b->out || !b->nonces || !b->tags || (!b->ad && (b->ad_lengths || b->ad_len))) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return false;
  }
  if (aead->kind == kAeadAesGcm) {
    if (b->nonce_len == 0) {  // e_aes.cc.inc:790-793
      PUT_ERROR(CIPHER_R_INVALID_NONCE_SIZE);
      return false;
    }
  } else if (b->nonce_len != aead->nonce_len) {  // e_chacha20poly1305.cc:127-130, 241-244
    PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
    return false;
  }
  return true;
}

// ---- single-record helper: host buffers -> one-record device batch --------

// Per-thread staging buffers and stream of the host-buffer calls, one set per
// device (a thread may use contexts of several GPUs): a pinned, mapped host
// buffer -- records up to one_record_map_max() are read and written by the
// kernel in place through its device address (`mapped`), with no DMA copy --
// and device memory for longer records, which take one H2D and one D2H copy
// through the pinned buffer (pageable copies cost ~10 us each).
struct Scratch {
  uint8_t *dev = nullptr;
  uint8_t *host = nullptr;
  uint8_t *mapped = nullptr;  // device address of `host`
  size_t cap = 0;
  hipStream_t stream = nullptr;
  int device = -1;  // the device that owns dev/stream (set on first use)
  ~Scratch() {
    if (device < 0) return;  // never used
    // Thread exit (or process teardown for the main thread): free on the
    // owning device.  If the HIP runtime is already shut down the calls fail
    // and the process is exiting anyway.
    DeviceGuard g(device);
    if (!g.ok) return;
    if (dev) hipFree(dev);
    if (host) hipHostFree(host);
    if (stream) hipStreamDestroy(stream);
  }
};
constexpr int kMaxDevices = 64;
thread_local Scratch t_scratch[kMaxDevices];

// Scratch of the current device (the caller holds a DeviceGuard).
Scratch *scratch(size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  Scratch &sc = t_scratch[dev];
  sc.device = dev;
  if (!sc.stream && hipStreamCreateWithFlags(&sc.stream, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  if (sc.cap < bytes) {
    if (sc.dev) hipFree(sc.dev);
    if (sc.host) hipHostFree(sc.host);
    sc.dev = sc.host = sc.mapped = nullptr;
    sc.cap = 0;
    size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
    if (hipMalloc(&sc.dev, cap) != hipSuccess) {
      sc.dev = nullptr;
      return nullptr;
    }
    // Mapped pinned memory, explicitly fine-grained (hipHostMallocCoherent:
    // with any flag but hipHostMallocDefault, HIP's coherence otherwise follows
    // HIP_HOST_COHERENT, 0 by default).  The host spins on the completion word
    // while the kernel runs, and the kernel re-reads lines the host rewrote in
    // place since the previous call; both need the coherent mapping.  The
    // kernels use its device address.  (Flag variants measured the same
    // single-record latency, profiles/r04/s10/.)
    if (hipHostMalloc(&sc.host, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      sc.host = nullptr;
      hipFree(sc.dev);
      sc.dev = nullptr;
      return nullptr;
    }
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&sc.mapped), sc.host, 0) !=
        hipSuccess) {
      hipHostFree(sc.host);
      hipFree(sc.dev);
      sc.host = sc.dev = nullptr;
      return nullptr;
    }
    sc.cap = cap;
  }
  return &sc;
}

size_t round16(size_t n) { return (n + 15) & ~size_t(15); }

// Largest record the single-record path seals in mapped host memory
// (BSSL_AMD_ONE_RECORD_MAP_MAX overrides; 0 = always copy).
size_t one_record_map_max() {
  static const size_t v = [] {
    const char *e = getenv("BSSL_AMD_ONE_RECORD_MAP_MAX");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)65536;
  }();
  return v;
}

// Waits for a single-record launch on stream s.  With `done` (mapped path and
// a one-record kernel launched: run_batch arms the word only then) the host
// spins on the completion word the kernel writes after its last store -- it
// lands a few microseconds before the stream's completion signal does -- and
// checks the stream every 256 polls, so a failed launch still ends.
// Otherwise (other kernels, records that took the copies) it blocks in
// hipStreamSynchronize.
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#elif defined(__aarch64__)
  asm volatile("yield");
#endif
}

bool wait_record(hipStream_t s, const uint32_t *done, uint32_t seq) {
  if (!done) return hipStreamSynchronize(s) == hipSuccess;
  for (uint32_t i = 1;; i++) {
    if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) return true;
    if ((i & 255) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) return true;
      if (e != hipErrorNotReady) return false;
    }
    cpu_relax();
  }
}

// Seal or open one record held in host memory.  `in`/`out` may be equal.
// For open, `tag` is read; for seal it is written (tag_len bytes).
// Staging layout (device and pinned host alike): nonce | AD | tag, status
// (32 B) | record -- one H2D copy of all of it, one D2H copy of tag, status
// and record.
int one_record(const EVP_AEAD_CTX *ctx, bool open, const uint8_t *in, uint8_t *out,
               size_t len, const uint8_t *nonce, size_t nonce_len, const uint8_t *ad,
               size_t ad_len, uint8_t *tag, size_t tag_len) {
  CtxState *st = state_of(ctx);
  DeviceGuard guard(st->km->device);
  if (!guard.ok) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  const size_t o_nonce = 0, o_ad = round16(nonce_len), o_tag = o_ad + round16(ad_len),
               o_status = o_tag + 16, o_in = o_status + 16, total = o_in + round16(len);
  Scratch *sc = scratch(total);
  if (!sc) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    return 0;
  }
  hipStream_t s = sc->stream;
  // Records up to kMapMax bytes are read and written by the kernels directly
  // in the pinned host buffer (mapped into the GPU's address space): no DMA
  // copies, whose two launches and completions were most of a short record's
  // latency.  Longer records take one H2D and one D2H copy.
  const bool mapped = len <= one_record_map_max();
  uint8_t *h = sc->host, *d = mapped ? sc->mapped : sc->dev;
  if (nonce_len) memcpy(h + o_nonce, nonce, nonce_len);
  if (ad_len) memcpy(h + o_ad, ad, ad_len);
  if (open && tag_len) memcpy(h + o_tag, tag, tag_len);
  if (len) memcpy(h + o_in, in, len);
  if (!mapped && hipMemcpyAsync(d, h, o_in + len, hipMemcpyHostToDevice, s) != hipSuccess) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  BSSL_AMD_BATCH b;
  memset(&b, 0, sizeof(b));
  b.num_records = 1;
  b.in = d + o_in;
  b.out = d + o_in;
  b.record_len = len;
  b.nonces = d + o_nonce;
  b.nonce_len = nonce_len;
  b.ad = d + o_ad;
  b.ad_len = ad_len;
  b.tags = d + o_tag;
  b.status = d + o_status;
  // Completion word (mapped path): the one-record kernels write `seq` there
  // last (BatchDesc::done).
  static thread_local uint32_t t_seq = 0;
  const uint32_t seq = ++t_seq ? t_seq : ++t_seq;  // (never 0)
  uint32_t *hdone = reinterpret_cast<uint32_t *>(h + o_status + 4);
  __atomic_store_n(hdone, 0u, __ATOMIC_RELAXED);
  BatchDesc one;
  memset(&one, 0, sizeof(one));
  one.done = mapped ? reinterpret_cast<uint32_t *>(d + o_status + 4) : nullptr;
  one.done_seq = seq;
  // The nonce and a short AD by value (BatchDesc::inl).
  if (nonce_len == 12) {
    memcpy(one.inl_nonce, nonce, 12);
    one.inl |= 1;
  }
  if (ad_len <= 16) {
    if (ad_len) memcpy(one.inl_ad, ad, ad_len);
    one.inl |= 2;
  }
  bool armed = false;
  if (!run_batch(st->km, tag_len, &b, open, false, s, nullptr, &one, &armed)) return 0;
  bool ok = mapped || hipMemcpyAsync(h + o_tag, d + o_tag, o_in - o_tag + len,
                                     hipMemcpyDeviceToHost, s) == hipSuccess;
  ok = ok && wait_record(s, armed ? hdone : nullptr, seq);
  if (!ok) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  if (len) memcpy(out, h + o_in, len);
  if (!open && tag_len) memcpy(tag, h + o_tag, tag_len);
  if (!h[o_status]) {
    PUT_ERROR(open ? CIPHER_R_BAD_DECRYPT : CIPHER_R_TOO_LARGE);
    return 0;
  }
  return 1;
}

int buffers_alias(const void *a, size_t a_len, const void *b, size_t b_len) {
  // crypto/internal.h:187-196
  uintptr_t au = (uintptr_t)a, bu = (uintptr_t)b;
  return au + a_len > bu && bu + b_len > au;
}

bool check_alias(const uint8_t *in, size_t in_len, const uint8_t *out, size_t out_len) {
  if (!buffers_alias(in, in_len, out, out_len)) return true;
  return in == out;
}

// iovec helpers (crypto/fipsmodule/cipher/internal.h:162-236).
bool iovec_total(const CRYPTO_IOVEC *v, size_t n, size_t *total) {
  size_t t = 0;
  for (size_t i = 0; i < n; i++) {
    if (t + v[i].len < t) return false;
    t += v[i].len;
  }
  *total = t;
  return true;
}

bool ivec_total(const CRYPTO_IVEC *v, size_t n, size_t *total) {
  size_t t = 0;
  for (size_t i = 0; i < n; i++) {
    if (t + v[i].len < t) return false;
    t += v[i].len;
  }
  *total = t;
  return true;
}

void clear_iovec(const CRYPTO_IOVEC *v, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (v[i].len) memset(v[i].out, 0, v[i].len);
}

bool iovec_internal_alias_ok(const CRYPTO_IOVEC *v, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (!check_alias(v[i].in, v[i].len, v[i].out, v[i].len)) return false;
  return true;
}

// Gather iovec inputs into one contiguous host buffer.
std::vector<uint8_t> gather_in(const CRYPTO_IOVEC *v, size_t n, size_t total) {
  std::vector<uint8_t> buf(total);
  size_t o = 0;
  for (size_t i = 0; i < n; i++) {
    if (v[i].len) memcpy(buf.data() + o, v[i].in, v[i].len);
    o += v[i].len;
  }
  return buf;
}

void scatter_out(const CRYPTO_IOVEC *v, size_t n, const uint8_t *src, size_t total) {
  size_t o = 0;
  for (size_t i = 0; i < n && o < total; i++) {
    size_t take = v[i].len < total - o ? v[i].len : total - o;
    if (take) memcpy(v[i].out, src + o, take);
    o += v[i].len;
  }
}

std::vector<uint8_t> gather_ad(const CRYPTO_IVEC *v, size_t n, size_t total) {
  std::vector<uint8_t> buf(total);
  size_t o = 0;
  for (size_t i = 0; i < n; i++) {
    if (v[i].len) memcpy(buf.data() + o, v[i].in, v[i].len);
    o += v[i].len;
  }
  return buf;
}

uint64_t load_be64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
  return v;
}

// The stateful TLS nonce checks of aead_aes_gcm_tls12_sealv /
// aead_aes_gcm_tls13_sealv (e_aes.cc.inc:1071-1100, 1162-1202).
bool tls_nonce_check(const EVP_AEAD_CTX *ctx, const uint8_t *nonce, size_t nonce_len) {
  const EVP_AEAD *aead = ctx->aead;
  if (!aead->tls) return true;
  CtxState *st = state_of(ctx);
  if (nonce_len != 12) {
    PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
    return false;
  }
  uint64_t given = load_be64(nonce + 4);
  if (aead->tls == 12) {
    if (given == UINT64_MAX || given < st->min_next_nonce) {
      PUT_ERROR(CIPHER_R_INVALID_NONCE);
      return false;
    }
    st->min_next_nonce = given + 1;
    return true;
  }
  if (st->min_next_nonce == 0) {
    st->mask = given;
    st->min_next_nonce = 1;
    return true;
  }
  given ^= st->mask;
  if (given == UINT64_MAX || given < st->min_next_nonce) {
    PUT_ERROR(CIPHER_R_INVALID_NONCE);
    return false;
  }
  st->min_next_nonce = given + 1;
  return true;
}

// Common per-AEAD record checks before any device work (sealv/openv paths).
bool aead_record_checks(const EVP_AEAD_CTX *ctx, size_t nonce_len, size_t in_len) {
  const EVP_AEAD *aead = ctx->aead;
  if (aead->kind == kAeadAesGcm) {
    if (nonce_len == 0) {
      PUT_ERROR(CIPHER_R_INVALID_NONCE_SIZE);
      return false;
    }
  } else if (aead->kind == kAeadAesGcmSiv) {
    if (nonce_len != 12) {  // e_aesgcmsiv.cc:805-808, 843-846
      PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
      return false;
    }
    if ((uint64_t)in_len > (UINT64_C(1) << 36)) {  // :794-798
      PUT_ERROR(CIPHER_R_TOO_LARGE);
      return false;
    }
  } else {
    if (nonce_len != aead->nonce_len) {  // 12, or 24 for XChaCha (e_chacha20poly1305.cc:241)
      PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
      return false;
    }
    if ((uint64_t)in_len >= (UINT64_C(1) << 32) * 64 - 64) {
      PUT_ERROR(CIPHER_R_TOO_LARGE);
      return false;
    }
  }
  return true;
}

// The per-AEAD tag-length rule of init (e_aes.cc.inc:742-749,
// e_chacha20poly1305.cc:51-57, e_aesgcmsiv.cc:542-548): 0 means the maximum.
bool resolve_tag_len(const EVP_AEAD *aead, size_t *tag_len) {
  if (*tag_len == EVP_AEAD_DEFAULT_TAG_LENGTH) *tag_len = aead->max_tag_len;
  if (*tag_len > aead->max_tag_len || (aead->kind == kAeadAesGcmSiv && *tag_len != 16)) {
    PUT_ERROR(aead->kind == kAeadAesGcm || aead->kind == kAeadAesGcmSiv ? CIPHER_R_TAG_TOO_LARGE
                                                                       : CIPHER_R_TOO_LARGE);
    return false;
  }
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// Method getters and sizes.
extern "C" {

const EVP_AEAD *EVP_aead_aes_128_gcm(void) { return &kAes128Gcm; }
const EVP_AEAD *EVP_aead_aes_192_gcm(void) { return &kAes192Gcm; }
const EVP_AEAD *EVP_aead_aes_256_gcm(void) { return &kAes256Gcm; }
const EVP_AEAD *EVP_aead_chacha20_poly1305(void) { return &kChaChaPoly; }
const EVP_AEAD *EVP_aead_xchacha20_poly1305(void) { return &kXChaChaPoly; }
const EVP_AEAD *EVP_aead_aes_128_gcm_siv(void) { return &kAes128GcmSiv; }
const EVP_AEAD *EVP_aead_aes_256_gcm_siv(void) { return &kAes256GcmSiv; }
const EVP_AEAD *EVP_aead_aes_128_gcm_tls12(void) { return &kAes128GcmTls12; }
const EVP_AEAD *EVP_aead_aes_256_gcm_tls12(void) { return &kAes256GcmTls12; }
const EVP_AEAD *EVP_aead_aes_128_gcm_tls13(void) { return &kAes128GcmTls13; }
const EVP_AEAD *EVP_aead_aes_256_gcm_tls13(void) { return &kAes256GcmTls13; }

size_t EVP_AEAD_key_length(const EVP_AEAD *aead) { return aead->key_len; }
size_t EVP_AEAD_nonce_length(const EVP_AEAD *aead) { return aead->nonce_len; }
size_t EVP_AEAD_max_overhead(const EVP_AEAD *aead) { return aead->overhead; }
size_t EVP_AEAD_max_tag_len(const EVP_AEAD *aead) { return aead->max_tag_len; }

void EVP_AEAD_CTX_zero(EVP_AEAD_CTX *ctx) { memset(ctx, 0, sizeof(*ctx)); }

EVP_AEAD_CTX *EVP_AEAD_CTX_new(const EVP_AEAD *aead, const uint8_t *key, size_t key_len,
                               size_t tag_len) {
  EVP_AEAD_CTX *ctx = static_cast<EVP_AEAD_CTX *>(calloc(1, sizeof(EVP_AEAD_CTX)));
  if (!ctx) return nullptr;
  if (!EVP_AEAD_CTX_init(ctx, aead, key, key_len, tag_len, nullptr)) {
    free(ctx);
    return nullptr;
  }
  return ctx;
}

void EVP_AEAD_CTX_free(EVP_AEAD_CTX *ctx) {
  if (!ctx) return;
  EVP_AEAD_CTX_cleanup(ctx);
  free(ctx);
}

int EVP_AEAD_CTX_init(EVP_AEAD_CTX *ctx, const EVP_AEAD *aead, const uint8_t *key,
                      size_t key_len, size_t tag_len, ENGINE *impl) {
  (void)impl;
  return EVP_AEAD_CTX_init_with_direction(ctx, aead, key, key_len, tag_len, evp_aead_open);
}

int EVP_AEAD_CTX_init_with_direction(EVP_AEAD_CTX *ctx, const EVP_AEAD *aead,
                                     const uint8_t *key, size_t key_len, size_t tag_len,
                                     enum evp_aead_direction_t dir) {
  (void)dir;
  // aead.cc.inc:82-106
  if (key_len != aead->key_len) {
    PUT_ERROR(CIPHER_R_UNSUPPORTED_KEY_SIZE);
    ctx->aead = nullptr;
    return 0;
  }
  if (!resolve_tag_len(aead, &tag_len)) {
    ctx->aead = nullptr;
    return 0;
  }
  KeyMaterial *km = make_keys(aead, key, 1);
  if (!km) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    ctx->aead = nullptr;
    return 0;
  }
  memset(&ctx->state, 0, sizeof(ctx->state));
  CtxState *st = state_of(ctx);
  st->km = km;
  ctx->aead = aead;
  ctx->tag_len = (uint8_t)tag_len;
  return 1;
}

void EVP_AEAD_CTX_cleanup(EVP_AEAD_CTX *ctx) {
  if (ctx->aead == nullptr) return;
  free_keys(state_of(ctx)->km);
  state_of(ctx)->km = nullptr;
  ctx->aead = nullptr;
}

const EVP_AEAD *EVP_AEAD_CTX_aead(const EVP_AEAD_CTX *ctx) { return ctx->aead; }

// aead.cc.inc:316-361
int EVP_AEAD_CTX_sealv(const EVP_AEAD_CTX *ctx, const CRYPTO_IOVEC *iovec, size_t num_iovec,
                       uint8_t *out_tag, size_t *out_tag_len, size_t max_out_tag_len,
                       const uint8_t *nonce, size_t nonce_len, const CRYPTO_IVEC *aadvec,
                       size_t num_aadvec) {
  bool ok = false;
  size_t total = 0, ad_total = 0;
  struct Cleanup {
    bool &ok;
    const CRYPTO_IOVEC *v;
    size_t n;
    uint8_t *tag;
    size_t tag_max;
    size_t *tag_len;
    ~Cleanup() {
      if (!ok) {
        clear_iovec(v, n);
        if (tag_max) memset(tag, 0, tag_max);
        *tag_len = 0;
      }
    }
  } cleanup{ok, iovec, num_iovec, out_tag, max_out_tag_len, out_tag_len};

  if (!iovec_total(iovec, num_iovec, &total) || !ivec_total(aadvec, num_aadvec, &ad_total)) {
    PUT_ERROR(CIPHER_R_TOO_LARGE);
    return 0;
  }
  if (!iovec_internal_alias_ok(iovec, num_iovec)) {
    PUT_ERROR(CIPHER_R_OUTPUT_ALIASES_INPUT);
    return 0;
  }
  for (size_t i = 0; i < num_iovec; i++)
    if (buffers_alias(iovec[i].out, iovec[i].len, out_tag, max_out_tag_len)) {
      PUT_ERROR(CIPHER_R_OUTPUT_ALIASES_INPUT);
      return 0;
    }
  if (max_out_tag_len < ctx->tag_len) {  // e_aes.cc.inc:785-788
    PUT_ERROR(CIPHER_R_BUFFER_TOO_SMALL);
    return 0;
  }
  if (ctx->aead->tls) {
    if (!tls_nonce_check(ctx, nonce, nonce_len)) return 0;
  } else if (!aead_record_checks(ctx, nonce_len, total)) {
    return 0;
  }
  std::vector<uint8_t> in = gather_in(iovec, num_iovec, total);
  std::vector<uint8_t> ad = gather_ad(aadvec, num_aadvec, ad_total);
  uint8_t tag[16];
  if (!one_record(ctx, false, in.data(), in.data(), total, nonce, nonce_len, ad.data(),
                  ad_total, tag, ctx->tag_len))
    return 0;
  scatter_out(iovec, num_iovec, in.data(), total);
  memcpy(out_tag, tag, ctx->tag_len);
  *out_tag_len = ctx->tag_len;
  ok = true;
  return 1;
}

// aead.cc.inc:531-584
int EVP_AEAD_CTX_openv_detached(const EVP_AEAD_CTX *ctx, const CRYPTO_IOVEC *iovec,
                                size_t num_iovec, const uint8_t *nonce, size_t nonce_len,
                                const uint8_t *in_tag, size_t in_tag_len,
                                const CRYPTO_IVEC *aadvec, size_t num_aadvec) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    const CRYPTO_IOVEC *v;
    size_t n;
    ~Cleanup() {
      if (!ok) clear_iovec(v, n);
    }
  } cleanup{ok, iovec, num_iovec};
  size_t total = 0, ad_total = 0;
  if (!iovec_total(iovec, num_iovec, &total) || !ivec_total(aadvec, num_aadvec, &ad_total)) {
    PUT_ERROR(CIPHER_R_TOO_LARGE);
    return 0;
  }
  if (in_tag_len > EVP_AEAD_MAX_OPEN_OVERHEAD) {
    PUT_ERROR(CIPHER_R_UNSUPPORTED_TAG_SIZE);
    return 0;
  }
  if (!iovec_internal_alias_ok(iovec, num_iovec)) {
    PUT_ERROR(CIPHER_R_OUTPUT_ALIASES_INPUT);
    return 0;
  }
  if (ctx->aead->kind == kAeadAesGcm) {
    if (nonce_len == 0) {
      PUT_ERROR(CIPHER_R_INVALID_NONCE_SIZE);
      return 0;
    }
    if (ctx->aead->tls && nonce_len != 12) {
      // The tls variants share aead_aes_gcm_openv_detached, which accepts any
      // non-empty nonce (e_aes.cc.inc:869-882).
    }
  } else if (!aead_record_checks(ctx, nonce_len, total)) {
    return 0;
  }
  if (in_tag_len != ctx->tag_len) {  // e_aes.cc.inc:838-841
    PUT_ERROR(CIPHER_R_BAD_DECRYPT);
    return 0;
  }
  std::vector<uint8_t> in = gather_in(iovec, num_iovec, total);
  std::vector<uint8_t> ad = gather_ad(aadvec, num_aadvec, ad_total);
  uint8_t tag[16];
  memcpy(tag, in_tag, in_tag_len);
  if (!one_record(ctx, true, in.data(), in.data(), total, nonce, nonce_len, ad.data(),
                  ad_total, tag, in_tag_len))
    return 0;
  scatter_out(iovec, num_iovec, in.data(), total);
  ok = true;
  return 1;
}

// aead.cc.inc:460-529 (the openv_detached fallback with the tag as a suffix).
int EVP_AEAD_CTX_openv(const EVP_AEAD_CTX *ctx, const CRYPTO_IOVEC *iovec, size_t num_iovec,
                       size_t *out_total_bytes, const uint8_t *nonce, size_t nonce_len,
                       const CRYPTO_IVEC *aadvec, size_t num_aadvec) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    const CRYPTO_IOVEC *v;
    size_t n;
    size_t *out;
    ~Cleanup() {
      if (!ok) {
        clear_iovec(v, n);
        *out = 0;
      }
    }
  } cleanup{ok, iovec, num_iovec, out_total_bytes};
  size_t total = 0, ad_total = 0;
  if (!iovec_total(iovec, num_iovec, &total) || !ivec_total(aadvec, num_aadvec, &ad_total)) {
    PUT_ERROR(CIPHER_R_TOO_LARGE);
    return 0;
  }
  if (!iovec_internal_alias_ok(iovec, num_iovec)) {
    PUT_ERROR(CIPHER_R_OUTPUT_ALIASES_INPUT);
    return 0;
  }
  if (total < ctx->tag_len) {
    PUT_ERROR(CIPHER_R_BAD_DECRYPT);
    return 0;
  }
  std::vector<uint8_t> in = gather_in(iovec, num_iovec, total);
  const size_t pt_len = total - ctx->tag_len;
  // Split the iovecs at pt_len: the plaintext goes to the prefix of the
  // output space (aead.cc.inc:488-512).
  std::vector<CRYPTO_IOVEC> det;
  size_t o = 0;
  for (size_t i = 0; i < num_iovec && o < pt_len; i++) {
    CRYPTO_IOVEC v = iovec[i];
    if (v.len > pt_len - o) v.len = pt_len - o;
    det.push_back(v);
    o += v.len;
  }
  // Build detached iovecs that read from the gathered copy (the tag bytes may
  // sit in an iovec that is also written).
  std::vector<CRYPTO_IOVEC> det2 = det;
  o = 0;
  for (auto &v : det2) {
    v.in = in.data() + o;
    o += v.len;
  }
  if (!EVP_AEAD_CTX_openv_detached(ctx, det2.data(), det2.size(), nonce, nonce_len,
                                   in.data() + pt_len, ctx->tag_len, aadvec, num_aadvec))
    return 0;
  *out_total_bytes = pt_len;
  ok = true;
  return 1;
}

// aead.cc.inc:127-161
int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX *ctx, uint8_t *out, size_t *out_len,
                      size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
                      const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    uint8_t *out;
    size_t max;
    size_t *len;
    ~Cleanup() {
      if (!ok) {
        if (max) memset(out, 0, max);
        *len = 0;
      }
    }
  } cleanup{ok, out, max_out_len, out_len};
  if (max_out_len < in_len) {
    PUT_ERROR(CIPHER_R_BUFFER_TOO_SMALL);
    return 0;
  }
  CRYPTO_IOVEC iov = {out, in, in_len};
  CRYPTO_IVEC aiv = {ad, ad_len};
  if (!EVP_AEAD_CTX_sealv(ctx, &iov, 1, out + in_len, out_len, max_out_len - in_len, nonce,
                          nonce_len, &aiv, 1)) {
    *out_len = 0;
    return 0;
  }
  *out_len += in_len;
  ok = true;
  return 1;
}

// aead.cc.inc:163-209
int EVP_AEAD_CTX_seal_scatter(const EVP_AEAD_CTX *ctx, uint8_t *out, uint8_t *out_tag,
                              size_t *out_tag_len, size_t max_out_tag_len,
                              const uint8_t *nonce, size_t nonce_len, const uint8_t *in,
                              size_t in_len, const uint8_t *extra_in, size_t extra_in_len,
                              const uint8_t *ad, size_t ad_len) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    uint8_t *out;
    size_t in_len;
    uint8_t *tag;
    size_t tag_max;
    size_t *tag_len;
    ~Cleanup() {
      if (!ok) {
        if (in_len) memset(out, 0, in_len);
        if (tag_max) memset(tag, 0, tag_max);
        *tag_len = 0;
      }
    }
  } cleanup{ok, out, in_len, out_tag, max_out_tag_len, out_tag_len};
  if (max_out_tag_len < extra_in_len) {
    PUT_ERROR(CIPHER_R_BUFFER_TOO_SMALL);
    return 0;
  }
  CRYPTO_IOVEC iov[2] = {{out, in, in_len}, {out_tag, extra_in, extra_in_len}};
  CRYPTO_IVEC aiv = {ad, ad_len};
  if (!EVP_AEAD_CTX_sealv(ctx, iov, extra_in_len ? 2 : 1, out_tag + extra_in_len, out_tag_len,
                          max_out_tag_len - extra_in_len, nonce, nonce_len, &aiv, 1)) {
    *out_tag_len = 0;
    return 0;
  }
  *out_tag_len += extra_in_len;
  ok = true;
  return 1;
}

// aead.cc.inc:363-428
int EVP_AEAD_CTX_open(const EVP_AEAD_CTX *ctx, uint8_t *out, size_t *out_len,
                      size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
                      const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    uint8_t *out;
    size_t max;
    size_t *len;
    ~Cleanup() {
      if (!ok) {
        if (max) memset(out, 0, max);
        *len = 0;
      }
    }
  } cleanup{ok, out, max_out_len, out_len};
  if (in_len < ctx->tag_len) {
    PUT_ERROR(CIPHER_R_BAD_DECRYPT);
    return 0;
  }
  size_t pt_len = in_len - ctx->tag_len;
  if (max_out_len < pt_len) {
    PUT_ERROR(CIPHER_R_BUFFER_TOO_SMALL);
    return 0;
  }
  CRYPTO_IOVEC iov = {out, in, pt_len};
  CRYPTO_IVEC aiv = {ad, ad_len};
  if (!EVP_AEAD_CTX_openv_detached(ctx, &iov, 1, nonce, nonce_len, in + pt_len, ctx->tag_len,
                                   &aiv, 1))
    return 0;
  *out_len = pt_len;
  ok = true;
  return 1;
}

// aead.cc.inc:430-458
int EVP_AEAD_CTX_open_gather(const EVP_AEAD_CTX *ctx, uint8_t *out, const uint8_t *nonce,
                             size_t nonce_len, const uint8_t *in, size_t in_len,
                             const uint8_t *in_tag, size_t in_tag_len, const uint8_t *ad,
                             size_t ad_len) {
  bool ok = false;
  struct Cleanup {
    bool &ok;
    uint8_t *out;
    size_t len;
    ~Cleanup() {
      if (!ok && len) memset(out, 0, len);
    }
  } cleanup{ok, out, in_len};
  CRYPTO_IOVEC iov = {out, in, in_len};
  CRYPTO_IVEC aiv = {ad, ad_len};
  if (!EVP_AEAD_CTX_openv_detached(ctx, &iov, 1, nonce, nonce_len, in_tag, in_tag_len, &aiv,
                                   1))
    return 0;
  ok = true;
  return 1;
}

// aead.cc.inc:598-619
int EVP_AEAD_CTX_tag_len(const EVP_AEAD_CTX *ctx, size_t *out_tag_len, size_t in_len,
                         size_t extra_in_len) {
  (void)in_len;
  size_t tag_len = ctx->tag_len;
  if (extra_in_len + tag_len < extra_in_len) {
    PUT_ERROR(ERR_R_OVERFLOW);
    *out_tag_len = 0;
    return 0;
  }
  *out_tag_len = extra_in_len + tag_len;
  return 1;
}

// aead.cc.inc:586-596: none of the AEADs here implement get_iv.
int EVP_AEAD_CTX_get_iv(const EVP_AEAD_CTX *ctx, const uint8_t **out_iv, size_t *out_len) {
  (void)ctx;
  (void)out_iv;
  (void)out_len;
  PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
  return 0;
}

// ---- batch extension --------------------------------------------------------

int EVP_AEAD_CTX_seal_batch_device(const EVP_AEAD_CTX *ctx, const BSSL_AMD_BATCH *batch,
                                   void *hip_stream) {
  if (!ctx || !ctx->aead || !check_batch(ctx->aead, batch)) return 0;
  if (batch->num_records == 0) return 1;
  CtxState *st = state_of(ctx);
  if (!on_key_device(st->km)) return 0;
  if (!ctx->aead->tls)
    return run_batch(st->km, ctx->tag_len, batch, false, false, hip_stream);
  if (batch->nonce_len != 12) {  // e_aes.cc.inc:1077-1080, 1168-1171 (seal only)
    PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
    return 0;
  }
  // tls12/tls13: the records are N sealv calls in order, each with the
  // monotonic-nonce check (tls_scan.hip); records that fail it fail like the
  // reference call (zeroed output, status 0) and leave the state unchanged.
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  uint8_t *valid = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&valid), batch->num_records, s) != hipSuccess) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    return 0;
  }
  int ok = tls_nonce_scan(batch->nonces, batch->num_records, ctx->aead->tls,
                          &st->min_next_nonce, &st->mask, valid, 0, hip_stream) == 0;
  if (!ok) PUT_ERROR(ERR_R_INTERNAL_ERROR);
  if (ok) ok = run_batch(st->km, ctx->tag_len, batch, false, false, hip_stream, valid);
  hipFreeAsync(valid, s);
  return ok;
}

int EVP_AEAD_CTX_open_batch_device(const EVP_AEAD_CTX *ctx, const BSSL_AMD_BATCH *batch,
                                   void *hip_stream) {
  if (!ctx || !ctx->aead || !check_batch(ctx->aead, batch)) return 0;
  if (batch->num_records == 0) return 1;
  if (!on_key_device(state_of(ctx)->km)) return 0;
  return run_batch(state_of(ctx)->km, ctx->tag_len, batch, true, false, hip_stream);
}

namespace {

// The bulk kernels of `km` over an iovec batch (they walk the chunks in place).
struct KeyRunner : IovRunner {
  const KeyMaterial *km;
  size_t tag_len;
  bool open;
  void *stream;
  const uint8_t *valid;
  KeyRunner(const KeyMaterial *k, size_t t, bool o, void *s, const uint8_t *v)
      : km(k), tag_len(t), open(o), stream(s), valid(v) {}
  int operator()(BatchDesc &d) const override {
    d.tag_len = (uint32_t)tag_len;
    d.num_keys = (uint32_t)km->num_keys;
    d.valid = valid;
    return launch_desc(km, d, open, stream);
  }
};

bool check_iov_batch(const EVP_AEAD *aead, const BSSL_AMD_IOV_BATCH *b) {
  if (!b) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return false;
  }
  if (b->num_records == 0) return true;
  if (!b->iovecs || !b->iovec_start || !b->nonces || !b->tags ||
      (b->aadvecs && !b->aadvec_start)) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return false;
  }
  BSSL_AMD_BATCH probe = {};
  probe.num_records = b->num_records;
  probe.in = probe.out = reinterpret_cast<uint8_t *>(1);
  probe.nonces = b->nonces;
  probe.nonce_len = b->nonce_len;
  probe.tags = b->tags;
  return check_batch(aead, &probe);  // nonce-length rules of the AEAD
}

IovBatchDesc iov_desc(const BSSL_AMD_IOV_BATCH *b) {
  static_assert(sizeof(IovecDev) == sizeof(CRYPTO_IOVEC), "CRYPTO_IOVEC layout");
  static_assert(sizeof(IvecDev) == sizeof(CRYPTO_IVEC), "CRYPTO_IVEC layout");
  IovBatchDesc d;
  d.num_records = b->num_records;
  d.iovecs = reinterpret_cast<const IovecDev *>(b->iovecs);
  d.iovec_start = b->iovec_start;
  d.aadvecs = reinterpret_cast<const IvecDev *>(b->aadvecs);
  d.aadvec_start = b->aadvec_start;
  d.nonces = b->nonces;
  d.nonce_len = b->nonce_len;
  d.tags = b->tags;
  d.status = b->status;
  return d;
}

}  // namespace

// aead.cc.inc:316-361 (sealv) for a batch of device records.
int EVP_AEAD_CTX_sealv_batch_device(const EVP_AEAD_CTX *ctx, const BSSL_AMD_IOV_BATCH *batch,
                                    void *hip_stream) {
  if (!ctx || !ctx->aead || !check_iov_batch(ctx->aead, batch)) return 0;
  if (batch->num_records == 0) return 1;
  CtxState *st = state_of(ctx);
  if (!on_key_device(st->km)) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  uint8_t *valid = nullptr;
  if (ctx->aead->tls) {  // the monotonic-nonce check, as for contiguous batches
    if (batch->nonce_len != 12) {
      PUT_ERROR(CIPHER_R_UNSUPPORTED_NONCE_SIZE);
      return 0;
    }
    if (hipMallocAsync(reinterpret_cast<void **>(&valid), batch->num_records, s) != hipSuccess) {
      PUT_ERROR(ERR_R_MALLOC_FAILURE);
      return 0;
    }
    if (tls_nonce_scan(batch->nonces, batch->num_records, ctx->aead->tls, &st->min_next_nonce,
                       &st->mask, valid, 0, hip_stream) != 0) {
      hipFreeAsync(valid, s);
      PUT_ERROR(ERR_R_INTERNAL_ERROR);
      return 0;
    }
  }
  const int rc = iov_batch_run(iov_desc(batch),
                               KeyRunner(st->km, ctx->tag_len, false, hip_stream, valid),
                               hip_stream);
  if (valid) hipFreeAsync(valid, s);
  if (rc != 0) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  return 1;
}

// aead.cc.inc:531-584 (openv_detached) for a batch of device records; the
// tags (tag_len bytes each) are read at tags + i*tag_len.
int EVP_AEAD_CTX_openv_detached_batch_device(const EVP_AEAD_CTX *ctx,
                                             const BSSL_AMD_IOV_BATCH *batch, void *hip_stream) {
  if (!ctx || !ctx->aead || !check_iov_batch(ctx->aead, batch)) return 0;
  if (batch->num_records == 0) return 1;
  if (!on_key_device(state_of(ctx)->km)) return 0;
  const int rc = iov_batch_run(
      iov_desc(batch), KeyRunner(state_of(ctx)->km, ctx->tag_len, true, hip_stream, nullptr),
      hip_stream);
  if (rc != 0) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  return 1;
}

struct bssl_amd_keyset_st {
  KeyMaterial *km;
  size_t tag_len;
};

BSSL_AMD_KEYSET *BSSL_AMD_KEYSET_new(const EVP_AEAD *aead, const uint8_t *keys,
                                     size_t num_keys, size_t tag_len) {
  if (!aead || !keys || num_keys == 0 || num_keys > 0xfffffffeu) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return nullptr;
  }
  if (!resolve_tag_len(aead, &tag_len)) return nullptr;
  KeyMaterial *km = make_keys(aead, keys, num_keys);
  if (!km) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    return nullptr;
  }
  BSSL_AMD_KEYSET *ks = new (std::nothrow) bssl_amd_keyset_st{km, tag_len};
  if (!ks) free_keys(km);
  return ks;
}

void BSSL_AMD_KEYSET_free(BSSL_AMD_KEYSET *ks) {
  if (!ks) return;
  free_keys(ks->km);
  delete ks;
}

size_t BSSL_AMD_KEYSET_num_keys(const BSSL_AMD_KEYSET *ks) { return ks ? ks->km->num_keys : 0; }

int BSSL_AMD_KEYSET_seal_batch_device(const BSSL_AMD_KEYSET *ks, const BSSL_AMD_BATCH *batch,
                                      void *hip_stream) {
  if (!ks || !check_batch(ks->km->aead, batch)) return 0;
  if (ks->km->aead->tls) {  // per-key nonce state: one EVP_AEAD_CTX per key instead
    PUT_ERROR(CIPHER_R_CTRL_NOT_IMPLEMENTED);
    return 0;
  }
  if (batch->num_records == 0) return 1;
  if (!on_key_device(ks->km)) return 0;
  return run_batch(ks->km, ks->tag_len, batch, false, true, hip_stream);
}

int BSSL_AMD_KEYSET_open_batch_device(const BSSL_AMD_KEYSET *ks, const BSSL_AMD_BATCH *batch,
                                      void *hip_stream) {
  if (!ks || !check_batch(ks->km->aead, batch)) return 0;
  if (batch->num_records == 0) return 1;
  if (!on_key_device(ks->km)) return 0;
  return run_batch(ks->km, ks->tag_len, batch, true, true, hip_stream);
}

int BSSL_AMD_set_device(int device) { return hipSetDevice(device) == hipSuccess; }

int BSSL_AMD_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int BSSL_AMD_synth_fill_device(uint64_t first_record, size_t n, const uint64_t *offsets,
                               const uint64_t *lengths, uint8_t *pt, uint8_t *nonces,
                               uint8_t *ads, void *hip_stream) {
  return launch_synth(first_record, n, offsets, lengths, pt, nonces, ads, hip_stream) == 0;
}

void BSSL_AMD_set_kernel_timing(int enable) { t_timing.enabled = enable != 0; }

size_t BSSL_AMD_collect_kernel_times(double *out_ms, size_t max) {
  size_t n = 0;
  for (auto &e : t_timing.pending) {
    float ms = 0;
    if (hipEventSynchronize(reinterpret_cast<hipEvent_t>(e.stop)) == hipSuccess &&
        hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(e.start),
                            reinterpret_cast<hipEvent_t>(e.stop)) == hipSuccess) {
      if (out_ms && n < max) out_ms[n] = ms;
      n++;
      t_timing.last_ms = ms;
    }
    t_timing.free_pairs.push_back(e);
  }
  t_timing.pending.clear();
  return n;
}

int BSSL_AMD_set_aes_gcm_engine(int engine) { return set_gcm_engine(engine); }
int BSSL_AMD_aes_gcm_engine(void) { return gcm_engine(); }
int BSSL_AMD_test_set_bs_ek0_producers(int on) { return set_bs_ek0_producers(on != 0) ? 1 : 0; }
int BSSL_AMD_test_set_gcm_mix(int bitsliced_waves) { return set_gcm_mix(bitsliced_waves); }

size_t BSSL_AMD_gcm_key_tables(const uint8_t *keys, size_t key_len, size_t n, int on_device,
                               uint8_t *out) {
  if (!out) return sizeof(GcmKeyDev);
  if (key_len != 16 && key_len != 24 && key_len != 32) return 0;
  GcmKeyDev *h = reinterpret_cast<GcmKeyDev *>(out);
  if (!on_device) {
    for (size_t i = 0; i < n; i++)
      if (!gcm_key_setup(keys + i * key_len, key_len, &h[i])) return 0;
    return n;
  }
  GcmKeyDev *d = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(&d), n * sizeof(GcmKeyDev)) != hipSuccess) return 0;
  bool ok = gcm_key_setup_device(keys, key_len, n, d, nullptr) == 0 &&
            hipMemcpy(out, d, n * sizeof(GcmKeyDev), hipMemcpyDeviceToHost) == hipSuccess;
  hipMemset(d, 0, n * sizeof(GcmKeyDev));
  hipDeviceSynchronize();
  hipFree(d);
  return ok ? n : 0;
}

double BSSL_AMD_last_kernel_ms(void) { return t_timing.last_ms; }
const char *BSSL_AMD_last_kernel_name(void) { return t_timing.last_name; }

}  // extern "C"

// ---- TLS record layer over device batches (bssl_amd/tls.h) ---------------
// SSLAEADContext (ssl/ssl_aead_ctx.cc) + do_seal_record / tls_open_record
// (ssl/tls_record.cc) for a batch of records; the per-record nonce, header,
// AD and inner type are built on the device (tls_records.hip) and the records
// go through the same bulk kernels as any batch.

struct bssl_amd_tls_aead_st {
  EVP_AEAD_CTX ctx;
  bool seal;
  bool tls13;
  bool xor_nonce;
  uint32_t explicit_len;
  uint8_t fixed_iv[12];
  uint64_t seq;
};

namespace {

const EVP_AEAD *tls_record_aead(const EVP_AEAD *aead, bool tls13) {
  // ssl_cipher_get_evp_aead (ssl/ssl_cipher.cc): the nonce-checking variants
  // for AES-GCM in TLS 1.2 / 1.3.
  if (aead == &kAes128Gcm) return tls13 ? &kAes128GcmTls13 : &kAes128GcmTls12;
  if (aead == &kAes256Gcm) return tls13 ? &kAes256GcmTls13 : &kAes256GcmTls12;
  if (aead == &kChaChaPoly) return aead;
  return nullptr;
}

int tls_records(BSSL_AMD_TLS_AEAD *t, const BSSL_AMD_TLS_RECORDS *r, void *stream) {
  if (!t || !r || (r->num_records && (!r->in || !r->out || !r->prefix || !r->suffix))) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return 0;
  }
  const uint64_t n = r->num_records;
  if (n == 0) return 1;
  // tls_record.cc:305-308: the sequence number must not wrap.
  if (t->seq > UINT64_MAX - n) {
    PUT_ERROR(ERR_R_OVERFLOW);
    return 0;
  }
  if (!t->seal && t->tls13 && !r->types) {  // open returns the inner types
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return 0;
  }
  const EVP_AEAD_CTX *ctx = &t->ctx;
  CtxState *st = state_of(ctx);
  if (!on_key_device(st->km)) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint32_t ad_stride = t->tls13 ? 5 : 13;
  const uint32_t extra_len = t->tls13 ? 1 : 0;
  const uint32_t tag_len = ctx->tag_len;
  const uint32_t prefix_len = 5 + t->explicit_len;
  const uint32_t suffix_len = extra_len + tag_len;
  // Scratch: nonces (12 B), AD, inner types (seal, TLS 1.3) and flags per record.
  uint8_t *buf = nullptr;
  const size_t bytes = n * (12 + ad_stride + 1 + 1);
  if (hipMallocAsync(reinterpret_cast<void **>(&buf), bytes, s) != hipSuccess) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    return 0;
  }
  uint8_t *d_nonce = buf, *d_ad = d_nonce + 12 * n, *d_type = d_ad + ad_stride * n,
          *d_valid = d_type + n;
  int ok = hipMemsetAsync(d_valid, 1, n, s) == hipSuccess;
  TlsPrepare p;
  p.n = n;
  p.lengths = r->lengths;
  p.record_len = r->record_len;
  p.types = r->types;
  p.type = r->type;
  memcpy(p.fixed_iv, t->fixed_iv, 12);
  p.seq = t->seq;
  p.xor_nonce = t->xor_nonce;
  p.tls13 = t->tls13;
  p.record_version = 0x0303;  // tls_record_version: TLS 1.3 records say TLS 1.2
  p.explicit_len = t->explicit_len;
  p.extra_len = extra_len;
  p.tag_len = tag_len;
  p.prefix_len = prefix_len;
  p.ad_stride = ad_stride;
  p.open = !t->seal;
  p.nonces = d_nonce;
  p.prefix = r->prefix;
  p.ad = d_ad;
  p.extra = d_type;
  p.valid = d_valid;
  if (ok) ok = launch_tls_prepare(p, stream) == 0;
  if (ok && t->seal && ctx->aead->tls)  // the AEAD's own nonce check (sealv)
    ok = tls_nonce_scan(d_nonce, n, ctx->aead->tls, &st->min_next_nonce, &st->mask, d_valid, 1,
                        stream) == 0;
  if (ok) {
    BatchDesc d;
    memset(&d, 0, sizeof(d));
    d.in = r->in;
    d.out = r->out;
    d.offsets = r->offsets;
    d.lengths = r->lengths;
    d.record_stride = r->record_stride;
    d.record_len = r->record_len;
    d.nonces = d_nonce;
    d.nonce_len = 12;
    d.ad = d_ad;
    d.ad_stride = ad_stride;
    d.ad_len = ad_stride;
    d.tags = r->suffix + extra_len;
    d.tag_stride = suffix_len;
    d.status = r->status;
    d.num_records = n;
    d.tag_len = tag_len;
    d.num_keys = 1;
    d.valid = d_valid;
    if (extra_len) {
      d.extra_len = extra_len;
      if (t->seal) {  // inner type in, its ciphertext to the suffix
        d.extra = d_type;
        d.extra_stride = 1;
        d.extra_out = r->suffix;
        d.extra_out_stride = suffix_len;
      } else {        // sealed inner type from the suffix, plaintext type out
        d.extra = r->suffix;
        d.extra_stride = suffix_len;
        d.extra_out = r->types;
        d.extra_out_stride = 1;
      }
    }
    const KernelEvents *ev = timing_pair();
    const int eng = gcm_engine();
    const int rc = ctx->aead->kind == kAeadAesGcm
                       ? launch_gcm(static_cast<const GcmKeyDev *>(st->km->dev), d, !t->seal,
                                    st->km->nr, stream, ev, eng)
                       : launch_chacha(static_cast<const ChaChaKeyDev *>(st->km->dev), d,
                                       !t->seal, false, stream, ev);
    t_timing.last_name = ctx->aead->kind == kAeadAesGcm ? gcm_kernel_name(eng) : "chacha_poly_kernel";
    ok = rc == 0;
    // TLS 1.2 open reports the header type (tls_record.cc:197-235).
    if (ok && !t->seal && !t->tls13 && r->types)
      ok = hipMemcpy2DAsync(r->types, 1, r->prefix, prefix_len, 1, n, hipMemcpyDeviceToDevice,
                            s) == hipSuccess;
  }
  hipFreeAsync(buf, s);
  if (!ok) {
    PUT_ERROR(ERR_R_INTERNAL_ERROR);
    return 0;
  }
  t->seq += n;
  return 1;
}

}  // namespace

extern "C" {

BSSL_AMD_TLS_AEAD *BSSL_AMD_TLS_AEAD_new(enum evp_aead_direction_t direction, uint16_t version,
                                         const EVP_AEAD *aead, const uint8_t *key,
                                         size_t key_len, const uint8_t *fixed_iv,
                                         size_t fixed_iv_len, uint64_t seq) {
  // SSLAEADContext::Create (ssl_aead_ctx.cc:44-123), AEAD suites only.
  if ((version != BSSL_AMD_TLS1_2_VERSION && version != BSSL_AMD_TLS1_3_VERSION) || !aead ||
      !fixed_iv) {
    PUT_ERROR(ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED);
    return nullptr;
  }
  const bool tls13 = version == BSSL_AMD_TLS1_3_VERSION;
  const EVP_AEAD *rec_aead = tls_record_aead(aead, tls13);
  if (!rec_aead) {
    PUT_ERROR(CIPHER_R_UNSUPPORTED_KEY_SIZE);
    return nullptr;
  }
  // TLS 1.3 and TLS 1.2 ChaCha20-Poly1305 XOR a 12-byte IV with the sequence
  // number; TLS 1.2 AES-GCM prepends a 4-byte IV to an 8-byte explicit nonce.
  const bool xor_nonce = tls13 || aead->kind == kAeadChaChaPoly;
  if (fixed_iv_len != (xor_nonce ? 12u : 4u)) {
    PUT_ERROR(CIPHER_R_INVALID_NONCE_SIZE);
    return nullptr;
  }
  BSSL_AMD_TLS_AEAD *t = new (std::nothrow) bssl_amd_tls_aead_st;
  if (!t) {
    PUT_ERROR(ERR_R_MALLOC_FAILURE);
    return nullptr;
  }
  EVP_AEAD_CTX_zero(&t->ctx);
  if (!EVP_AEAD_CTX_init_with_direction(&t->ctx, rec_aead, key, key_len,
                                        EVP_AEAD_DEFAULT_TAG_LENGTH, direction)) {
    delete t;
    return nullptr;
  }
  t->seal = direction == evp_aead_seal;
  t->tls13 = tls13;
  t->xor_nonce = xor_nonce;
  t->explicit_len = xor_nonce ? 0 : 8;
  memset(t->fixed_iv, 0, sizeof(t->fixed_iv));
  memcpy(t->fixed_iv, fixed_iv, fixed_iv_len);
  t->seq = seq;
  if (t->seal && tls13 && t->ctx.aead->tls == 13 && seq != 0) {
    // The tls13 AEAD takes its nonce mask from the first sealed nonce, which
    // it assumes is sequence number 0 (e_aes.cc.inc:1181-1185).  A writer
    // that starts mid-stream gets the state the AEAD would have after
    // sealing records 0 .. seq-1: mask = the IV's low 64 bits, next >= seq.
    CtxState *st = state_of(&t->ctx);
    st->mask = load_be64(t->fixed_iv + 4);
    st->min_next_nonce = seq;
  }
  return t;
}

void BSSL_AMD_TLS_AEAD_free(BSSL_AMD_TLS_AEAD *t) {
  if (!t) return;
  EVP_AEAD_CTX_cleanup(&t->ctx);
  delete t;
}

size_t BSSL_AMD_TLS_AEAD_prefix_len(const BSSL_AMD_TLS_AEAD *t) { return 5 + t->explicit_len; }

size_t BSSL_AMD_TLS_AEAD_suffix_len(const BSSL_AMD_TLS_AEAD *t) {
  return (t->tls13 ? 1 : 0) + t->ctx.tag_len;
}

uint64_t BSSL_AMD_TLS_AEAD_sequence(const BSSL_AMD_TLS_AEAD *t) { return t->seq; }

int BSSL_AMD_TLS_AEAD_seal_records_device(BSSL_AMD_TLS_AEAD *t, const BSSL_AMD_TLS_RECORDS *r,
                                          void *hip_stream) {
  if (t && !t->seal) {
    PUT_ERROR(CIPHER_R_INVALID_OPERATION);
    return 0;
  }
  return tls_records(t, r, hip_stream);
}

int BSSL_AMD_TLS_AEAD_open_records_device(BSSL_AMD_TLS_AEAD *t, const BSSL_AMD_TLS_RECORDS *r,
                                          void *hip_stream) {
  if (t && t->seal) {
    PUT_ERROR(CIPHER_R_INVALID_OPERATION);
    return 0;
  }
  return tls_records(t, r, hip_stream);
}

}  // extern "C"
