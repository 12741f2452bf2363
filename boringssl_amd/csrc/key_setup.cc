// key_setup.cc -- per-key setup, the analogue of the reference's
// CRYPTO_gcm128_init_aes_key (crypto/fipsmodule/aes/gcm.cc.inc:253-296): the
// tables of key_sched.h built on the host for one key (EVP_AEAD_CTX_init) and
// by a device kernel, one lane per key, for keysets (BSSL_AMD_KEYSET_new:
// 64K keys of config 5 in about a millisecond instead of seconds of host
// work and a host-to-device copy of 12,816 B per key).  Both run the same
// code, so their tables are the same bytes (tests/test_key_setup.py).
#include <string.h>

#include "key_sched.h"

namespace bssl_amd {

void secure_zero(void *p, size_t n) {
  if (n) explicit_bzero(p, n);
}

bool gcm_key_setup(const uint8_t *key, size_t key_len, GcmKeyDev *out) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return false;
  return gcm_key_tables(key, (int)key_len, out);
}

namespace {

// Key i's tables from raw key bytes keys[i * key_len ...].  The tables are
// written by their own lane (12,816 B each, scattered 16-byte stores that
// L2 merges into full lines).
__global__ __launch_bounds__(64) void gcm_key_setup_kernel(const uint8_t *__restrict__ keys,
                                                            int key_len, uint64_t n,
                                                            GcmKeyDev *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint8_t k[32];
  for (int j = 0; j < 32; j++) k[j] = j < key_len ? keys[i * key_len + j] : 0;
  gcm_key_tables(k, key_len, out + i);
  ks_wipe(k, sizeof(k));
}

}  // namespace

// n keys of key_len bytes (host memory) -> their tables in device memory
// `out` (n entries), on `s`; returns 0 or a HIP error.  The raw keys pass
// through a device staging buffer that is zeroed before it is freed.
int gcm_key_setup_device(const uint8_t *keys, size_t key_len, size_t n, GcmKeyDev *out,
                         hipStream_t s) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return 1;
  if (!n) return 0;
  uint8_t *raw = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void **>(&raw), n * key_len, s);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyAsync(raw, keys, n * key_len, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(gcm_key_setup_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, raw,
                       (int)key_len, (uint64_t)n, out);
    e = hipGetLastError();
  }
  hipMemsetAsync(raw, 0, n * key_len, s);
  hipFreeAsync(raw, s);
  const hipError_t e2 = hipStreamSynchronize(s);
  return (int)(e != hipSuccess ? e : e2);
}

void chacha_key_setup(const uint8_t *key, ChaChaKeyDev *out) {
  for (int i = 0; i < 8; i++) {
    const uint8_t *p = key + 4 * i;
    out->k[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                ((uint32_t)p[3] << 24);
  }
}

}  // namespace bssl_amd
