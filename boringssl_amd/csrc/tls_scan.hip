// tls_scan.hip -- the stateful nonce checks of the tls12 / tls13 AES-GCM AEADs
// over a device batch of seal calls.
//
// Reference (one record per call): aead_aes_gcm_tls12_sealv
// (crypto/fipsmodule/cipher/e_aes.cc.inc:1071-1100) requires the nonce's
// last 8 bytes, as a big-endian counter, to be >= min_next_nonce and not
// UINT64_MAX, then sets min_next_nonce = counter + 1; aead_aes_gcm_tls13_sealv
// (:1162-1202) does the same on counter ^ mask, where the first call ever
// records mask = its counter and passes.
//
// A batch means N such calls in record order.  Record i passes iff
// c_i != MAX and c_i >= M_i with M_i = max(min_next_0, max_{k<i} x_k) and
// x_k = c_k + 1 (0 for c_k == MAX): a failing record k has c_k < M_k, so
// x_k <= M_k and leaving it in the running max changes nothing -- the
// sequential rule is exactly an exclusive prefix-max scan.  The state after
// the batch is max(min_next_0, max_k x_k).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace bssl_amd {
namespace {

constexpr uint64_t kMax = ~uint64_t(0);

__device__ __forceinline__ uint64_t be64(const uint8_t *p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
  return v;
}

// state[0] = min_next_nonce, state[1] = mask, state[2] = mask known (tls12: 1).
__global__ void tls_counters(const uint8_t *__restrict__ nonces, uint64_t n,
                             const uint64_t *__restrict__ state, uint64_t *__restrict__ x) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t mask = state[2] ? state[1] : be64(nonces + 4);
  const uint64_t c = be64(nonces + 12 * i + 4) ^ mask;
  x[i] = c == kMax ? 0 : c + 1;
}

__global__ void tls_valid(const uint8_t *__restrict__ nonces, uint64_t n,
                          const uint64_t *__restrict__ state, const uint64_t *__restrict__ prefix,
                          uint8_t *__restrict__ valid, int and_into) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool first = !state[2];  // tls13 first call: record 0 sets the mask
  const uint64_t mask = first ? be64(nonces + 4) : state[1];
  const uint64_t c = be64(nonces + 12 * i + 4) ^ mask;
  const uint8_t ok = ((first && i == 0) || (c != kMax && c >= prefix[i])) ? 1 : 0;
  valid[i] = and_into ? (uint8_t)(valid[i] & ok) : ok;
}

__global__ void tls_final(const uint8_t *__restrict__ nonces, uint64_t n,
                          const uint64_t *__restrict__ prefix, const uint64_t *__restrict__ x,
                          uint64_t *__restrict__ state) {
  const uint64_t m = prefix[n - 1] > x[n - 1] ? prefix[n - 1] : x[n - 1];
  if (!state[2]) {
    state[1] = be64(nonces + 4);
    state[2] = 1;
  }
  state[0] = m;
}

struct MaxOp {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const {
    return a > b ? a : b;
  }
};

}  // namespace

int tls_nonce_scan(const uint8_t *nonces, uint64_t n, int tls, uint64_t *min_next,
                   uint64_t *mask, uint8_t *valid, int and_into, void *stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return 0;
  // tls13 before its first call: min_next_nonce == 0, mask unknown.
  const uint64_t h_state[3] = {*min_next, tls == 13 ? *mask : 0,
                               (tls == 12 || *min_next != 0) ? 1u : 0u};
  size_t temp = 0;
  if (hipcub::DeviceScan::ExclusiveScan(nullptr, temp, (const uint64_t *)nullptr,
                                        (uint64_t *)nullptr, MaxOp(), uint64_t(0), n, s) !=
      hipSuccess)
    return 1;
  const size_t bytes = 64 + 2 * n * sizeof(uint64_t) + temp;
  uint8_t *buf = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&buf), bytes, s) != hipSuccess) return 2;
  uint64_t *d_state = reinterpret_cast<uint64_t *>(buf);
  uint64_t *x = d_state + 8;
  uint64_t *prefix = x + n;
  void *d_temp = prefix + n;
  int rc = 0;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (hipMemcpyAsync(d_state, h_state, sizeof(h_state), hipMemcpyHostToDevice, s) != hipSuccess)
    rc = 1;
  if (!rc) {
    hipLaunchKernelGGL(tls_counters, dim3(grid), dim3(256), 0, s, nonces, n, d_state, x);
    // The first record's exclusive prefix is min_next_0 (init of the scan).
    if (hipcub::DeviceScan::ExclusiveScan(d_temp, temp, x, prefix, MaxOp(), h_state[0], n, s) !=
        hipSuccess)
      rc = 1;
  }
  if (!rc) {
    hipLaunchKernelGGL(tls_valid, dim3(grid), dim3(256), 0, s, nonces, n, d_state, prefix, valid,
                       and_into);
    hipLaunchKernelGGL(tls_final, dim3(1), dim3(1), 0, s, nonces, n, prefix, x, d_state);
    uint64_t out[3];
    // The context's nonce state lives on the host (as the reference's lives in
    // the EVP_AEAD_CTX): read it back, which synchronises the stream.
    if (hipMemcpyAsync(out, d_state, sizeof(out), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = 1;
    } else {
      *min_next = out[0];
      *mask = out[1];
    }
  }
  hipFreeAsync(buf, s);
  if (!rc && hipGetLastError() != hipSuccess) rc = 1;
  return rc;
}

}  // namespace bssl_amd
