// synth.hip -- device-side generator of the synthetic record workload
// (BENCH/TEST SUPPORT, not part of the AEAD path).  Same definitions as
// oracle/synth.h, implemented independently for the GPU so that 16-64 GiB
// batches are produced in HBM without a host round trip.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace bssl_amd {
namespace {

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr uint64_t kIvSeed = 0x1D5EED, kPtSeed = 1;

// One workgroup per record; threads fill 8-byte words.
__global__ void synth_kernel(uint64_t first, uint64_t n, const uint64_t *__restrict__ offsets,
                             const uint64_t *__restrict__ lengths, uint8_t *pt,
                             uint8_t *nonces, uint8_t *ads) {
  for (uint64_t j = blockIdx.x; j < n; j += gridDim.x) {
    const uint64_t i = first + j;
    const uint64_t len = lengths[j];
    uint8_t *p = pt ? pt + offsets[j] : nullptr;
    const uint64_t words = len / 8;
    if (p) {
      if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        for (uint64_t w = threadIdx.x; w < words; w += blockDim.x)
          reinterpret_cast<uint64_t *>(p)[w] = splitmix(kPtSeed ^ (i << 32) ^ w);
      } else {
        for (uint64_t w = threadIdx.x; w < words; w += blockDim.x) {
          uint64_t v = splitmix(kPtSeed ^ (i << 32) ^ w);
          for (int b = 0; b < 8; b++) p[8 * w + b] = (uint8_t)(v >> (8 * b));
        }
      }
      if (threadIdx.x == 0 && (len & 7)) {
        uint64_t v = splitmix(kPtSeed ^ (i << 32) ^ words);
        for (uint64_t b = 0; b < (len & 7); b++) p[8 * words + b] = (uint8_t)(v >> (8 * b));
      }
    }
    if (threadIdx.x == 0) {
      if (nonces) {
        uint8_t *nn = nonces + 12 * j;
        for (int b = 0; b < 12; b++) {
          uint8_t v = (uint8_t)(splitmix(kIvSeed + (uint64_t)b / 8) >> (8 * (b % 8)));
          if (b >= 4) v ^= (uint8_t)(i >> (8 * (11 - b)));
          nn[b] = v;
        }
      }
      if (ads) {
        uint8_t *a = ads + 13 * j;
        for (int b = 0; b < 8; b++) a[b] = (uint8_t)(i >> (8 * (7 - b)));
        a[8] = 0x17;
        a[9] = 0x03;
        a[10] = 0x03;
        a[11] = (uint8_t)(len >> 8);
        a[12] = (uint8_t)len;
      }
    }
  }
}

}  // namespace

int launch_synth(uint64_t first, size_t n, const uint64_t *offsets, const uint64_t *lengths,
                 uint8_t *pt, uint8_t *nonces, uint8_t *ads, void *stream) {
  if (n == 0) return 0;
  const unsigned grid = (unsigned)(n < 65536 ? n : 65536);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (uint64_t)first, (uint64_t)n,
                     offsets, lengths, pt, nonces, ads);
  return (int)hipGetLastError();
}

}  // namespace bssl_amd
