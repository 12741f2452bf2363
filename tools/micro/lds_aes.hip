// Microbenchmark: LDS T-table lookup throughput of AES-like rounds vs waves
// per CU and independent blocks per lane (diagnostic tool, not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int K>
__device__ __forceinline__ uint32_t taddr(uint32_t lc, uint32_t s) {
  return __builtin_amdgcn_perm(lc, s, 0x0c0c0004u | (K << 8));
}
__device__ __forceinline__ uint32_t tl(const uint8_t *smem, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(smem + a);
}
__device__ __forceinline__ uint32_t rotl16(uint32_t v) { return __builtin_amdgcn_alignbit(v, v, 16); }

template <int S>
__global__ void k(uint32_t *out, int rounds, uint32_t key) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[65536];
  for (int e = threadIdx.x; e < 16384; e += blockDim.x)
    reinterpret_cast<uint32_t *>(smem)[e] = e * 0x9E3779B9u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t lc0 = (lane & 31) * 4, lc1 = lc0 + 128;
  uint32_t s[S][4];
  for (int i = 0; i < S; i++)
    for (int c = 0; c < 4; c++) s[i][c] = (threadIdx.x + blockIdx.x * 977) * (i + 3) * (c + 7);
  for (int r = 0; r < rounds; r++) {
#pragma unroll
    for (int i = 0; i < S; i++) {
      uint32_t s0 = s[i][0], s1 = s[i][1], s2 = s[i][2], s3 = s[i][3];
      const uint32_t x00 = tl(smem, taddr<0>(lc0, s0)), x01 = tl(smem, taddr<1>(lc1, s1)),
                     x02 = tl(smem, taddr<2>(lc0, s2)), x03 = tl(smem, taddr<3>(lc1, s3));
      const uint32_t x10 = tl(smem, taddr<0>(lc0, s1)), x11 = tl(smem, taddr<1>(lc1, s2)),
                     x12 = tl(smem, taddr<2>(lc0, s3)), x13 = tl(smem, taddr<3>(lc1, s0));
      const uint32_t x20 = tl(smem, taddr<0>(lc0, s2)), x21 = tl(smem, taddr<1>(lc1, s3)),
                     x22 = tl(smem, taddr<2>(lc0, s0)), x23 = tl(smem, taddr<3>(lc1, s1));
      const uint32_t x30 = tl(smem, taddr<0>(lc0, s3)), x31 = tl(smem, taddr<1>(lc1, s0)),
                     x32 = tl(smem, taddr<2>(lc0, s1)), x33 = tl(smem, taddr<3>(lc1, s2));
      s[i][0] = xor3(x00, x01, rotl16(xor3(x02, x03, key)));
      s[i][1] = xor3(x10, x11, rotl16(xor3(x12, x13, key + 1)));
      s[i][2] = xor3(x20, x21, rotl16(xor3(x22, x23, key + 2)));
      s[i][3] = xor3(x30, x31, rotl16(xor3(x32, x33, key + 3)));
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < S; i++) acc ^= s[i][0] ^ s[i][1] ^ s[i][2] ^ s[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int S>
void run(int waves, int cus, uint32_t *d) {
  const int rounds = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = cus;  // one workgroup per CU (64 KiB LDS each... 2 fit; use 1 by size)
  hipLaunchKernelGGL(k<S>, dim3(grid), dim3(waves * 64), 0, 0, d, rounds, 1u);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<S>, dim3(grid), dim3(waves * 64), 0, 0, d, rounds, 1u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  // LDS array cycles needed per CU: waves * S * rounds * 16 b32 reads * 2 cycles
  const double need = (double)waves * S * rounds * 16 * 2;
  printf("S=%d waves=%2d  %.3f ms  lds-array-cycles/CU=%.3g  -> util @2.4GHz %.1f%%  lookups/ns/CU %.2f\n", S, waves, ms,
         need, 100.0 * need / (ms * 1e-3 * 2.4e9), waves * 64.0 * S * rounds * 16 / (ms * 1e6));
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *d;
  hipMalloc(&d, 256 * 1024 * 64 * 4);
  for (int w : {4, 8, 12, 16}) run<1>(w, cus, d);
  for (int w : {4, 8, 12, 16}) run<2>(w, cus, d);
  for (int w : {4, 8}) run<4>(w, cus, d);
  return 0;
}
