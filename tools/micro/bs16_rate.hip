// Issue-rate probe of the bs16 bitsliced AES rounds (csrc/bs16_aes.h) on
// gfx950: AES-only keystream throughput of the round code at 16 and 8 waves
// per CU, plus an S-box-only variant, and a known-answer self-check of the
// bs16 cipher (16 blocks per lane, two state columns per register).
// Diagnostic tool, not product code.
//   hipcc --offload-arch=gfx950 -O3 -I../../boringssl_amd/csrc -o bs16_rate bs16_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "bs16_aes.h"

using namespace bssl_amd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

// Round-key masks of the bs16 layout, precomputed per round (64 per round):
// mask (r, h, b) of round rd at [rd][r][h][b].
struct Masks { uint32_t m[15][4][2][8]; };

template <int NR>
__device__ __forceinline__ void bs16_cipher_tab(uint32_t (&p)[4][2][8], const uint32_t *__restrict__ mt) {
#pragma unroll 1
  for (int rd = 1; rd <= NR; rd++) {
    const uint32_t *km_rd = mt + rd * 64;
    const bool last = rd == NR;
    uint32_t np[4][2][8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t a[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        sbox_planes(p[r][(h + r) & 1], a[r]);
        if (((h + r) >> 1) & 1) {
#pragma unroll
          for (int b = 0; b < 8; b++) a[r][b] = swap16(a[r][b]);
        }
      }
      uint32_t km[4][8];
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 8; b++) km[r][b] = __builtin_amdgcn_readfirstlane(km_rd[(r * 2 + h) * 8 + b]);
      if (!last) {
        uint32_t o[4][8];
        bs16_mix(a, o, km);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = o[r][b];
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int b = 0; b < 8; b++) np[r][h][b] = a[r][b] ^ km[r][b];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int b = 0; b < 8; b++) p[r][h][b] = np[r][h][b];
  }
}

__device__ __forceinline__ void init_state(uint32_t (&p)[4][2][8]) {
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int b = 0; b < 8; b++) p[r][h][b] = (threadIdx.x + 1) * 0x9E3779B9u * (r * 16 + h * 8 + b + 1);
}

__device__ __forceinline__ uint32_t fold(const uint32_t (&p)[4][2][8]) {
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int b = 0; b < 8; b++) acc ^= p[r][h][b];
  return acc;
}

// V 0: product bs16_cipher (SALU masks); 1: masks by scalar loads; 2: S-boxes only.
template <int V, int T>
__global__ __launch_bounds__(T) void thr(uint32_t *out, const uint32_t *rkp, const uint32_t *mt,
                                        int iters) {
  uint32_t p[4][2][8];
  init_state(p);
  for (int it = 0; it < iters; it++) {
    if constexpr (V == 0) {
      bs16_cipher<10>(p, rkp);
    } else if constexpr (V == 1) {
      bs16_cipher_tab<10>(p, mt);
    } else {
#pragma unroll 1
      for (int rd = 0; rd < 10; rd++) {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int h = 0; h < 2; h++) {
            uint32_t a[8];
            sbox_planes(p[r][h], a);
#pragma unroll
            for (int b = 0; b < 8; b++) p[r][h][b] = a[b];
          }
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = fold(p);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // Any round keys do for throughput (the code path does not depend on them).
  std::vector<uint32_t> rk(60), mt(15 * 64);
  for (int i = 0; i < 60; i++) rk[i] = 0x01234567u * (i + 1) ^ (i << 24);
  for (int rd = 0; rd < 15; rd++)
    for (int r = 0; r < 4; r++)
      for (int h = 0; h < 2; h++)
        for (int b = 0; b < 8; b++) {
          const uint32_t *w = &rk[4 * (rd % 11)];
          const uint32_t lo = (w[h] >> (8 * r + b)) & 1u, hi = (w[h + 2] >> (8 * r + b)) & 1u;
          mt[rd * 64 + (r * 2 + h) * 8 + b] = (lo | (hi << 16)) * 0xffffu;
        }
  uint32_t *drk, *dmt, *dsink;
  CK(hipMalloc(&drk, 60 * 4));
  CK(hipMalloc(&dmt, mt.size() * 4));
  CK(hipMalloc(&dsink, 64 << 20));
  CK(hipMemcpy(drk, rk.data(), 60 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmt, mt.data(), mt.size() * 4, hipMemcpyHostToDevice));
  auto run = [&](const char *name, auto kern, int threads) -> int {
    const int iters = 64, grid = cus;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, dsink, drk, dmt, 2);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, dsink, drk, dmt, iters);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double blocks = (double)grid * threads * 16 * iters;
    printf("%-34s waves/CU=%2d: %.3f ms  %.1f GiB/s of AES-128 keystream  %.3f blocks/ns/CU\n",
           name, threads / 64, best, blocks * 16 / (best * 1e-3) / (1 << 30),
           blocks / (best * 1e6) / cus);
    return 0;
  };
  if (run("bs16 rounds (SALU masks)", thr<0, 1024>, 1024)) return 1;
  if (run("bs16 rounds (SALU masks)", thr<0, 512>, 512)) return 1;
  if (run("bs16 rounds (scalar-load masks)", thr<1, 1024>, 1024)) return 1;
  if (run("bs16 rounds (scalar-load masks)", thr<1, 512>, 512)) return 1;
  if (run("S-boxes only (8 per round)", thr<2, 1024>, 1024)) return 1;
  if (run("S-boxes only (8 per round)", thr<2, 512>, 512)) return 1;
  return 0;
}
