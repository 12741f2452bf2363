// Microbenchmark: can the vector-memory path (TA/TCP, vector L1) serve
// table lookups beside the LDS?  Per iteration each wave issues NL
// conflict-free ds_read_b32 lookups and NV buffer_load_dword (or _ubyte)
// gathers at random offsets into a small global table (L1-resident), then
// waits for both.  Reported: CU cycles per wave-iteration, so mixes can be
// compared with the LDS-only loop.  Diagnostic tool, not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int NL, int NV, int TBYTES, bool U8>
__global__ void __launch_bounds__(1024) k(const uint32_t *tbl, uint32_t *out, int iters, uint64_t *clk) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[65536];
  for (int e = threadIdx.x; e < 16384; e += blockDim.x)
    reinterpret_cast<uint32_t *>(smem)[e] = e * 0x9E3779B9u;
  __syncthreads();
  v4i rsrc;
  const uint64_t base = reinterpret_cast<uint64_t>(tbl);
  rsrc[0] = (int)(uint32_t)base;
  rsrc[1] = (int)(uint32_t)(base >> 32);
  rsrc[2] = TBYTES;
  rsrc[3] = 0x00020000;  // gfx950 raw buffer: data format 32
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = threadIdx.x * 0x9E3779B9u + blockIdx.x * 0x85EBCA6Bu;
  uint32_t acc = 0;
  for (int i = 0; i < iters; i++) {
    uint32_t v[NL + NV + 1];
#pragma unroll
    for (int u = 0; u < NL; u++) {
      uint32_t a = ((((x >> (u & 15)) ^ (u * 37)) & 255) * 128 + (lane & 31) * 4) & 0xffff;
      asm volatile("ds_read_b32 %0, %1" : "=v"(v[u]) : "v"(a));
    }
#pragma unroll
    for (int u = 0; u < NV; u++) {
      uint32_t off = U8 ? (((x >> (u & 15)) ^ (u * 53)) & (TBYTES - 1))
                        : ((((x >> (u & 15)) ^ (u * 53)) * 4) & (TBYTES - 4));
      if (U8)
        asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen" : "=v"(v[NL + u]) : "v"(off), "s"(rsrc));
      else
        asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(v[NL + u]) : "v"(off), "s"(rsrc));
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < NL + NV; u++) acc += v[u];
    x = x * 1664525u + 1013904223u + acc;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NL, int NV, int TBYTES, bool U8>
void run(int waves, int cus, const uint32_t *tbl, uint32_t *d, uint64_t *clk) {
  const int iters = 2000;
  hipLaunchKernelGGL((k<NL, NV, TBYTES, U8>), dim3(cus), dim3(waves * 64), 0, 0, tbl, d, iters, clk);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k<NL, NV, TBYTES, U8>), dim3(cus), dim3(waves * 64), 0, 0, tbl, d, iters, clk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  uint64_t c;
  hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
  // CU cycles per wave-iteration (s_memtime counts shader clocks).
  const double cyc = (double)c / ((double)iters * waves);
  printf("NL=%2d NV=%2d tbl=%5dB %s waves=%2d  %.3f ms  %.1f CU-cycles/wave-iter  %.2f cyc/lookup\n", NL, NV,
         TBYTES, U8 ? "u8 " : "u32", waves, ms, cyc, cyc / (NL + NV));
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *d, *tbl;
  uint64_t *clk;
  hipMalloc(&d, 256 * 1024 * 64 * 4);
  hipMalloc(&tbl, 65536);
  hipMemset(tbl, 0x5a, 65536);
  hipMalloc(&clk, 16);
  for (int w : {8, 16}) {
    run<16, 0, 1024, false>(w, cus, tbl, d, clk);
    run<0, 16, 1024, false>(w, cus, tbl, d, clk);
    run<0, 16, 256, true>(w, cus, tbl, d, clk);
    run<0, 16, 4096, false>(w, cus, tbl, d, clk);
    run<12, 4, 1024, false>(w, cus, tbl, d, clk);
    run<14, 2, 1024, false>(w, cus, tbl, d, clk);
    run<16, 4, 1024, false>(w, cus, tbl, d, clk);
    run<16, 4, 256, true>(w, cus, tbl, d, clk);
    run<16, 8, 1024, false>(w, cus, tbl, d, clk);
  }
  return 0;
}
