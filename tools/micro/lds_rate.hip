// Microbenchmark: raw LDS read issue rate on gfx950 for independent (not
// dependent) conflict-free random lookups, b32 / b64 / b128, vs waves per CU,
// plus the shader clock (s_memtime vs s_memrealtime at 100 MHz).
// Diagnostic tool, not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int W>  // bytes per lookup: 4, 8, 16
__global__ void k(uint32_t *out, int iters, uint64_t *clk) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[65536];
  for (int e = threadIdx.x; e < 16384; e += blockDim.x)
    reinterpret_cast<uint32_t *>(smem)[e] = e * 0x9E3779B9u;
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t lane = threadIdx.x & 63;
  // Conflict-free: b32 lane l -> bank l%32; b64 lane l -> banks 2(l%32),+1;
  // b128 lane l -> slot (l%16) (16 B).  Row (random) in the upper bits.
  const uint32_t lanepart = W == 4 ? (lane & 31) * 4 : W == 8 ? (lane & 31) * 8 : (lane & 15) * 16;
  const uint32_t rowbytes = W == 4 ? 128 : 256;
  uint32_t x = threadIdx.x * 0x9E3779B9u + blockIdx.x;
  uint32_t addr[16];
#pragma unroll
  for (int u = 0; u < 16; u++) addr[u] = ((((x >> u) ^ (u * 37)) & 255) * rowbytes + lanepart) & 0xffff;
  uint32_t acc = 0;
  for (int i = 0; i < iters; i++) {
    uint32_t v[16][W / 4];
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if constexpr (W == 4)
        asm volatile("ds_read_b32 %0, %1" : "=v"(v[u][0]) : "v"(addr[u]));
      else if constexpr (W == 8)
        asm volatile("ds_read_b64 %0, %1" : "=v"(*reinterpret_cast<uint2 *>(v[u])) : "v"(addr[u]));
      else
        asm volatile("ds_read_b128 %0, %1" : "=v"(*reinterpret_cast<uint4 *>(v[u])) : "v"(addr[u]));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 16; u++) acc += v[u][0] ^ (W > 4 ? v[u][W / 4 - 1] : 0u);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int W>
void run(int waves, int cus, uint32_t *d, uint64_t *clk) {
  const int iters = 4000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<W>, dim3(cus), dim3(waves * 64), 0, 0, d, iters, clk);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<W>, dim3(cus), dim3(waves * 64), 0, 0, d, iters, clk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  uint64_t c[2];
  hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)c[0] / ((double)c[1] * 10.0);  // realtime = 100 MHz
  const double cyc_per_instr = W == 16 ? 4 : 2;
  const double need = (double)waves * iters * 16 * cyc_per_instr;
  const double have = ms * 1e-3 * ghz * 1e9;
  printf("b%-3d waves=%2d  %.3f ms  clk %.2f GHz  LDS util %.1f%%  B/clk/CU %.0f\n", W * 8, waves, ms, ghz,
         100.0 * need / have, (double)waves * iters * 16 * 64 * W / have);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *d;
  uint64_t *clk;
  hipMalloc(&d, 256 * 1024 * 64 * 4);
  hipMalloc(&clk, 16);
  for (int w : {4, 8, 12, 16}) run<4>(w, cus, d, clk);
  for (int w : {4, 8, 12, 16}) run<8>(w, cus, d, clk);
  for (int w : {4, 8, 12, 16}) run<16>(w, cus, d, clk);
  return 0;
}
