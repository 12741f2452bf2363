// Microbenchmark + self-check of the bitsliced AES core (csrc/bs_aes.h):
// 32 blocks per lane, AES-128.  Diagnostic tool, not product code; the
// known-answer check uses the oracle's AES (oracle/aead_oracle.c).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "bs_aes.h"
extern "C" {
#include "aead_oracle.h"
}
using namespace bssl_amd;

struct Keys { uint32_t w[11][4]; };

__device__ __forceinline__ void load_planes(const uint32_t *blk /*32 blocks x 4 words*/, uint32_t p[16][8]) {
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t m[32];
#pragma unroll
    for (int n = 0; n < 32; n++) m[n] = blk[4 * n + w];
    bs_transpose32(m);
#pragma unroll
    for (int k = 0; k < 32; k++) p[4 * w + k / 8][k % 8] = m[k];
  }
}
__device__ __forceinline__ void store_planes(uint32_t *blk, uint32_t p[16][8]) {
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t m[32];
#pragma unroll
    for (int k = 0; k < 32; k++) m[k] = p[4 * w + k / 8][k % 8];
    bs_transpose32(m);
#pragma unroll
    for (int n = 0; n < 32; n++) blk[4 * n + w] = m[n];
  }
}

__device__ __forceinline__ void encrypt(uint32_t p[16][8], const Keys &k) {
  uint32_t w0[4], w10[4];
  for (int c = 0; c < 4; c++) {
    w0[c] = k.w[0][c];
    w10[c] = k.w[10][c];
    asm volatile("" : "+s"(w0[c]), "+s"(w10[c]));  // keep the masks from being hoisted
  }
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) p[i][b] ^= bs_kmask(w0, i, b);
#pragma unroll 1
  for (int r = 1; r < 10; r++) {
    uint32_t w[4];
    for (int c = 0; c < 4; c++) w[c] = __builtin_amdgcn_readfirstlane(k.w[r][c]);
    bs_round(p, w);
  }
  bs_last_round(p, w10);
}

// Known-answer mode: one lane per 32 blocks, in -> out.
__global__ __launch_bounds__(64) void kat(const uint32_t *in, uint32_t *out, Keys k) {
  uint32_t p[16][8];
  load_planes(in + threadIdx.x * 128, p);
  encrypt(p, k);
  store_planes(out + threadIdx.x * 128, p);
}

// Throughput mode: iters encryptions per lane, state fed back.
__global__ __launch_bounds__(256) void thr(uint32_t *out, Keys k, int iters) {
  uint32_t p[16][8];
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) p[i][b] = (threadIdx.x + 1) * 0x9E3779B9u * (i * 8 + b + 1);
  for (int it = 0; it < iters; it++) encrypt(p, k);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc ^= p[i][b];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static uint8_t sb[256];
static void host_expand(const uint8_t key[16], Keys &k) {
  // S-box from the oracle: S[x] = AES_K=0-independent -> compute via GF inverse.
  auto mul = [](uint8_t a, uint8_t b) { uint8_t p = 0; for (int i = 0; i < 8; i++) { if (b & 1) p ^= a; a = (a << 1) ^ ((a & 0x80) ? 0x1b : 0); b >>= 1; } return p; };
  for (int x = 0; x < 256; x++) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; y++) if (mul(x, y) == 1) { inv = y; break; }
    uint8_t s = inv, r = inv;
    for (int i = 0; i < 4; i++) { r = (r << 1) | (r >> 7); s ^= r; }
    sb[x] = s ^ 0x63;
  }
  uint8_t w[176];
  memcpy(w, key, 16);
  uint8_t rcon = 1;
  for (int i = 16; i < 176; i += 4) {
    uint8_t t[4] = {w[i - 4], w[i - 3], w[i - 2], w[i - 1]};
    if (i % 16 == 0) {
      uint8_t u = t[0]; t[0] = sb[t[1]] ^ rcon; t[1] = sb[t[2]]; t[2] = sb[t[3]]; t[3] = sb[u];
      rcon = mul(rcon, 2);
    }
    for (int j = 0; j < 4; j++) w[i + j] = w[i - 16 + j] ^ t[j];
  }
  for (int r = 0; r < 11; r++)
    for (int c = 0; c < 4; c++) memcpy(&k.w[r][c], w + 16 * r + 4 * c, 4);
}

int main() {
  uint8_t key[16];
  for (int i = 0; i < 16; i++) key[i] = i * 17 + 3;
  Keys k;
  host_expand(key, k);
  const int lanes = 64, nblk = lanes * 32;
  std::vector<uint8_t> pt(nblk * 16), ct(nblk * 16);
  for (size_t i = 0; i < pt.size(); i++) pt[i] = (uint8_t)(i * 131 + 7);
  uint32_t *din, *dout;
  hipMalloc(&din, pt.size());
  hipMalloc(&dout, pt.size());
  hipMemcpy(din, pt.data(), pt.size(), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kat, dim3(1), dim3(lanes), 0, 0, din, dout, k);
  hipMemcpy(ct.data(), dout, ct.size(), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int b = 0; b < nblk; b++) {
    uint8_t ref[16];
    oracle_aes_encrypt_block(key, 16, pt.data() + 16 * b, ref);
    if (memcmp(ref, ct.data() + 16 * b, 16)) bad++;
  }
  printf("KAT: %d/%d blocks mismatch\n", bad, nblk);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *dsink;
  hipMalloc(&dsink, 64 << 20);
  for (int wpc : {4, 8, 12, 16}) {
    const int iters = 200, threads = 256, grid = cus * wpc / 4;
    hipLaunchKernelGGL(thr, dim3(grid), dim3(threads), 0, 0, dsink, k, 2);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(thr, dim3(grid), dim3(threads), 0, 0, dsink, k, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double blocks = (double)grid * threads * 32 * iters;
    printf("waves/CU=%2d: %.3f ms, %.3g blocks/s = %.1f GiB/s keystream, %.2f blocks/ns/CU\n", wpc, ms,
           blocks / (ms * 1e-3), blocks * 16 / (ms * 1e-3) / (1 << 30), blocks / (ms * 1e6) / cus);
  }
  return bad != 0;
}
