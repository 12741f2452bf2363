// FETCH_SIZE / WRITE_SIZE calibration for the record access patterns of the
// AEAD kernels (MI355X_MICROARCH.md, HBM section: only 16 B/lane streaming
// reads and stores are calibrated; other widths must be calibrated on a known
// byte count).  Each kernel copies the same records (1M x 1350 B at a 1360-byte
// stride, plus a 16-byte tag per record) with a different lane pattern:
//   copy_stream  : 16 B per lane, consecutive lanes consecutive 16 B chunks
//                  over the whole padded buffer (the guide's calibrated case)
//   copy_chacha  : chacha.hip's pattern: 4 lanes per record, lane q moves
//                  64-byte block 4*it+q as four 16-byte loads / stores
//   copy_quad    : same bytes, transposed: store k of lane q is chunk q of
//                  block 4*it+k (each instruction covers 64 contiguous bytes
//                  per record)
//   copy_gcm     : gcm.hip's pattern: 16 lanes per record, lane q moves
//                  16-byte block 16*it+q (256 contiguous bytes per record)
//   copy_gcm8    : the same at 8 lanes per record (128-byte runs: the
//                  T-table kernel's L = 8 of configs 2 and 4)
//   (copy_quad is the L = 4 pattern: 64-byte runs, config G)
//   copy_quad_slow_t: copy_quad_slow with temporal loads (the T-table
//                  kernel's 4-lane loads since late round 6)
//   copy_quad_slow: copy_quad with the T-table kernel's pacing at L = 4 --
//                  non-temporal loads, and ~4 us (s_sleep) between a record's
//                  iterations, as the kernel spends an iteration of AES and
//                  GHASH between a record's consecutive 64-byte runs (config
//                  G: ~4.5 us), so the two halves of a 128-byte line are
//                  requested apart in time instead of back to back
//                  (does the counter count such a stream
//                  like the fast copy's?)
// Known bytes per launch: read = write = records * 1350 (+ tags written).
// Build: hipcc --offload-arch=gfx950 -O3 -o calib_copy calib_copy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

struct Geo {
  uint64_t recs, len, stride;
};

// Tail of a record: dword copies of the last (len % 16) bytes' 16-byte chunk.
__device__ __forceinline__ void copy_tail(const uint8_t *s, uint8_t *d, uint32_t n) {
  for (uint32_t i = 0; i + 4 <= n; i += 4)
    *reinterpret_cast<uint32_t *>(d + i) = *reinterpret_cast<const uint32_t *>(s + i);
  const uint32_t r = n & ~3u;
  if (n & 2) *reinterpret_cast<uint16_t *>(d + r) = *reinterpret_cast<const uint16_t *>(s + r);
  if (n & 1) d[n - 1] = s[n - 1];
}

__global__ __launch_bounds__(256) void copy_stream(const uint4 *s, uint4 *d, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) d[i] = s[i];
}

template <int MODE>  // 0 chacha, 1 quad, 2 quad paced like the kernel, 3 the same with temporal loads
__global__ __launch_bounds__(256) void copy_rec4(const uint8_t *s, uint8_t *d, uint8_t *tags, Geo g) {
  const uint64_t rec = (blockIdx.x * 256ull + threadIdx.x) / 4;
  const int q = threadIdx.x & 3;
  if (rec >= g.recs) return;
  const uint64_t kLen = g.len;
  const uint8_t *sp = s + rec * g.stride;
  uint8_t *dp = d + rec * g.stride;
  const uint32_t kFull = (uint32_t)(kLen / 64);
  for (uint32_t it = 0; it * 4 < kFull + 1; it++) {
    const uint32_t blk = it * 4 + q;
    if (MODE == 0) {
      if (blk < kFull) {
        const uint4 *a = reinterpret_cast<const uint4 *>(sp + 64 * blk);
        uint4 v[4];
        for (int k = 0; k < 4; k++) v[k] = a[k];
        uint4 *b = reinterpret_cast<uint4 *>(dp + 64 * blk);
        for (int k = 0; k < 4; k++) b[k] = v[k];
      } else if (blk == kFull && kLen > 64ull * kFull) {
        copy_tail(sp + 64 * blk, dp + 64 * blk, (uint32_t)(kLen - 64 * kFull));
      }
    } else {
      uint4 v[4];
      for (int k = 0; k < 4; k++) {
        const uint32_t bk = it * 4 + k;
        if (bk < kFull) {
          const uint4 *a = reinterpret_cast<const uint4 *>(sp + 64 * bk) + q;
          if (MODE == 2) {  // (non-temporal, as the kernel's load_blk_nt until round 6)
            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
            const u4 x = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(a));
            v[k] = make_uint4(x.x, x.y, x.z, x.w);
          } else {
            v[k] = *a;
          }
        }
      }
      if (MODE >= 2) __builtin_amdgcn_s_sleep(127);
      for (int k = 0; k < 4; k++) {
        const uint32_t bk = it * 4 + k;
        if (bk < kFull) reinterpret_cast<uint4 *>(dp + 64 * bk)[q] = v[k];
        else if (bk == kFull && q == 0 && kLen > 64ull * kFull)
          copy_tail(sp + 64 * bk, dp + 64 * bk, (uint32_t)(kLen - 64 * kFull));
      }
    }
  }
  if (q == 0) reinterpret_cast<uint4 *>(tags)[rec] = make_uint4(rec, 1, 2, 3);
}

template <int LN>  // lanes per record
__global__ __launch_bounds__(256) void copy_gcm(const uint8_t *s, uint8_t *d, uint8_t *tags, Geo g) {
  const uint64_t rec = (blockIdx.x * 256ull + threadIdx.x) / LN;
  const int q = threadIdx.x & (LN - 1);
  if (rec >= g.recs) return;
  const uint64_t kLen = g.len;
  const uint8_t *sp = s + rec * g.stride;
  uint8_t *dp = d + rec * g.stride;
  const uint32_t kFull = (uint32_t)(kLen / 16);
  for (uint32_t j = q; j <= kFull; j += LN) {
    if (j < kFull) reinterpret_cast<uint4 *>(dp)[j] = reinterpret_cast<const uint4 *>(sp)[j];
    else if (kLen > 16ull * kFull) copy_tail(sp + 16 * j, dp + 16 * j, (uint32_t)(kLen - 16 * kFull));
  }
  if (q == 0) reinterpret_cast<uint4 *>(tags)[rec] = make_uint4(rec, 1, 2, 3);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  Geo g{argc > 4 ? strtoull(argv[4], nullptr, 10) : (1ull << 20),
        argc > 2 ? strtoull(argv[2], nullptr, 10) : 1350,
        argc > 3 ? strtoull(argv[3], nullptr, 10) : 1360};
  const uint64_t kRecs = g.recs, kLen = g.len;
  const uint64_t bytes = g.recs * g.stride;
  uint8_t *s, *d, *t;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&t, kRecs * 16));
  CK(hipMemset(s, 0x5a, bytes));
  CK(hipMemset(d, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[7] = {"copy_stream", "copy_chacha", "copy_quad", "copy_gcm", "copy_gcm8",
                          "copy_quad_slow", "copy_quad_slow_t"};
  for (int v = 0; v < 7; v++) {
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
      CK(hipEventRecord(e0));
      if (v == 0) copy_stream<<<8192, 256>>>((const uint4 *)s, (uint4 *)d, bytes / 16);
      if (v == 1) copy_rec4<0><<<(unsigned)((kRecs * 4 + 255) / 256), 256>>>(s, d, t, g);
      if (v == 2) copy_rec4<1><<<(unsigned)((kRecs * 4 + 255) / 256), 256>>>(s, d, t, g);
      if (v == 3) copy_gcm<16><<<(unsigned)((kRecs * 16 + 255) / 256), 256>>>(s, d, t, g);
      if (v == 4) copy_gcm<8><<<(unsigned)((kRecs * 8 + 255) / 256), 256>>>(s, d, t, g);
      if (v == 5) copy_rec4<2><<<(unsigned)((kRecs * 4 + 255) / 256), 256>>>(s, d, t, g);
      if (v == 6) copy_rec4<3><<<(unsigned)((kRecs * 4 + 255) / 256), 256>>>(s, d, t, g);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double moved = v == 0 ? 2.0 * bytes : 2.0 * kRecs * kLen + 16.0 * kRecs;
    printf("%-12s best %.3f ms  %.0f GB/s (known bytes read %.0f write %.0f)\n", names[v], best,
           moved / best / 1e6, v == 0 ? (double)bytes : (double)kRecs * kLen,
           v == 0 ? (double)bytes : kRecs * kLen + 16.0 * kRecs);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
