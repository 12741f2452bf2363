// iovec.hip -- EVP_AEAD_CTX_sealv / _openv_detached over device batches of
// non-contiguous records.
//
// Reference: EVP_AEAD_CTX_sealv / _openv_detached (crypto/fipsmodule/cipher/
// aead.cc.inc:316-361, 531-584) take one record as an array of CRYPTO_IOVEC
// {out, in, len} chunks and its AD as an array of CRYPTO_IVEC {in, len}
// (include/openssl/aead.h:400-414); the AEADs walk the chunks with
// bssl::iovec::ForEachBlockRange (crypto/cipher/internal.h:283-411), i.e. the
// record is the concatenation of its chunks.
//
// AES-GCM (round 3): the bulk kernels walk the chunks in place
// (BatchDesc::iovecs, gcm.hip IOV): each lane keeps a cursor on the chunk of
// its current block and loads / stores 16-byte blocks at any alignment;
// only the per-record totals are computed here (iov_lengths), with no
// staging, copies or stream synchronisation.
//
// ChaCha20-Poly1305, XChaCha20-Poly1305 and AES-GCM-SIV: the chunks are
// gathered into one contiguous device staging area (records 16-byte aligned,
// so the bulk kernels take their aligned fast path), sealed or opened in place
// by the same bulk kernels as any batch, and scattered back to the chunks'
// `out` pointers.  A failed record is zero-filled in the staging area by the
// bulk kernel, so the scatter zeroes its chunks (clear_iovec,
// aead.cc.inc:310-314, 325-333).  Copies: one wave per record walks its
// chunks in order; each chunk is copied in aligned 16-byte destination words
// loaded by one dwordx4 at any source alignment, with a byte loop for the
// head and tail.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "internal.h"

namespace bssl_amd {
namespace {

constexpr int kCopyThreads = 256;

// dst[0, n) = src[0, n) for one chunk, by the 64 lanes of one wave.
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  // Head: bytes until dst is 16-byte aligned.
  const uint64_t head = min<uint64_t>(n, (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
  if (lane < head) dst[lane] = src[lane];
  const uint64_t words = (n - head) / 16;
  uint4 *d = reinterpret_cast<uint4 *>(dst + head);
  // Source words at any alignment: one dwordx4 each (the shader memory runs
  // in unaligned mode; the loads stay inside the chunk).
  typedef uint32_t u32_any __attribute__((aligned(1)));
  const u32_any *sp = reinterpret_cast<const u32_any *>(src + head);
  for (uint64_t w = lane; w < words; w += 64)
    d[w] = make_uint4(sp[4 * w], sp[4 * w + 1], sp[4 * w + 2], sp[4 * w + 3]);
  for (uint64_t i = head + 16 * words + lane; i < n; i += 64) dst[i] = src[i];
}

// Per record: message and AD lengths, and their 16-byte padded sizes for the
// staging layout.
__global__ void iov_lengths(const IovBatchDesc b, uint64_t *__restrict__ len,
                            uint64_t *__restrict__ padded, uint64_t *__restrict__ ad_len,
                            uint64_t *__restrict__ ad_padded) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.num_records) return;
  uint64_t t = 0, a = 0;
  for (uint64_t c = b.iovec_start[i]; c < b.iovec_start[i + 1]; c++) t += b.iovecs[c].len;
  if (b.aadvecs)
    for (uint64_t c = b.aadvec_start[i]; c < b.aadvec_start[i + 1]; c++) a += b.aadvecs[c].len;
  len[i] = t;
  padded[i] = (t + 15) & ~uint64_t(15);
  ad_len[i] = a;
  ad_padded[i] = (a + 15) & ~uint64_t(15);
}

// Gather (TO_STAGE) or scatter (!TO_STAGE) the chunks of records: one wave
// per record, grid-stride over the batch.
template <bool TO_STAGE>
__global__ __launch_bounds__(kCopyThreads) void iov_copy(const IovBatchDesc b,
                                                         uint8_t *__restrict__ stage,
                                                         const uint64_t *__restrict__ off,
                                                         uint8_t *__restrict__ ad_stage,
                                                         const uint64_t *__restrict__ ad_off) {
  constexpr uint32_t kWaves = kCopyThreads / 64;
  for (uint64_t i = (uint64_t)blockIdx.x * kWaves + threadIdx.x / 64; i < b.num_records;
       i += (uint64_t)gridDim.x * kWaves) {
    uint64_t pos = off[i];
    for (uint64_t c = b.iovec_start[i]; c < b.iovec_start[i + 1]; c++) {
      const IovecDev v = b.iovecs[c];
      if (TO_STAGE)
        copy_bytes(stage + pos, v.in, v.len);
      else
        copy_bytes(v.out, stage + pos, v.len);
      pos += v.len;
    }
    if (TO_STAGE && b.aadvecs) {
      uint64_t apos = ad_off[i];
      for (uint64_t c = b.aadvec_start[i]; c < b.aadvec_start[i + 1]; c++) {
        const IvecDev v = b.aadvecs[c];
        copy_bytes(ad_stage + apos, v.in, v.len);
        apos += v.len;
      }
    }
  }
}

// In-place form (AES-GCM): only the per-record totals are computed; the bulk
// kernels read and write the chunks themselves (BatchDesc::iovecs).  No
// staging, no copies, no synchronisation.
int iov_batch_run_in_place(const IovBatchDesc &b, const IovRunner &run, hipStream_t s) {
  const uint64_t n = b.num_records;
  uint64_t *meta = nullptr;  // len, padded, ad_len, ad_padded (n each)
  if (hipMallocAsync(reinterpret_cast<void **>(&meta), 4 * n * 8 + 64, s) != hipSuccess) return 2;
  uint64_t *len = meta, *padded = meta + n, *ad_len = meta + 2 * n, *ad_padded = meta + 3 * n;
  hipLaunchKernelGGL(iov_lengths, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, len,
                     padded, ad_len, ad_padded);
  BatchDesc d = {};
  d.lengths = len;
  d.ad_lengths = ad_len;
  d.nonces = b.nonces;
  d.nonce_len = b.nonce_len;
  d.tags = b.tags;
  d.status = b.status;
  d.num_records = n;
  d.iovecs = b.iovecs;
  d.iovec_start = b.iovec_start;
  d.aadvecs = b.aadvecs;
  d.aadvec_start = b.aadvec_start;
  int rc = run(d);
  hipFreeAsync(meta, s);
  if (!rc && hipGetLastError() != hipSuccess) rc = 1;
  return rc;
}

}  // namespace

int iov_batch_run(const IovBatchDesc &b, const IovRunner &run, void *stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint64_t n = b.num_records;
  if (n == 0) return 0;
  if (run.in_place()) return iov_batch_run_in_place(b, run, s);
  size_t temp = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (const uint64_t *)nullptr,
                                       (uint64_t *)nullptr, n + 1, s) != hipSuccess)
    return 1;
  // len, padded (n+1, last = 0), off (n+1), ad_len, ad_padded (n+1), ad_off (n+1)
  const size_t words = 6 * (n + 1) + 2;
  uint8_t *meta = nullptr;
  if (hipMallocAsync(reinterpret_cast<void **>(&meta), words * 8 + temp, s) != hipSuccess) return 2;
  uint64_t *len = reinterpret_cast<uint64_t *>(meta);
  uint64_t *padded = len + (n + 1);
  uint64_t *off = padded + (n + 1);
  uint64_t *ad_len = off + (n + 1);
  uint64_t *ad_padded = ad_len + (n + 1);
  uint64_t *ad_off = ad_padded + (n + 1);
  void *d_temp = meta + words * 8;
  int rc = 0;
  if (hipMemsetAsync(padded + n, 0, 8, s) != hipSuccess ||
      hipMemsetAsync(ad_padded + n, 0, 8, s) != hipSuccess)
    rc = 1;
  if (!rc) {
    hipLaunchKernelGGL(iov_lengths, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, len,
                       padded, ad_len, ad_padded);
    if (hipcub::DeviceScan::ExclusiveSum(d_temp, temp, padded, off, n + 1, s) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(d_temp, temp, ad_padded, ad_off, n + 1, s) !=
            hipSuccess)
      rc = 1;
  }
  // The staging size is known only on the device: read the two totals back
  // (this synchronises the stream once per batch).
  uint64_t totals[2] = {0, 0};
  if (!rc && (hipMemcpyAsync(&totals[0], off + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipMemcpyAsync(&totals[1], ad_off + n, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
    rc = 1;
  uint8_t *stage = nullptr;
  if (!rc && hipMallocAsync(reinterpret_cast<void **>(&stage), totals[0] + totals[1] + 16, s) !=
                 hipSuccess)
    rc = 2;
  if (!rc) {
    uint8_t *ad_stage = stage + totals[0];
    const uint64_t wgs = (n + 3) / 4;  // 4 records (waves) per workgroup
    const unsigned grid = (unsigned)(wgs < 65536 ? wgs : 65536);
    hipLaunchKernelGGL(iov_copy<true>, dim3(grid), dim3(kCopyThreads), 0, s, b, stage, off,
                       ad_stage, ad_off);
    BatchDesc d = {};
    d.in = stage;
    d.out = stage;
    d.offsets = off;
    d.lengths = len;
    d.nonces = b.nonces;
    d.nonce_len = b.nonce_len;
    d.ad = ad_stage;
    d.ad_offsets = ad_off;
    d.ad_lengths = ad_len;
    d.tags = b.tags;
    d.status = b.status;
    d.num_records = n;
    rc = run(d);
    if (!rc)
      hipLaunchKernelGGL(iov_copy<false>, dim3(grid), dim3(kCopyThreads), 0, s, b, stage, off,
                         ad_stage, ad_off);
    hipFreeAsync(stage, s);
  }
  hipFreeAsync(meta, s);
  if (!rc && hipGetLastError() != hipSuccess) rc = 1;
  return rc;
}

}  // namespace bssl_amd
