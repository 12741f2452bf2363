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
// Round 3: every AEAD's bulk kernels walk the chunks in place
// (BatchDesc::iovecs; gcm.hip, chacha.hip, gcm_siv.hip with IOV = true and
// the per-lane cursors of iov_dev.h): each lane loads and stores its blocks
// at any alignment inside a chunk and splits the blocks that straddle chunks.
// This file only computes the per-record totals (iov_lengths): no staging,
// no copies, no stream synchronisation.  (Rounds 1-2 gathered the chunks
// into a staging area and scattered them back: two extra HBM passes.)
#include <hip/hip_runtime.h>

#include "internal.h"

namespace bssl_amd {
namespace {

// Per record: message and AD lengths (the sums of its chunks).
__global__ void iov_lengths(const IovBatchDesc b, uint64_t *__restrict__ len,
                            uint64_t *__restrict__ ad_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.num_records) return;
  uint64_t t = 0, a = 0;
  for (uint64_t c = b.iovec_start[i]; c < b.iovec_start[i + 1]; c++) t += b.iovecs[c].len;
  if (b.aadvecs)
    for (uint64_t c = b.aadvec_start[i]; c < b.aadvec_start[i + 1]; c++) a += b.aadvecs[c].len;
  len[i] = t;
  ad_len[i] = a;
}

}  // namespace

int iov_batch_run(const IovBatchDesc &b, const IovRunner &run, void *stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint64_t n = b.num_records;
  if (n == 0) return 0;
  uint64_t *meta = nullptr;  // len, ad_len (n each)
  if (hipMallocAsync(reinterpret_cast<void **>(&meta), 2 * n * 8 + 64, s) != hipSuccess) return 2;
  uint64_t *len = meta, *ad_len = meta + n;
  hipLaunchKernelGGL(iov_lengths, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, len,
                     ad_len);
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

}  // namespace bssl_amd
