// tls_records.hip -- per-record inputs of the TLS record layer, built on the
// device for a batch of records of one connection direction.
//
// Reference (one record per call): do_seal_record (ssl/tls_record.cc:266-317)
// writes the 5-byte header (TLS 1.3: outer type application_data, the real
// type sealed as `extra_in`), then SSLAEADContext::SealScatter
// (ssl/ssl_aead_ctx.cc:299-380) forms the nonce -- TLS 1.2 AES-GCM: 4-byte
// fixed IV || be64(seq), the 8 explicit bytes also written after the header;
// TLS 1.3 and TLS 1.2 ChaCha20-Poly1305: fixed_iv XOR (0^4 || be64(seq)) --
// and the additional data (GetAdditionalData, :207-224): TLS 1.2
// be64(seq) || type || version || be16(plaintext length), TLS 1.3 the header.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace bssl_amd {
namespace {

__global__ void tls_prepare_kernel(TlsPrepare p) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t len = p.lengths ? p.lengths[i] : p.record_len;
  const uint64_t seq = p.seq + i;
  uint8_t *pre = p.prefix + p.prefix_len * i;
  // Seal: the caller's type; open: the received header's (tls_record.cc:197-235).
  const uint8_t type = p.open ? pre[0] : p.types ? p.types[i] : p.type;
  // Nonce (ssl_aead_ctx.cc:326-365 seal, 248-279 open).
  uint8_t *nonce = p.nonces + 12 * i;
  for (int k = 0; k < 12; k++) {
    const uint8_t sb = k >= 4 ? (uint8_t)(seq >> (8 * (11 - k))) : 0;
    uint8_t v;
    if (p.xor_nonce)
      v = (uint8_t)(p.fixed_iv[k] ^ sb);
    else if (k < 4)
      v = p.fixed_iv[k];
    else
      v = p.open ? pre[5 + (k - 4)] : sb;  // the explicit nonce travels in the record
    nonce[k] = v;
  }
  // Header (seal): ciphertext length = explicit nonce + plaintext + extra + tag.
  uint8_t hdr[5];
  if (p.open) {
    for (int k = 0; k < 5; k++) hdr[k] = pre[k];
  } else {
    const uint64_t ctlen = p.explicit_len + len + p.extra_len + p.tag_len;
    hdr[0] = p.tls13 ? (uint8_t)23 : type;  // SSL3_RT_APPLICATION_DATA outside in TLS 1.3
    hdr[1] = (uint8_t)(p.record_version >> 8);
    hdr[2] = (uint8_t)p.record_version;
    hdr[3] = (uint8_t)(ctlen >> 8);
    hdr[4] = (uint8_t)ctlen;
    for (int k = 0; k < 5; k++) pre[k] = hdr[k];
    for (uint32_t k = 0; k < p.explicit_len; k++) pre[5 + k] = nonce[4 + k];
  }
  // Additional data (GetAdditionalData, ssl_aead_ctx.cc:207-224).
  uint8_t *ad = p.ad + p.ad_stride * i;
  if (p.tls13) {
    for (int k = 0; k < 5; k++) ad[k] = hdr[k];
  } else {
    for (int k = 0; k < 8; k++) ad[k] = (uint8_t)(seq >> (8 * (7 - k)));
    ad[8] = type;
    ad[9] = hdr[1];
    ad[10] = hdr[2];
    ad[11] = (uint8_t)(len >> 8);
    ad[12] = (uint8_t)len;
  }
  if (p.tls13 && !p.open) p.extra[i] = type;  // the inner content type (tls_record.cc:272-276)
  // Plaintext records are at most 2^14 bytes (SSL3_RT_MAX_PLAIN_LENGTH); a
  // longer one fails like a rejected call.
  if (len > 16384) p.valid[i] = 0;
}

}  // namespace

int launch_tls_prepare(const TlsPrepare &p, void *stream) {
  if (p.n == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(tls_prepare_kernel, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace bssl_amd
