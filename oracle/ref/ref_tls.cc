// ref_tls.cc -- golden TLS records from the REFERENCE record-protection code
// (test infrastructure; built by oracle/ref/Makefile into oracle/_ref/ref_tls,
// never shipped in the product).
//
// For TLS 1.2 and TLS 1.3 with AES-128-GCM, AES-256-GCM and
// ChaCha20-Poly1305 it creates the reference's SSLAEADContext
// (ssl/ssl_aead_ctx.cc:44-123, compiled from /root/reference) for the seal
// direction and seals consecutive records with SSLAEADContext::SealScatter
// (ssl_aead_ctx.cc:299-381), framed as do_seal_record frames them
// (ssl/tls_record.cc:266-317: the 5-byte header with the outer type, record
// version 0x0303 and ciphertext length; TLS 1.3 seals the real type as the
// one-byte extra_in).  That function is static and needs a whole SSL
// connection, so its 20 lines of header framing are restated here; the nonce,
// AD and explicit-nonce construction and the AEAD all run in the reference's
// code.  Output: JSON on stdout, one object per (version, suite, starting
// sequence number) with every record's prefix (header || explicit nonce),
// ciphertext (hex up to 64 bytes, else its SHA-256) and suffix.
// tests/golden/make_golden.py stores it as tests/golden/ref_tls.json.
#include <openssl/sha.h>
#include <openssl/ssl.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "internal.h"  // the reference's ssl/internal.h (SSLAEADContext)

using namespace bssl;

namespace {

std::string hex(const uint8_t *p, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; i++) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

// Deterministic test bytes (tests/test_tls_golden.py restates it).
void fill(uint8_t *p, size_t n, uint32_t seed) {
  uint32_t x = seed * 2654435761u + 12345u;
  for (size_t i = 0; i < n; i++) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    p[i] = (uint8_t)(x >> 7);
  }
}

struct Suite {
  uint16_t version;
  uint16_t cipher_id;
  const char *aead;
  size_t key_len, iv_len;
};

}  // namespace

int main() {
  const Suite suites[] = {
      {TLS1_2_VERSION, 0xc02f, "aes-128-gcm", 16, 4},
      {TLS1_2_VERSION, 0xc030, "aes-256-gcm", 32, 4},
      {TLS1_2_VERSION, 0xcca8, "chacha20-poly1305", 32, 12},
      {TLS1_3_VERSION, 0x1301, "aes-128-gcm", 16, 12},
      {TLS1_3_VERSION, 0x1302, "aes-256-gcm", 32, 12},
      {TLS1_3_VERSION, 0x1303, "chacha20-poly1305", 32, 12},
  };
  const uint64_t seq_starts[] = {0, 0x1234567890ull};
  const size_t lens[] = {0, 1, 13, 15, 16, 17, 64, 255, 1350, 4096, 16383, 16384};
  const uint8_t types[] = {23, 22, 21};
  printf("[\n");
  bool first_obj = true;
  uint32_t seed = 1;
  for (const Suite &su : suites) {
    for (uint64_t seq0 : seq_starts) {
      // TLS 1.3 traffic keys start at sequence number 0 (RFC 8446 5.3): the
      // reference's tls13 AES-GCM AEAD derives its nonce mask from the first
      // nonce it sees (e_aes.cc.inc:1180-1185), so a context started at
      // seq0 != 0 rejects later records.  Only ChaCha20-Poly1305 and TLS 1.2
      // are sealed from a mid-stream sequence number.
      if (su.version >= TLS1_3_VERSION && su.iv_len == 12 &&
          strcmp(su.aead, "chacha20-poly1305") != 0 && seq0 != 0)
        continue;
      const SSL_CIPHER *cipher = SSL_get_cipher_by_value(su.cipher_id);
      if (!cipher) {
        fprintf(stderr, "no cipher %04x\n", su.cipher_id);
        return 1;
      }
      uint8_t key[32], iv[12];
      fill(key, su.key_len, seed++);
      fill(iv, su.iv_len, seed++);
      UniquePtr<SSLAEADContext> ctx = SSLAEADContext::Create(
          evp_aead_seal, su.version, cipher, Span<const uint8_t>(key, su.key_len),
          Span<const uint8_t>(), Span<const uint8_t>(iv, su.iv_len));
      if (!ctx) {
        fprintf(stderr, "SSLAEADContext::Create failed\n");
        return 1;
      }
      const bool tls13 = su.version >= TLS1_3_VERSION;
      printf("%s{\"version\": %u, \"aead\": \"%s\", \"key\": \"%s\", \"fixed_iv\": \"%s\", "
             "\"seq0\": %llu, \"records\": [\n",
             first_obj ? "" : ",\n", su.version, su.aead, hex(key, su.key_len).c_str(),
             hex(iv, su.iv_len).c_str(), (unsigned long long)seq0);
      first_obj = false;
      uint64_t seq = seq0;
      bool first_rec = true;
      for (size_t len : lens) {
        for (uint8_t type : types) {
          const uint32_t pt_seed = seed++;
          std::vector<uint8_t> in(len + 1), out(len + 1);
          fill(in.data(), len, pt_seed);
          uint8_t inner = type;
          const uint8_t *extra_in = tls13 ? &inner : nullptr;
          const size_t extra_len = tls13 ? 1 : 0;
          size_t suffix_len = 0, ct_len = 0;
          if (!ctx->SuffixLen(&suffix_len, len, extra_len) ||
              !ctx->CiphertextLen(&ct_len, len, extra_len)) {
            fprintf(stderr, "length\n");
            return 1;
          }
          const size_t explicit_len = ctx->ExplicitNonceLen();
          uint8_t prefix[5 + 16], suffix[64];
          // do_seal_record's header (tls_record.cc:288-299).
          prefix[0] = extra_len ? 23 : type;
          prefix[1] = 0x03;
          prefix[2] = 0x03;
          prefix[3] = (uint8_t)(ct_len >> 8);
          prefix[4] = (uint8_t)ct_len;
          if (!ctx->SealScatter(prefix + 5, out.data(), suffix, prefix[0], 0x0303, seq,
                                Span<const uint8_t>(prefix, 5), in.data(), len, extra_in,
                                extra_len)) {
            fprintf(stderr, "SealScatter failed\n");
            return 1;
          }
          std::string body;
          if (len <= 64) {
            body = "\"" + hex(out.data(), len) + "\"";
          } else {
            uint8_t md[32];
            SHA256(out.data(), len, md);
            body = "\"sha256:" + hex(md, 32) + "\"";
          }
          printf("%s {\"seq\": %llu, \"type\": %u, \"len\": %zu, \"pt_seed\": %u, "
                 "\"prefix\": \"%s\", \"body\": %s, \"suffix\": \"%s\"}",
                 first_rec ? "" : ",\n", (unsigned long long)seq, type, len, pt_seed,
                 hex(prefix, 5 + explicit_len).c_str(), body.c_str(),
                 hex(suffix, suffix_len).c_str());
          first_rec = false;
          seq++;
        }
      }
      printf("]}");
    }
  }
  printf("\n]\n");
  return 0;
}
