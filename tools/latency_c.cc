// Single-record latency of EVP_AEAD_CTX_seal_scatter called from C, as a
// BoringSSL caller (SSLAEADContext::SealScatter, ssl/ssl_aead_ctx.cc:299-409)
// makes it: host buffers, one record per call.  The same calls as
// tools/latency_bench.py without the Python/ctypes layer.  Prints one JSON
// line: median / p90 microseconds per call for each AEAD and record size.
//   make -C tools latency_c && tools/latency_c
#include <bssl_amd/aead.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

struct Result {
  double median_us, p90_us;
};

bool measure(const EVP_AEAD *aead, size_t size, int n, Result *r) {
  EVP_AEAD_CTX ctx;
  EVP_AEAD_CTX_zero(&ctx);
  std::vector<uint8_t> key(EVP_AEAD_key_length(aead), 0);
  if (!EVP_AEAD_CTX_init(&ctx, aead, key.data(), key.size(), EVP_AEAD_DEFAULT_TAG_LENGTH,
                         nullptr))
    return false;
  std::vector<uint8_t> pt(size, 0), out(size + 1), tag(16), ad(13, 0), nonce(12, 0);
  std::vector<double> ts;
  bool ok = true;
  for (int i = 0; i < n + 50 && ok; i++) {
    size_t tag_len = 0;
    const auto t0 = std::chrono::steady_clock::now();
    ok = EVP_AEAD_CTX_seal_scatter(&ctx, out.data(), tag.data(), &tag_len, tag.size(),
                                   nonce.data(), nonce.size(), pt.data(), pt.size(), nullptr, 0,
                                   ad.data(), ad.size()) == 1;
    const auto t1 = std::chrono::steady_clock::now();
    if (i >= 50) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  EVP_AEAD_CTX_cleanup(&ctx);
  if (!ok) return false;
  std::sort(ts.begin(), ts.end());
  r->median_us = ts[ts.size() / 2];
  r->p90_us = ts[ts.size() * 9 / 10];
  return true;
}

}  // namespace

int main() {
  struct {
    const char *name;
    const EVP_AEAD *aead;
  } aeads[] = {{"aes-128-gcm", EVP_aead_aes_128_gcm()},
               {"chacha20-poly1305", EVP_aead_chacha20_poly1305()}};
  std::printf("{\"single_record_seal_scatter_latency_c\": {");
  bool first = true;
  for (const auto &a : aeads) {
    for (size_t size : {size_t(1350), size_t(16384)}) {
      Result r;
      if (!measure(a.aead, size, 500, &r)) {
        std::fprintf(stderr, "%s/%zu: seal failed\n", a.name, size);
        return 1;
      }
      std::printf("%s\"%s/%zu\": {\"median_us\": %.1f, \"p90_us\": %.1f}", first ? "" : ", ",
                  a.name, size, r.median_us, r.p90_us);
      first = false;
    }
  }
  std::printf("}}\n");
  return 0;
}
