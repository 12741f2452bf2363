// ref_tool.cc -- drives the REFERENCE library (compiled from /root/reference by
// oracle/ref/Makefile) to produce golden vectors and the CPU baseline.
//
// TEST/BENCH INFRASTRUCTURE ONLY.  This is our own harness; it calls the
// reference's public EVP_AEAD API (include/openssl/aead.h) exactly the way
// bench/aead.cc:41-133 does (EVP_AEAD_CTX_init_with_direction, then
// EVP_AEAD_CTX_seal_scatter with a 13-byte AD).
//
//   ref_tool edge                          edge-case vectors (JSON, stdout)
//   ref_tool digest AEAD NKEYS RPK LEN [T] batch digests over the synthetic
//                                          workload (oracle/synth.h); LEN is a
//                                          byte count or "mixed"
//   ref_tool shard AEAD LEN FIRST N RPK [T]  digest of records [FIRST,
//                                          FIRST+N) (one bench rank's shard;
//                                          key i/RPK, RPK = 0: one key)
//   ref_tool bench AEAD LEN NREC T SECS    CPU baseline: T threads seal a
//                                          resident sample of NREC synthetic
//                                          records for about SECS seconds
//   ref_tool bench1 AEAD seal|open LEN SECS  one thread, exactly BM_SpeedAEAD
//                                          (bench/aead.cc:41-133): zero key,
//                                          nonce, 13-byte AD and input, one
//                                          16-byte-aligned buffer resealed
//                                          (reopened) for about SECS seconds
#include <openssl/aead.h>
#include <openssl/sha.h>
#include <omp.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "synth.h"

namespace {

const EVP_AEAD *aead_by_name(const std::string &n, size_t *key_len) {
  if (n == "aes-128-gcm") { *key_len = 16; return EVP_aead_aes_128_gcm(); }
  if (n == "aes-192-gcm") { *key_len = 24; return EVP_aead_aes_192_gcm(); }
  if (n == "aes-256-gcm") { *key_len = 32; return EVP_aead_aes_256_gcm(); }
  if (n == "chacha20-poly1305") { *key_len = 32; return EVP_aead_chacha20_poly1305(); }
  if (n == "xchacha20-poly1305") { *key_len = 32; return EVP_aead_xchacha20_poly1305(); }
  if (n == "aes-128-gcm-siv") { *key_len = 16; return EVP_aead_aes_128_gcm_siv(); }
  if (n == "aes-256-gcm-siv") { *key_len = 32; return EVP_aead_aes_256_gcm_siv(); }
  fprintf(stderr, "unknown aead %s\n", n.c_str());
  exit(2);
}

std::string hex(const uint8_t *p, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

void fill_stream(uint64_t seed, uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; i++)
    p[i] = (uint8_t)(synth_splitmix(seed * 0x10001 + i / 8) >> (8 * (i % 8)));
}

int cmd_edge() {
  const char *names[] = {"aes-128-gcm", "aes-192-gcm", "aes-256-gcm", "chacha20-poly1305"};
  const size_t lens[] = {0, 1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129,
                         255, 256, 257, 1000, 1023, 1024, 1025, 1350, 4095, 4096,
                         4097, 16383, 16384, 16385};
  const size_t ad_lens[] = {0, 1, 13, 15, 16, 17, 31, 64, 100, 1000, 4097};
  const size_t gcm_nonce_lens[] = {1, 8, 12, 15, 16, 17, 60, 128, 1024};
  const size_t tag_lens[] = {1, 4, 8, 12, 13, 15, 16};
  printf("[\n");
  bool first = true;
  uint64_t seed = 1000;
  for (const char *name : names) {
    size_t key_len;
    const EVP_AEAD *aead = aead_by_name(name, &key_len);
    bool gcm = std::string(name) != "chacha20-poly1305";
    struct Case { size_t len, ad, nonce, tag; };
    std::vector<Case> cases;
    for (size_t l : lens) cases.push_back({l, 13, 12, 16});
    if (std::string(name) == "aes-128-gcm") cases.push_back({65543, 13, 12, 16});
    for (size_t a : ad_lens) cases.push_back({100, a, 12, 16});
    for (size_t a : ad_lens) cases.push_back({1350, a, 12, 16});
    for (size_t t : tag_lens) cases.push_back({333, 13, 12, t});
    if (gcm)
      for (size_t nl : gcm_nonce_lens) {
        cases.push_back({100, 13, nl, 16});
        cases.push_back({4097, 20, nl, 16});
      }
    for (const Case &c : cases) {
      seed++;
      std::vector<uint8_t> key(key_len), nonce(c.nonce), ad(c.ad), pt(c.len),
          ct(c.len + 1), tag(16);
      fill_stream(seed * 4 + 0, key.data(), key.size());
      fill_stream(seed * 4 + 1, nonce.data(), nonce.size());
      fill_stream(seed * 4 + 2, ad.data(), ad.size());
      fill_stream(seed * 4 + 3, pt.data(), pt.size());
      bssl::ScopedEVP_AEAD_CTX ctx;
      if (!EVP_AEAD_CTX_init(ctx.get(), aead, key.data(), key.size(), c.tag, nullptr)) return 1;
      size_t tag_out = 0;
      if (!EVP_AEAD_CTX_seal_scatter(ctx.get(), ct.data(), tag.data(), &tag_out, tag.size(),
                                     nonce.data(), nonce.size(), pt.data(), pt.size(),
                                     nullptr, 0, ad.data(), ad.size()))
        return 1;
      printf("%s{\"aead\": \"%s\", \"key\": \"%s\", \"nonce\": \"%s\", \"ad\": \"%s\", "
             "\"pt\": \"%s\", \"ct\": \"%s\", \"tag\": \"%s\"}",
             first ? "" : ",\n", name, hex(key.data(), key.size()).c_str(),
             hex(nonce.data(), nonce.size()).c_str(), hex(ad.data(), ad.size()).c_str(),
             hex(pt.data(), pt.size()).c_str(), hex(ct.data(), c.len).c_str(),
             hex(tag.data(), tag_out).c_str());
      first = false;
    }
  }
  printf("\n]\n");
  return 0;
}

// Digest definitions (mirrored by tests/golden_digest.py):
//   tags_sha256 = SHA-256(tag_0 || tag_1 || ... )
//   ct_sha256   = SHA-256(SHA-256(ct of records [0,1024)) || SHA-256(ct of
//                 records [1024,2048)) || ...)   ("checksum of checksums")
// Synthetic nonce of record i: synth_nonce(i) (12 bytes) and, for 24-byte
// (XChaCha20-Poly1305) nonces, synth_nonce(i) again with bytes 4..11 XOR 0xff
// (= synth_nonce(~i)).
size_t make_nonce(uint64_t i, size_t nonce_len, uint8_t *out) {
  synth_nonce(i, out);
  if (nonce_len == 24) {
    memcpy(out + 12, out, 12);
    for (int b = 4; b < 12; b++) out[12 + b] ^= 0xff;
  }
  return nonce_len;
}

// Digest of the records [first, first + n) of the synthetic sequence: record
// i is sealed under key (rpk ? i / rpk : 0) with len (mixed ? synth_mixed_len(i)
// : fixed_len), nonce make_nonce(i) and AD synth_ad(i, len) -- exactly what
// rank r of `bench.py --gpus N` seals for its shard (bench.shard_plan), so a
// shard's digest is defined independently of which process sealed it.  Chunks
// of 1024 records count from `first`.
int digest_range(const char *name, uint64_t first, uint64_t n, uint64_t rpk, const char *len_arg,
                 int threads, const char *extra_json) {
  size_t key_len;
  const EVP_AEAD *aead = aead_by_name(name, &key_len);
  bool mixed = std::string(len_arg) == "mixed";
  uint64_t fixed_len = mixed ? 0 : strtoull(len_arg, nullptr, 0);
  const uint64_t kChunk = 1024;
  uint64_t nchunks = (n + kChunk - 1) / kChunk;
  std::vector<uint8_t> tags(n * 16);
  std::vector<uint8_t> chunk_digests(nchunks * 32);
  uint64_t total_bytes = 0;
#pragma omp parallel num_threads(threads) reduction(+ : total_bytes)
  {
    std::vector<uint8_t> pt, ct;
    bssl::ScopedEVP_AEAD_CTX ctx;
    uint64_t cur_key = UINT64_MAX;
#pragma omp for schedule(dynamic, 1)
    for (long long c = 0; c < (long long)nchunks; c++) {
      SHA256_CTX sha;
      SHA256_Init(&sha);
      uint64_t lo = c * kChunk, hi = lo + kChunk < n ? lo + kChunk : n;
      for (uint64_t j = lo; j < hi; j++) {
        const uint64_t i = first + j;
        uint64_t k = rpk ? i / rpk : 0;
        if (k != cur_key) {
          std::vector<uint8_t> key(key_len);
          synth_key(k, key_len, key.data());
          ctx.Reset();
          if (!EVP_AEAD_CTX_init(ctx.get(), aead, key.data(), key_len, 16, nullptr)) abort();
          cur_key = k;
        }
        uint64_t len = mixed ? synth_mixed_len(i) : fixed_len;
        pt.resize(len + 1);
        ct.resize(len + 1);
        synth_pt(i, len, pt.data());
        uint8_t nonce[24], ad[13];
        const size_t nl = make_nonce(i, EVP_AEAD_nonce_length(aead), nonce);
        synth_ad(i, len, ad);
        size_t tag_out = 0;
        if (!EVP_AEAD_CTX_seal_scatter(ctx.get(), ct.data(), &tags[16 * j], &tag_out, 16, nonce,
                                       nl, pt.data(), len, nullptr, 0, ad, 13))
          abort();
        SHA256_Update(&sha, ct.data(), len);
        total_bytes += len;
      }
      SHA256_Final(&chunk_digests[32 * c], &sha);
    }
  }
  uint8_t tags_d[32], ct_d[32];
  SHA256(tags.data(), tags.size(), tags_d);
  SHA256(chunk_digests.data(), chunk_digests.size(), ct_d);
  printf("{\"aead\": \"%s\", %s\"len\": \"%s\", \"records\": %llu, \"bytes\": %llu, "
         "\"tags_sha256\": \"%s\", \"ct_sha256\": \"%s\", \"tag_first\": \"%s\", "
         "\"tag_last\": \"%s\"}\n",
         name, extra_json, len_arg, (unsigned long long)n, (unsigned long long)total_bytes,
         hex(tags_d, 32).c_str(), hex(ct_d, 32).c_str(), n ? hex(&tags[0], 16).c_str() : "",
         n ? hex(&tags[16 * (n - 1)], 16).c_str() : "");
  return 0;
}

// ref_tool digest AEAD NKEYS RPK LEN [T]: the whole sequence of NKEYS keys x
// RPK records (records [0, NKEYS*RPK), key i / RPK).
int cmd_digest(int argc, char **argv) {
  if (argc < 6) return 2;
  uint64_t nkeys = strtoull(argv[3], nullptr, 0);
  uint64_t rpk = strtoull(argv[4], nullptr, 0);
  int threads = argc > 6 ? atoi(argv[6]) : 8;
  char extra[128];
  snprintf(extra, sizeof extra, "\"nkeys\": %llu, \"records_per_key\": %llu, ",
           (unsigned long long)nkeys, (unsigned long long)rpk);
  return digest_range(argv[2], 0, nkeys * rpk, rpk, argv[5], threads, extra);
}

// ref_tool shard AEAD LEN FIRST N RPK [T]: records [FIRST, FIRST + N) of the
// sequence, key i / RPK (RPK = 0: one key, key 0) -- one rank's shard.
int cmd_shard(int argc, char **argv) {
  if (argc < 7) return 2;
  uint64_t first = strtoull(argv[4], nullptr, 0);
  uint64_t n = strtoull(argv[5], nullptr, 0);
  uint64_t rpk = strtoull(argv[6], nullptr, 0);
  int threads = argc > 7 ? atoi(argv[7]) : 8;
  char extra[160];
  snprintf(extra, sizeof extra, "\"first\": %llu, \"records_per_key\": %llu, ",
           (unsigned long long)first, (unsigned long long)rpk);
  return digest_range(argv[2], first, n, rpk, argv[3], threads, extra);
}

int cmd_bench(int argc, char **argv) {
  if (argc < 7) return 2;
  size_t key_len;
  const char *name = argv[2];
  const EVP_AEAD *aead = aead_by_name(name, &key_len);
  uint64_t len = strtoull(argv[3], nullptr, 0);
  uint64_t nrec = strtoull(argv[4], nullptr, 0);
  int threads = atoi(argv[5]);
  double secs = atof(argv[6]);
  const uint64_t stride = (len + 63) / 64 * 64;
  std::vector<uint8_t> pt(nrec * stride), ct(nrec * stride), tags(nrec * 16);
  const size_t nl = EVP_AEAD_nonce_length(aead);
  std::vector<uint8_t> nonces(nrec * nl), ads(nrec * 13);
  for (uint64_t i = 0; i < nrec; i++) {
    synth_pt(i, len, &pt[i * stride]);
    make_nonce(i, nl, &nonces[nl * i]);
    synth_ad(i, len, &ads[13 * i]);
  }
  std::vector<uint8_t> key(key_len);
  synth_key(0, key_len, key.data());
  bssl::ScopedEVP_AEAD_CTX ctx;
  if (!EVP_AEAD_CTX_init_with_direction(ctx.get(), aead, key.data(), key_len,
                                        EVP_AEAD_DEFAULT_TAG_LENGTH, evp_aead_seal))
    return 1;
  std::vector<uint64_t> done(threads, 0);
  auto t0 = std::chrono::steady_clock::now();
  double elapsed = 0;
#pragma omp parallel num_threads(threads)
  {
    int t = omp_get_thread_num();
    uint64_t lo = nrec * t / threads, hi = nrec * (t + 1) / threads;
    uint64_t count = 0;
    for (;;) {
      for (uint64_t i = lo; i < hi; i++) {
        size_t tag_out;
        if (!EVP_AEAD_CTX_seal_scatter(ctx.get(), &ct[i * stride], &tags[16 * i], &tag_out, 16,
                                       &nonces[nl * i], nl, &pt[i * stride], len, nullptr, 0,
                                       &ads[13 * i], 13))
          abort();
        count++;
      }
      double e = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (e >= secs) break;
    }
    done[t] = count;
  }
  elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t recs = 0;
  for (uint64_t c : done) recs += c;
  double bytes = (double)recs * (double)len;
  printf("{\"aead\": \"%s\", \"len\": %llu, \"sample_records\": %llu, \"threads\": %d, "
         "\"records_sealed\": %llu, \"seconds\": %.4f, \"gib_per_s\": %.4f}\n",
         name, (unsigned long long)len, (unsigned long long)nrec, threads,
         (unsigned long long)recs, elapsed, bytes / elapsed / (1024.0 * 1024 * 1024));
  return 0;
}

// bench/aead.cc:41-133 for one (AEAD, direction, input size): the CPU
// baseline of BASELINE.md section 3, one single-threaded process per core.
int cmd_bench1(int argc, char **argv) {
  if (argc < 6) return 2;
  size_t key_len;
  const char *name = argv[2];
  const EVP_AEAD *aead = aead_by_name(name, &key_len);
  const bool open = std::string(argv[3]) == "open";
  const size_t len = strtoull(argv[4], nullptr, 0);
  const double secs = atof(argv[5]);
  const size_t nl = EVP_AEAD_nonce_length(aead), overhead = EVP_AEAD_max_overhead(aead);
  const size_t kAlign = 16, kAdLen = 13;
  std::vector<uint8_t> key(key_len), nonce(nl), ad(kAdLen);
  std::vector<uint8_t> in_s(len + kAlign), out_s(len + overhead + kAlign),
      in2_s(len + overhead + kAlign), tag_s(overhead + kAlign);
  auto align = [](uint8_t *p) {
    return reinterpret_cast<uint8_t *>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
  };
  uint8_t *in = align(in_s.data()), *out = align(out_s.data()), *in2 = align(in2_s.data()),
          *tag = align(tag_s.data());
  bssl::ScopedEVP_AEAD_CTX ctx;
  if (!EVP_AEAD_CTX_init_with_direction(ctx.get(), aead, key.data(), key_len,
                                        EVP_AEAD_DEFAULT_TAG_LENGTH, evp_aead_seal))
    return 1;
  size_t out_len = 0;
  if (open) {
    if (!EVP_AEAD_CTX_seal(ctx.get(), out, &out_len, len + overhead, nonce.data(), nl, in, len,
                           ad.data(), kAdLen))
      return 1;
    ctx.Reset();
    if (!EVP_AEAD_CTX_init_with_direction(ctx.get(), aead, key.data(), key_len,
                                          EVP_AEAD_DEFAULT_TAG_LENGTH, evp_aead_open))
      return 1;
  }
  uint64_t iters = 0;
  auto t0 = std::chrono::steady_clock::now();
  double e = 0;
  do {
    for (int k = 0; k < 64; k++) {
      size_t l;
      int ok = open ? EVP_AEAD_CTX_open(ctx.get(), in2, &l, len + overhead, nonce.data(), nl, out,
                                        out_len, ad.data(), kAdLen)
                    : EVP_AEAD_CTX_seal_scatter(ctx.get(), out, tag, &l, overhead, nonce.data(),
                                                nl, in, len, nullptr, 0, ad.data(), kAdLen);
      if (!ok) return 1;
      __asm__ volatile("" ::: "memory");  // benchmark::ClobberMemory
    }
    iters += 64;
    e = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  } while (e < secs);
  printf("{\"aead\": \"%s\", \"op\": \"%s\", \"len\": %zu, \"iterations\": %llu, "
         "\"seconds\": %.4f, \"gib_per_s\": %.4f}\n",
         name, open ? "open" : "seal", len, (unsigned long long)iters, e,
         (double)iters * (double)len / e / (1024.0 * 1024 * 1024));
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: ref_tool edge|digest|bench ...\n");
    return 2;
  }
  std::string cmd = argv[1];
  if (cmd == "edge") return cmd_edge();
  if (cmd == "digest") return cmd_digest(argc, argv);
  if (cmd == "shard") return cmd_shard(argc, argv);
  if (cmd == "bench") return cmd_bench(argc, argv);
  if (cmd == "bench1") return cmd_bench1(argc, argv);
  return 2;
}
