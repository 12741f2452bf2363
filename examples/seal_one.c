/* examples/seal_one.c -- a plain C caller of the drop-in EVP_AEAD surface.
 * Build: cc -Iinclude examples/seal_one.c -Lboringssl_amd -lbssl_amd -o seal_one
 * Seals the all-zero 16 KiB record of bench/aead.cc (zero key, nonce, 13-byte
 * AD) and prints the tag; the reference prints f9ff3fa1f8bade711aa97c0f652d67fe. */
#include <stdio.h>
#include <string.h>

#include <bssl_amd/aead.h>

int main(void) {
  static uint8_t key[16], nonce[12], ad[13], in[16384], out[16384 + 16];
  EVP_AEAD_CTX ctx;
  EVP_AEAD_CTX_zero(&ctx);
  if (!EVP_AEAD_CTX_init(&ctx, EVP_aead_aes_128_gcm(), key, sizeof(key),
                         EVP_AEAD_DEFAULT_TAG_LENGTH, NULL)) {
    fprintf(stderr, "init failed: %08x\n", ERR_get_error());
    return 1;
  }
  size_t out_len = 0;
  if (!EVP_AEAD_CTX_seal(&ctx, out, &out_len, sizeof(out), nonce, sizeof(nonce), in,
                         sizeof(in), ad, sizeof(ad))) {
    fprintf(stderr, "seal failed: %08x\n", ERR_get_error());
    return 1;
  }
  for (size_t i = out_len - 16; i < out_len; i++) printf("%02x", out[i]);
  printf("\n");
  EVP_AEAD_CTX_cleanup(&ctx);
  return 0;
}
