// Decryption of encrypted input files (reference: water/parser/DecryptionTool.java, GenericDecryptionTool.java,
// water/api/DecryptionSetupHandler.java) on OpenSSL's libcrypto.
//
//  * h2o_pbe_md5_3des_decrypt: the PBEWithMD5AndTripleDES cipher that seals JCEKS secret-key entries
//    (com.sun.crypto.provider.KeyProtector): the 8-byte salt is split into halves (the first half reversed when the
//    halves are equal), each half is digested `iters` times as md5(prev || password) and the two 16-byte digests
//    give the 24-byte DESede key and the 8-byte CBC IV; DESede/CBC/PKCS5Padding.
//  * h2o_cipher_decrypt: Cipher.getInstance(spec) + init(DECRYPT_MODE, key) + doFinal for the IV-less specs
//    GenericDecryptionTool can run: AES/ECB and DESede/ECB, PKCS5Padding or NoPadding.
//  * h2o_cipher_encrypt: the inverse (test fixtures and export of encrypted files).
// The keystore container and the Java serialisation around the sealed key are parsed in io/decrypt.py.
#include <openssl/evp.h>
#include <string.h>

#include "abi.h"

namespace {

const EVP_CIPHER* ecb_cipher(int algo, int keylen) {
  if (algo == 0) {                     // AES
    if (keylen == 16) return EVP_aes_128_ecb();
    if (keylen == 24) return EVP_aes_192_ecb();
    if (keylen == 32) return EVP_aes_256_ecb();
    return nullptr;
  }
  if (algo == 1 && keylen == 24) return EVP_des_ede3_ecb();   // DESede
  return nullptr;
}

int run_cipher(const EVP_CIPHER* c, int enc, const unsigned char* key, const unsigned char* iv, int padding,
               const unsigned char* in, long long inlen, unsigned char* out, long long* outlen) {
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  if (!ctx) return -1;
  int rc = -2;
  int n1 = 0, n2 = 0;
  long long done = 0;
  if (EVP_CipherInit_ex(ctx, c, nullptr, key, iv, enc) == 1 && EVP_CIPHER_CTX_set_padding(ctx, padding) == 1) {
    rc = 0;
    // EVP_CipherUpdate takes int lengths: feed 1 GiB slices
    while (done < inlen) {
      const long long step = inlen - done > (1ll << 30) ? (1ll << 30) : inlen - done;
      if (EVP_CipherUpdate(ctx, out + *outlen, &n1, in + done, (int)step) != 1) { rc = -3; break; }
      *outlen += n1;
      done += step;
    }
    if (rc == 0 && EVP_CipherFinal_ex(ctx, out + *outlen, &n2) != 1) rc = -4;   // bad padding / wrong key
    if (rc == 0) *outlen += n2;
  }
  EVP_CIPHER_CTX_free(ctx);
  return rc;
}

}  // namespace

extern "C" {

// out: >= inlen bytes. Returns 0 and the plaintext length in *outlen, or < 0.
int h2o_pbe_md5_3des_decrypt(const unsigned char* salt8, int iters, const unsigned char* pw, int pwlen,
                             const unsigned char* in, long long inlen, unsigned char* out, long long* outlen) {
  unsigned char salt[8];
  memcpy(salt, salt8, 8);
  if (memcmp(salt, salt + 4, 4) == 0) {
    // identical halves: the JDK's PBES1Core means to reverse the first half but stores the swapped byte at index
    // 3 - 1 on both turns, so [a, b, c, d] becomes [d, a, b, d]; keystores sealed by the JDK need the same bytes
    for (int i = 0; i < 2; ++i) { const unsigned char t = salt[i]; salt[i] = salt[3 - i]; salt[3 - 1] = t; }
  }
  unsigned char derived[32];
  EVP_MD_CTX* md = EVP_MD_CTX_new();
  if (!md) return -1;
  for (int h = 0; h < 2; ++h) {
    unsigned char buf[16];
    unsigned int blen = 4;
    memcpy(buf, salt + 4 * h, 4);
    for (int j = 0; j < iters; ++j) {
      if (EVP_DigestInit_ex(md, EVP_md5(), nullptr) != 1 || EVP_DigestUpdate(md, buf, blen) != 1 ||
          EVP_DigestUpdate(md, pw, (size_t)pwlen) != 1 || EVP_DigestFinal_ex(md, buf, &blen) != 1) {
        EVP_MD_CTX_free(md);
        return -2;
      }
    }
    memcpy(derived + 16 * h, buf, 16);
  }
  EVP_MD_CTX_free(md);
  *outlen = 0;
  return run_cipher(EVP_des_ede3_cbc(), 0, derived, derived + 24, 1, in, inlen, out, outlen);
}

// algo: 0 AES, 1 DESede (ECB). padding: 1 PKCS5Padding, 0 NoPadding. out: >= inlen (+ one block when encrypting).
int h2o_cipher_decrypt(int algo, const unsigned char* key, int keylen, int padding, const unsigned char* in,
                       long long inlen, unsigned char* out, long long* outlen) {
  const EVP_CIPHER* c = ecb_cipher(algo, keylen);
  if (!c) return -10;
  *outlen = 0;
  return run_cipher(c, 0, key, nullptr, padding, in, inlen, out, outlen);
}

int h2o_cipher_encrypt(int algo, const unsigned char* key, int keylen, int padding, const unsigned char* in,
                       long long inlen, unsigned char* out, long long* outlen) {
  const EVP_CIPHER* c = ecb_cipher(algo, keylen);
  if (!c) return -10;
  *outlen = 0;
  return run_cipher(c, 1, key, nullptr, padding, in, inlen, out, outlen);
}

}  // extern "C"
