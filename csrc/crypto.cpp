#include "crypto.h"

#include <openssl/bn.h>
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/param_build.h>
#include <openssl/rand.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace dfs::crypto {

namespace {
struct CtxFree {
  void operator()(EVP_CIPHER_CTX* c) const { EVP_CIPHER_CTX_free(c); }
};
using CipherCtx = std::unique_ptr<EVP_CIPHER_CTX, CtxFree>;
const unsigned char* u(const std::string& s) { return reinterpret_cast<const unsigned char*>(s.data()); }
}  // namespace

std::string aes256gcm_encrypt(const std::string& key, const std::string& nonce, const std::string& pt,
                              const std::string& aad) {
  if (key.size() != 32) throw std::runtime_error("AES-256-GCM key must be 32 bytes");
  CipherCtx ctx(EVP_CIPHER_CTX_new());
  int len = 0;
  std::string out(pt.size() + 16, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  if (!EVP_EncryptInit_ex(ctx.get(), EVP_aes_256_gcm(), nullptr, nullptr, nullptr) ||
      !EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_IVLEN, static_cast<int>(nonce.size()), nullptr) ||
      !EVP_EncryptInit_ex(ctx.get(), nullptr, nullptr, u(key), u(nonce)))
    throw std::runtime_error("aes-gcm init failed");
  if (!aad.empty() && !EVP_EncryptUpdate(ctx.get(), nullptr, &len, u(aad), static_cast<int>(aad.size())))
    throw std::runtime_error("aes-gcm aad failed");
  int total = 0;
  if (!pt.empty()) {
    if (!EVP_EncryptUpdate(ctx.get(), o, &len, u(pt), static_cast<int>(pt.size())))
      throw std::runtime_error("aes-gcm update failed");
    total = len;
  }
  if (!EVP_EncryptFinal_ex(ctx.get(), o + total, &len)) throw std::runtime_error("aes-gcm final failed");
  total += len;
  if (!EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_GET_TAG, 16, o + total))
    throw std::runtime_error("aes-gcm tag failed");
  out.resize(static_cast<size_t>(total) + 16);
  return out;
}

std::string aes256gcm_decrypt(const std::string& key, const std::string& nonce, const std::string& ct,
                              const std::string& aad) {
  if (key.size() != 32) throw std::runtime_error("AES-256-GCM key must be 32 bytes");
  if (ct.size() < 16) throw std::runtime_error("ciphertext too short");
  CipherCtx ctx(EVP_CIPHER_CTX_new());
  size_t body = ct.size() - 16;
  std::string out(body, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  int len = 0, total = 0;
  if (!EVP_DecryptInit_ex(ctx.get(), EVP_aes_256_gcm(), nullptr, nullptr, nullptr) ||
      !EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_IVLEN, static_cast<int>(nonce.size()), nullptr) ||
      !EVP_DecryptInit_ex(ctx.get(), nullptr, nullptr, u(key), u(nonce)))
    throw std::runtime_error("aes-gcm init failed");
  if (!aad.empty() && !EVP_DecryptUpdate(ctx.get(), nullptr, &len, u(aad), static_cast<int>(aad.size())))
    throw std::runtime_error("aes-gcm aad failed");
  if (body) {
    if (!EVP_DecryptUpdate(ctx.get(), o, &len, u(ct), static_cast<int>(body)))
      throw std::runtime_error("aes-gcm update failed");
    total = len;
  }
  std::string tag = ct.substr(body);
  if (!EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_TAG, 16, const_cast<char*>(tag.data())))
    throw std::runtime_error("aes-gcm set tag failed");
  if (EVP_DecryptFinal_ex(ctx.get(), o + total, &len) <= 0)
    throw std::runtime_error("aead::Error: authentication failed");
  out.resize(static_cast<size_t>(total + len));
  return out;
}

void aes256gcm_encrypt_inplace(const uint8_t* key, const uint8_t* nonce, uint8_t* p, size_t n, uint8_t* tag) {
  CipherCtx ctx(EVP_CIPHER_CTX_new());
  int len = 0;
  if (!EVP_EncryptInit_ex(ctx.get(), EVP_aes_256_gcm(), nullptr, nullptr, nullptr) ||
      !EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) ||
      !EVP_EncryptInit_ex(ctx.get(), nullptr, nullptr, key, nonce))
    throw std::runtime_error("aes-gcm init failed");
  for (size_t off = 0; off < n;) {  // GCM is a stream mode: in place is allowed
    const int k = static_cast<int>(std::min<size_t>(n - off, 1u << 30));
    if (!EVP_EncryptUpdate(ctx.get(), p + off, &len, p + off, k)) throw std::runtime_error("aes-gcm update failed");
    off += static_cast<size_t>(k);
  }
  if (!EVP_EncryptFinal_ex(ctx.get(), p + n, &len) || len != 0) throw std::runtime_error("aes-gcm final failed");
  if (!EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_GET_TAG, 16, tag)) throw std::runtime_error("aes-gcm tag failed");
}

bool aes256gcm_decrypt_inplace(const uint8_t* key, const uint8_t* nonce, uint8_t* p, size_t n, const uint8_t* tag) {
  CipherCtx ctx(EVP_CIPHER_CTX_new());
  int len = 0;
  if (!EVP_DecryptInit_ex(ctx.get(), EVP_aes_256_gcm(), nullptr, nullptr, nullptr) ||
      !EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) ||
      !EVP_DecryptInit_ex(ctx.get(), nullptr, nullptr, key, nonce))
    return false;
  for (size_t off = 0; off < n;) {
    const int k = static_cast<int>(std::min<size_t>(n - off, 1u << 30));
    if (!EVP_DecryptUpdate(ctx.get(), p + off, &len, p + off, k)) return false;
    off += static_cast<size_t>(k);
  }
  uint8_t t[16];
  std::memcpy(t, tag, 16);
  if (!EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_GCM_SET_TAG, 16, t)) return false;
  uint8_t fin[16];
  return EVP_DecryptFinal_ex(ctx.get(), fin, &len) > 0;
}

std::string md5_hex(const uint8_t* p, size_t n) {
  unsigned char d[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_Digest(p, n, d, &len, EVP_md5(), nullptr);
  static const char* hx = "0123456789abcdef";
  std::string out;
  for (unsigned i = 0; i < len; ++i) {
    out.push_back(hx[d[i] >> 4]);
    out.push_back(hx[d[i] & 15]);
  }
  return out;
}

std::string base64_encode(const std::string& raw) {
  std::string out(4 * ((raw.size() + 2) / 3) + 1, '\0');
  const int n = EVP_EncodeBlock(reinterpret_cast<unsigned char*>(&out[0]), u(raw), static_cast<int>(raw.size()));
  out.resize(static_cast<size_t>(n));
  return out;
}

bool base64_decode(const std::string& b64, std::string* raw) {
  if (b64.size() % 4) return false;
  for (char ch : b64)
    if (!(std::isalnum(static_cast<unsigned char>(ch)) || ch == '+' || ch == '/' || ch == '=')) return false;
  std::string out(b64.size() / 4 * 3 + 1, '\0');
  const int n = EVP_DecodeBlock(reinterpret_cast<unsigned char*>(&out[0]), u(b64), static_cast<int>(b64.size()));
  if (n < 0) return false;
  size_t pad = 0;  // EVP_DecodeBlock keeps the padding's zero bytes
  if (!b64.empty() && b64.back() == '=') ++pad;
  if (b64.size() > 1 && b64[b64.size() - 2] == '=') ++pad;
  out.resize(static_cast<size_t>(n) - pad);
  *raw = std::move(out);
  return true;
}

bool rsa_sha256_verify(const std::string& n, const std::string& e, const std::string& msg, const std::string& sig) {
  BIGNUM* bn_n = BN_bin2bn(u(n), static_cast<int>(n.size()), nullptr);
  BIGNUM* bn_e = BN_bin2bn(u(e), static_cast<int>(e.size()), nullptr);
  OSSL_PARAM_BLD* bld = OSSL_PARAM_BLD_new();
  OSSL_PARAM_BLD_push_BN(bld, OSSL_PKEY_PARAM_RSA_N, bn_n);
  OSSL_PARAM_BLD_push_BN(bld, OSSL_PKEY_PARAM_RSA_E, bn_e);
  OSSL_PARAM* params = OSSL_PARAM_BLD_to_param(bld);
  EVP_PKEY_CTX* pctx = EVP_PKEY_CTX_new_from_name(nullptr, "RSA", nullptr);
  EVP_PKEY* pkey = nullptr;
  bool ok = pctx && EVP_PKEY_fromdata_init(pctx) > 0 &&
            EVP_PKEY_fromdata(pctx, &pkey, EVP_PKEY_PUBLIC_KEY, params) > 0;
  if (ok) {
    EVP_MD_CTX* md = EVP_MD_CTX_new();
    ok = EVP_DigestVerifyInit(md, nullptr, EVP_sha256(), nullptr, pkey) > 0 &&
         EVP_DigestVerify(md, u(sig), sig.size(), u(msg), msg.size()) == 1;
    EVP_MD_CTX_free(md);
  }
  EVP_PKEY_free(pkey);
  EVP_PKEY_CTX_free(pctx);
  OSSL_PARAM_free(params);
  OSSL_PARAM_BLD_free(bld);
  BN_free(bn_n);
  BN_free(bn_e);
  return ok;
}

std::string random_bytes(size_t n) {
  std::string s(n, '\0');
  if (n && RAND_bytes(reinterpret_cast<unsigned char*>(&s[0]), static_cast<int>(n)) != 1)
    throw std::runtime_error("RAND_bytes failed");
  return s;
}

}  // namespace dfs::crypto
