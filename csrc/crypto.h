// OpenSSL-backed primitives for the S3 gateway: AES-256-GCM (SSE-S3 envelope and STS
// session tokens; reference dfs/common/src/auth/sse.rs, sts.rs) and RS256 signature
// verification for OIDC JWTs (reference auth/oidc.rs). SigV4 HMAC/SHA-256 and MD5 ETags
// use Python's hashlib/hmac, which are the same OpenSSL routines.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace dfs::crypto {

// Returns ciphertext || 16-byte tag.
std::string aes256gcm_encrypt(const std::string& key, const std::string& nonce, const std::string& plaintext,
                              const std::string& aad);
// Throws std::runtime_error on authentication failure.
std::string aes256gcm_decrypt(const std::string& key, const std::string& nonce, const std::string& ct_and_tag,
                              const std::string& aad);
// n, e: big-endian unsigned integers (JWK "n", "e" after base64url decoding).
bool rsa_sha256_verify(const std::string& n, const std::string& e, const std::string& msg, const std::string& sig);
std::string random_bytes(size_t n);
// In place over [p, p + n): encrypt writes the 16-byte tag to `tag`; decrypt returns false
// when the tag does not authenticate (the buffer then holds garbage).
void aes256gcm_encrypt_inplace(const uint8_t* key32, const uint8_t* nonce12, uint8_t* p, size_t n, uint8_t* tag);
bool aes256gcm_decrypt_inplace(const uint8_t* key32, const uint8_t* nonce12, uint8_t* p, size_t n,
                               const uint8_t* tag);
std::string md5_hex(const uint8_t* p, size_t n);
std::string base64_encode(const std::string& raw);
bool base64_decode(const std::string& b64, std::string* raw);  // strict standard alphabet

}  // namespace dfs::crypto
