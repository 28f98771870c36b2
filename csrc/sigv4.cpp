#include "sigv4.h"

#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>

#include <algorithm>

namespace dfs::sigv4 {

namespace {
const char kHex[] = "0123456789abcdef";

std::string hex(const unsigned char* p, size_t n) {
  std::string o(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    o[2 * i] = kHex[p[i] >> 4];
    o[2 * i + 1] = kHex[p[i] & 15];
  }
  return o;
}

std::string hmac(const std::string& key, const std::string& msg) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()), reinterpret_cast<const unsigned char*>(msg.data()),
       msg.size(), out, &n);
  return std::string(reinterpret_cast<char*>(out), n);
}

bool unreserved(unsigned char c) {
  return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
         c == '.' || c == '~';
}
}  // namespace

std::string uri_encode(const std::string& s, bool encode_slash) {
  static const char kUp[] = "0123456789ABCDEF";
  std::string o;
  o.reserve(s.size() * 3);
  for (unsigned char c : s) {
    if (unreserved(c) || (c == '/' && !encode_slash)) {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(kUp[c >> 4]);
      o.push_back(kUp[c & 15]);
    }
  }
  return o;
}

std::string normalize_query(const std::string& raw) {
  std::vector<std::pair<std::string, std::string>> kv;
  size_t p = 0;
  while (p <= raw.size()) {
    size_t e = raw.find('&', p);
    if (e == std::string::npos) e = raw.size();
    std::string part = raw.substr(p, e - p);
    p = e + 1;
    if (part.empty() || part == "X-Amz-Signature" || part.rfind("X-Amz-Signature=", 0) == 0) continue;
    size_t eq = part.find('=');
    kv.emplace_back(part.substr(0, eq), eq == std::string::npos ? "" : part.substr(eq + 1));
  }
  std::sort(kv.begin(), kv.end());
  std::string o;
  for (size_t i = 0; i < kv.size(); ++i) {
    if (i) o.push_back('&');
    o += kv[i].first;
    o.push_back('=');
    o += kv[i].second;
  }
  return o;
}

std::string canonical_request(const Request& r) {
  std::string o = r.method + "\n" + r.path + "\n" + r.query;
  for (auto& h : r.headers) o += "\n" + h.first + ":" + h.second;
  return o + "\n\n" + r.signed_headers + "\n" + r.payload_hash;
}

std::string sha256_hex(const void* data, size_t len) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  EVP_Digest(data, len, out, &n, EVP_sha256(), nullptr);
  return hex(out, n);
}

std::string sha256_hex(const std::string& data) { return sha256_hex(data.data(), data.size()); }

std::string string_to_sign(const std::string& timestamp, const std::string& scope, const std::string& creq) {
  return "AWS4-HMAC-SHA256\n" + timestamp + "\n" + scope + "\n" + sha256_hex(creq);
}

std::string signing_key(const std::string& secret, const std::string& date, const std::string& region,
                        const std::string& service) {
  return hmac(hmac(hmac(hmac("AWS4" + secret, date), region), service), "aws4_request");
}

std::string signature(const std::string& key, const std::string& sts) {
  std::string mac = hmac(key, sts);
  return hex(reinterpret_cast<const unsigned char*>(mac.data()), mac.size());
}

bool verify(const Request& r, const std::string& timestamp, const std::string& scope, const std::string& key,
            const std::string& sig, std::string* creq) {
  *creq = canonical_request(r);
  return same_signature(signature(key, string_to_sign(timestamp, scope, *creq)), sig);
}

bool same_signature(const std::string& expected, const std::string& sig) {
  return expected.size() == sig.size() && CRYPTO_memcmp(expected.data(), sig.data(), sig.size()) == 0;
}

namespace {
std::string chunk_signature(const ChunkChain& c, const void* chunk, size_t n) {
  static const char kEmpty[] = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855";
  return signature(c.key, "AWS4-HMAC-SHA256-PAYLOAD\n" + c.timestamp + "\n" + c.scope + "\n" + c.prev + "\n" +
                              kEmpty + "\n" + sha256_hex(chunk, n));
}
}  // namespace

bool ChunkChain::verify(const void* chunk, size_t n, const std::string& sig) {
  std::string expected = chunk_signature(*this, chunk, n);
  if (!same_signature(expected, sig)) return false;
  prev = std::move(expected);
  return true;
}

std::string ChunkChain::next(const void* chunk, size_t n) {
  prev = chunk_signature(*this, chunk, n);
  return prev;
}

}  // namespace dfs::sigv4
