// AWS Signature Version 4 on the server side (C08 signing, C10 URI encoding; reference
// dfs/common/src/auth/{signing,encoding}.rs and s3_server auth_middleware.rs:676-716):
// canonical request, string to sign, the HMAC-SHA256 key chain and a constant-time
// signature check, on OpenSSL. The S3 gateway verifies every signed request through here.
#pragma once
#include <string>
#include <utility>
#include <vector>

namespace dfs::sigv4 {

// Percent-encoding with uppercase hex; unreserved = A-Z a-z 0-9 - _ . ~
std::string uri_encode(const std::string& s, bool encode_slash);
// Sort key=value pairs of a raw query, dropping X-Amz-Signature (values stay as sent).
std::string normalize_query(const std::string& raw);

struct Request {
  std::string method, path, query;                        // path/query already canonical
  std::vector<std::pair<std::string, std::string>> headers;  // lower-case names, canonical values, sorted
  std::string signed_headers;                               // "host;x-amz-date"
  std::string payload_hash;
};

std::string canonical_request(const Request& r);
std::string sha256_hex(const std::string& data);
std::string sha256_hex(const void* data, size_t n);
std::string string_to_sign(const std::string& timestamp, const std::string& scope, const std::string& creq);
std::string signing_key(const std::string& secret, const std::string& date, const std::string& region,
                        const std::string& service);  // 32 raw bytes
std::string signature(const std::string& key, const std::string& sts);  // lower-case hex
// Constant-time comparison of the expected signature with `sig`; *creq receives the
// canonical request (for the SignatureDoesNotMatch diagnostics).
bool verify(const Request& r, const std::string& timestamp, const std::string& scope, const std::string& key,
            const std::string& sig, std::string* creq);
// Constant-time equality of two lower-case hex signatures.
bool same_signature(const std::string& expected, const std::string& sig);

// The per-chunk signature chain of a STREAMING-AWS4-HMAC-SHA256-PAYLOAD body (aws-chunked;
// reference auth_middleware.rs streaming payloads): every chunk's signature signs the previous
// one and the chunk's SHA-256, starting from the request's own (seed) signature.
struct ChunkChain {
  std::string key, timestamp, scope, prev;
  // True (and the chain advanced) when `sig` is the expected signature of this chunk.
  bool verify(const void* chunk, size_t n, const std::string& sig);
  // The client side: this chunk's signature (the chain advanced to it).
  std::string next(const void* chunk, size_t n);
};

}  // namespace dfs::sigv4
