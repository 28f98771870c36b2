// STS AssumeRoleWithWebIdentity for the native S3 gateway (C15 OIDC, C16 STS tokens, C55 the
// endpoint; reference dfs/s3_server/src/sts_handler.rs:65-395, common/src/auth/oidc.rs:33-120,
// auth/sts.rs:60-98). The same token format and validation rules as tests/models/s3_identity.py, so a
// session issued by either gateway opens in the other:
//   * OIDC: <issuer>/.well-known/openid-configuration -> jwks_uri -> JWKS (cached, refetched
//     when a kid is unknown); RS256 (RSA JWKs) always, HS256 ("oct" JWKs) only when allowed;
//     aud must contain the client id, iss equal the issuer, exp / nbf with 60 s leeway;
//   * token = base64(kid u32 BE || nonce 12 || AES-256-GCM(JSON{role_arn, temp_secret_key,
//     expiration, claims})).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "json.h"

namespace dfs::sts {

struct Claims {
  std::string sub, aud, iss;
  int64_t exp = 0, iat = 0;
  std::vector<std::string> groups;
  Json extra = Json::object();  // every other claim, kept for the session token
  Json to_json() const;
};

// One HTTP(S)/1.1 GET; false with *err on a connection, TLS or status failure.
bool http_get(const std::string& url, int timeout_ms, const std::string& ca, std::string* body, std::string* err);

class OidcValidator {
 public:
  // An unknown kid triggers at most one discovery + JWKS fetch per this many seconds
  // (concurrent validations share the running one): unauthenticated callers cannot drive
  // unbounded outbound fetches from the gateway's request threads.
  static constexpr double kRefetchGapS = 10.0;
  OidcValidator(std::string issuer, std::string client_id, bool allow_hs256, std::string ca = "");
  // Discovery + JWKS; false with *err.
  bool fetch_jwks(std::string* err);
  // True with *out; else *kind is "invalid_token" or "internal" (the AuthError kinds) and
  // *detail says why.
  bool validate(const std::string& token, Claims* out, std::string* kind, std::string* detail, double now = 0);
  uint64_t fetches_ok() const { return ok_; }
  uint64_t fetches_failed() const { return failed_; }
  double last_fetch() const { return last_; }

 private:
  std::string issuer_, client_id_, ca_;
  bool allow_hs256_;
  std::mutex mu_;
  std::condition_variable fetch_cv_;
  bool fetching_ = false;   // a refetch is running: others wait for it instead of fetching too
  double last_try_ = 0;     // last fetch attempt (unknown kids refetch at most every kRefetchGapS)
  bool have_ = false;
  std::map<std::string, Json> keys_;  // kid -> JWK
  uint64_t ok_ = 0, failed_ = 0;
  double last_ = 0;
};

std::string b64url_decode(const std::string& s, bool* ok);
std::string random_alnum(size_t n);
// The session token of StsTokenManager.generate_token.
std::string make_token(const std::string& key32, uint32_t kid, const std::string& role_arn,
                       const std::string& temp_secret, int64_t expiration, const Claims& claims);

}  // namespace dfs::sts
