#include "sts.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>

#include <chrono>
#include <cmath>
#include <cstring>

#include "crypto.h"
#include "tls.h"

namespace dfs::sts {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

int connect_to(const std::string& host, const std::string& port, int timeout_ms, std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_socktype = SOCK_STREAM;
  if (int rc = ::getaddrinfo(host.c_str(), port.c_str(), &hints, &res); rc != 0) {
    *err = "resolve " + host + ": " + gai_strerror(rc);
    return -1;
  }
  int fd = -1;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
  }
  ::freeaddrinfo(res);
  if (fd < 0) *err = "connect " + host + ":" + port + ": " + std::strerror(errno);
  return fd;
}

bool hmac_sha256_eq(const std::string& key, const std::string& msg, const std::string& sig) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()), reinterpret_cast<const unsigned char*>(msg.data()),
       msg.size(), out, &n);
  return n == sig.size() && CRYPTO_memcmp(out, sig.data(), n) == 0;
}

}  // namespace

Json Claims::to_json() const {
  Json d = extra.is_object() ? extra : Json::object();
  d.set("sub", sub);
  d.set("aud", aud);
  d.set("iss", iss);
  d.set("exp", exp);
  d.set("iat", iat);
  Json g = Json::array();
  for (auto& x : groups) g.push_back(Json(x));
  d.set("groups", g);
  return d;
}

bool http_get(const std::string& url, int timeout_ms, const std::string& ca, std::string* body, std::string* err) {
  const bool https = url.compare(0, 8, "https://") == 0;
  if (!https && url.compare(0, 7, "http://") != 0) return (*err = "unsupported URL " + url, false);
  std::string rest = url.substr(https ? 8 : 7);
  const size_t slash = rest.find('/');
  const std::string hostport = rest.substr(0, slash), path = slash == std::string::npos ? "/" : rest.substr(slash);
  std::string host = hostport, port = https ? "443" : "80";
  if (size_t c = hostport.rfind(':'); c != std::string::npos && hostport.find(']') == std::string::npos) {
    host = hostport.substr(0, c);
    port = hostport.substr(c + 1);
  }
  int fd = connect_to(host, port, timeout_ms, err);
  if (fd < 0) return false;
  std::unique_ptr<TlsConn> tls;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  if (https) {
    auto ctx = TlsContext::client_http1(ca, err);
    if (!ctx) {
      ::close(fd);
      return false;
    }
    tls = std::make_unique<TlsConn>(ctx, fd);
    if (!tls->handshake(host, deadline, err)) {
      tls.reset();
      ::close(fd);
      return false;
    }
  }
  const std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + hostport +
                          "\r\nAccept: application/json\r\nConnection: close\r\n\r\n";
  bool ok = tls ? tls->write_all(req.data(), req.size(), deadline)
                : ::send(fd, req.data(), req.size(), MSG_NOSIGNAL) == static_cast<ssize_t>(req.size());
  std::string resp;
  char buf[16 << 10];
  while (ok) {
    long n = tls ? tls->read(buf, sizeof buf) : static_cast<long>(::recv(fd, buf, sizeof buf, 0));
    if (n <= 0) break;
    resp.append(buf, static_cast<size_t>(n));
    if (resp.size() > (8u << 20)) break;
  }
  tls.reset();
  ::close(fd);
  const size_t he = resp.find("\r\n\r\n");
  if (!ok || he == std::string::npos) return (*err = "no HTTP response from " + url, false);
  const std::string head = resp.substr(0, he);
  const size_t sp = head.find(' ');
  const int status = sp == std::string::npos ? 0 : std::atoi(head.c_str() + sp + 1);
  if (status != 200) return (*err = "HTTP " + std::to_string(status) + " from " + url, false);
  std::string b = resp.substr(he + 4);
  std::string lower;
  for (char ch : head) lower.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(ch))));
  if (lower.find("transfer-encoding: chunked") != std::string::npos) {  // de-chunk
    std::string out;
    size_t p = 0;
    while (p < b.size()) {
      size_t e = b.find("\r\n", p);
      if (e == std::string::npos) break;
      const size_t n = std::strtoull(b.substr(p, e - p).c_str(), nullptr, 16);
      if (n == 0) break;
      out += b.substr(e + 2, n);
      p = e + 2 + n + 2;
    }
    b = out;
  }
  *body = std::move(b);
  return true;
}

std::string b64url_decode(const std::string& s, bool* ok) {
  std::string t = s;
  for (auto& ch : t) {
    if (ch == '-') ch = '+';
    else if (ch == '_') ch = '/';
  }
  while (t.size() % 4) t.push_back('=');
  std::string out;
  *ok = crypto::base64_decode(t, &out);
  return out;
}

OidcValidator::OidcValidator(std::string issuer, std::string client_id, bool allow_hs256, std::string ca)
    : issuer_(std::move(issuer)), client_id_(std::move(client_id)), ca_(std::move(ca)), allow_hs256_(allow_hs256) {}

bool OidcValidator::fetch_jwks(std::string* err) {
  {
    std::lock_guard<std::mutex> g(mu_);
    last_try_ = now_s();
  }
  std::string base = issuer_;
  while (!base.empty() && base.back() == '/') base.pop_back();
  std::string body;
  std::map<std::string, Json> keys;
  try {
    if (!http_get(base + "/.well-known/openid-configuration", 5000, ca_, &body, err)) throw std::runtime_error(*err);
    const std::string uri = Json::parse(body)["jwks_uri"].str();
    if (uri.empty()) throw std::runtime_error("missing jwks_uri in OIDC config");
    if (!http_get(uri, 5000, ca_, &body, err)) throw std::runtime_error(*err);
    Json jwks = Json::parse(body);
    const Json& arr = jwks["keys"];
    if (arr.is_array())
      for (auto& k : arr.items())
        if (k.is_object() && k["kid"].is_string()) keys[k["kid"].str()] = k;
  } catch (const std::exception& e) {
    *err = std::string("failed to fetch JWKS: ") + e.what();
    std::lock_guard<std::mutex> g(mu_);
    ++failed_;
    return false;
  }
  std::lock_guard<std::mutex> g(mu_);
  keys_ = std::move(keys);
  have_ = true;
  ++ok_;
  last_ = now_s();
  return true;
}

bool OidcValidator::validate(const std::string& token, Claims* out, std::string* kind, std::string* detail, double now) {
  auto bad = [&](const std::string& k, const std::string& d) {
    *kind = k;
    *detail = d;
    return false;
  };
  const size_t d1 = token.find('.'), d2 = d1 == std::string::npos ? d1 : token.find('.', d1 + 1);
  if (d1 == std::string::npos || d2 == std::string::npos || token.find('.', d2 + 1) != std::string::npos)
    return bad("invalid_token", "invalid JWT: not three segments");
  const std::string h64 = token.substr(0, d1), p64 = token.substr(d1 + 1, d2 - d1 - 1), s64 = token.substr(d2 + 1);
  Json header, payload;
  std::string sig;
  try {
    bool ok1, ok2, ok3;
    header = Json::parse(b64url_decode(h64, &ok1));
    payload = Json::parse(b64url_decode(p64, &ok2));
    sig = b64url_decode(s64, &ok3);
    if (!ok1 || !ok2 || !ok3 || !header.is_object() || !payload.is_object()) throw std::runtime_error("bad encoding");
  } catch (const std::exception& e) {
    return bad("invalid_token", std::string("invalid JWT: ") + e.what());
  }
  const std::string kid = header["kid"].str();
  if (kid.empty()) return bad("invalid_token", "missing kid in JWT header");
  Json jwk;
  {
    bool have;
    {
      std::lock_guard<std::mutex> g(mu_);
      have = have_ && keys_.count(kid);
    }
    if (!have) {
      // a rotated key: refetch, but at most once per kRefetchGapS, and never two at a time
      std::unique_lock<std::mutex> lk(mu_);
      if (fetching_) {
        fetch_cv_.wait_for(lk, std::chrono::seconds(12), [&] { return !fetching_; });
      } else if (last_try_ == 0 || now_s() - last_try_ >= kRefetchGapS) {
        fetching_ = true;
        lk.unlock();
        std::string err;
        (void)fetch_jwks(&err);
        lk.lock();
        fetching_ = false;
        fetch_cv_.notify_all();
      }
    }
    std::lock_guard<std::mutex> g(mu_);
    if (!have_) return bad("internal", "JWKS is not available");
    auto it = keys_.find(kid);
    if (it == keys_.end()) return bad("invalid_token", "kid " + kid + " not found in JWKS");
    jwk = it->second;
  }
  const std::string alg = header["alg"].str(), msg = h64 + "." + p64;
  bool verified;
  if (alg == "RS256" && jwk["kty"].str() == "RSA") {
    bool okn, oke;
    const std::string n = b64url_decode(jwk["n"].str(), &okn), e = b64url_decode(jwk["e"].str(), &oke);
    verified = okn && oke && crypto::rsa_sha256_verify(n, e, msg, sig);
  } else if (alg == "HS256" && jwk["kty"].str() == "oct" && allow_hs256_) {
    bool okk;
    const std::string k = b64url_decode(jwk["k"].str(), &okk);
    verified = okk && hmac_sha256_eq(k, msg, sig);
  } else {
    return bad("invalid_token", "unsupported algorithm " + alg);
  }
  if (!verified) return bad("invalid_token", "signature verification failed");
  if (now == 0) now = now_s();
  const Json& aud = payload["aud"];
  bool aud_ok = false;
  if (aud.is_array()) {
    for (auto& x : aud.items()) aud_ok |= x.str() == client_id_;
  } else {
    aud_ok = aud.str() == client_id_;
  }
  if (!aud_ok) return bad("invalid_token", "audience mismatch");
  if (payload["iss"].str() != issuer_) return bad("invalid_token", "issuer mismatch");
  if (!payload["exp"].is_number() || payload["exp"].as_double() + 60 < now) return bad("invalid_token", "token expired");
  if (payload.has("nbf") && payload["nbf"].as_double() - 60 > now) return bad("invalid_token", "token not yet valid");
  // Claims.from_json: sub, aud, iss, exp, iat required
  if (!payload.has("sub") || !payload.has("aud") || !payload.has("iss") || !payload.has("exp") || !payload.has("iat"))
    return bad("invalid_token", "missing or invalid claim");
  Claims c;
  const Json& sub = payload["sub"];
  c.sub = sub.is_string() ? sub.str() : sub.dump();
  c.aud = aud.is_array() ? (aud.size() ? aud[0].str() : std::string()) : aud.str();
  c.iss = payload["iss"].str();
  c.exp = static_cast<int64_t>(payload["exp"].as_double());
  c.iat = static_cast<int64_t>(payload["iat"].as_double());
  if (payload["groups"].is_array())
    for (auto& g : payload["groups"].items()) c.groups.push_back(g.is_string() ? g.str() : g.dump());
  for (auto& kv : payload.fields())
    if (kv.first != "sub" && kv.first != "aud" && kv.first != "iss" && kv.first != "exp" && kv.first != "iat" &&
        kv.first != "groups")
      c.extra.set(kv.first, kv.second);
  *out = std::move(c);
  return true;
}

std::string random_alnum(size_t n) {
  static const char kAlnum[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
  std::string out;
  while (out.size() < n) {
    const std::string r = crypto::random_bytes(2 * n);
    for (unsigned char b : r) {
      if (b < 248) out.push_back(kAlnum[b % 62]);  // 248 = 4 * 62: unbiased
      if (out.size() == n) break;
    }
  }
  return out;
}

std::string make_token(const std::string& key32, uint32_t kid, const std::string& role_arn,
                       const std::string& temp_secret, int64_t expiration, const Claims& claims) {
  Json d = Json::object();
  d.set("role_arn", role_arn);
  d.set("temp_secret_key", temp_secret);
  d.set("expiration", expiration);
  d.set("claims", claims.to_json());
  const std::string nonce = crypto::random_bytes(12);
  std::string raw;
  raw.push_back(static_cast<char>(kid >> 24));
  raw.push_back(static_cast<char>(kid >> 16));
  raw.push_back(static_cast<char>(kid >> 8));
  raw.push_back(static_cast<char>(kid));
  raw += nonce + crypto::aes256gcm_encrypt(key32, nonce, d.dump(), "");
  return crypto::base64_encode(raw);
}

}  // namespace dfs::sts
