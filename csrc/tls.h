// TLS for the native HTTP/2 wire (C06; reference dfs/common/src/security.rs:33-105: PEM
// loading, server config from --tls-cert/--tls-key, client config from --ca-cert with the
// domain defaulting to the URL host, https:// endpoints).
//
// OpenSSL with ALPN "h2" — grpc-core (the Python grpcio clients and servers) and tonic refuse
// a TLS peer that does not negotiate h2. One TlsContext (an SSL_CTX) is shared by every
// connection of a server or client pool; a TlsConn is one SSL session bound to one socket and
// is driven by exactly one thread at a time (the connection owner), like the nghttp2 session
// it carries. Both blocking sockets (server connection threads) and non-blocking ones (the
// client pool, which waits with poll() against a call deadline) are supported.
#pragma once
#include <chrono>
#include <memory>
#include <string>

typedef struct ssl_ctx_st SSL_CTX;
typedef struct ssl_st SSL;

namespace dfs {

class TlsContext {
 public:
  ~TlsContext();
  // Server side: certificate chain + private key (PEM files), ALPN h2.
  static std::shared_ptr<TlsContext> server(const std::string& cert, const std::string& key, std::string* err);
  // Server side for HTTP/1.1 (the S3 front): ALPN "http/1.1" when the client offers it,
  // none otherwise (S3 clients mostly send no ALPN at all).
  static std::shared_ptr<TlsContext> server_http1(const std::string& cert, const std::string& key, std::string* err);
  bool http1() const { return http1_; }
  // Client side: trust `ca` (PEM; empty = system roots), verify the peer's name against
  // `domain` (empty = the host of each target), offer ALPN h2.
  static std::shared_ptr<TlsContext> client(const std::string& ca, const std::string& domain, std::string* err);
  // Client side for HTTP/1.1 fetches (OIDC discovery / JWKS): the same trust and name
  // checks, no ALPN requirement.
  static std::shared_ptr<TlsContext> client_http1(const std::string& ca, std::string* err);
  bool is_server() const { return server_; }
  const std::string& domain() const { return domain_; }
  SSL_CTX* ctx() const { return ctx_; }

 private:
  SSL_CTX* ctx_ = nullptr;
  bool server_ = false;
  bool http1_ = false;
  std::string domain_;
};

class TlsConn {
 public:
  using Deadline = std::chrono::steady_clock::time_point;
  TlsConn(std::shared_ptr<TlsContext> ctx, int fd);
  ~TlsConn();
  TlsConn(const TlsConn&) = delete;
  // Handshake (server: accept; client: connect with SNI / name check for `host`). Until
  // `deadline` on non-blocking sockets. False with *err on failure or if h2 was not agreed.
  bool handshake(const std::string& host, Deadline deadline, std::string* err);
  // >0 bytes, 0 = would block (non-blocking socket), -1 = closed / error.
  long read(void* buf, size_t n);
  // Writes everything (waits for the socket until `deadline` when non-blocking); false on error.
  bool write_all(const void* buf, size_t n, Deadline deadline);
  // Decrypted bytes already buffered inside the session (read them before poll()ing).
  bool pending() const;

 private:
  bool wait(int ssl_err, Deadline deadline);
  std::shared_ptr<TlsContext> ctx_;
  SSL* ssl_ = nullptr;
  int fd_;
};

}  // namespace dfs
