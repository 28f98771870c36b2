// TLS for the native HTTP/2 wire; design notes in tls.h.
#include "tls.h"

#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <arpa/inet.h>
#include <poll.h>

#include <algorithm>

#include <cerrno>
#include <cstring>

namespace dfs {

namespace {

std::string ssl_errors() {
  std::string o;
  unsigned long e;
  char buf[256];
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof buf);
    if (!o.empty()) o += "; ";
    o += buf;
  }
  return o.empty() ? "unknown TLS error" : o;
}

const unsigned char kAlpnH2[] = {2, 'h', '2'};

int select_h2(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in, unsigned int inlen,
              void*) {
  unsigned char* o = nullptr;
  if (SSL_select_next_proto(&o, outlen, kAlpnH2, sizeof kAlpnH2, in, inlen) != OPENSSL_NPN_NEGOTIATED)
    return SSL_TLSEXT_ERR_ALERT_FATAL;  // gRPC over TLS is h2 only
  *out = o;
  return SSL_TLSEXT_ERR_OK;
}

const unsigned char kAlpnHttp1[] = {8, 'h', 't', 't', 'p', '/', '1', '.', '1'};

int select_http1(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in,
                 unsigned int inlen, void*) {
  unsigned char* o = nullptr;
  if (SSL_select_next_proto(&o, outlen, kAlpnHttp1, sizeof kAlpnHttp1, in, inlen) != OPENSSL_NPN_NEGOTIATED)
    return SSL_TLSEXT_ERR_NOACK;  // proceed without ALPN
  *out = o;
  return SSL_TLSEXT_ERR_OK;
}

}  // namespace

std::shared_ptr<TlsContext> TlsContext::server_http1(const std::string& cert, const std::string& key,
                                                     std::string* err) {
  auto t = server(cert, key, err);
  if (!t) return t;
  t->http1_ = true;
  SSL_CTX_set_alpn_select_cb(t->ctx_, &select_http1, nullptr);
  return t;
}

TlsContext::~TlsContext() {
  if (ctx_) SSL_CTX_free(ctx_);
}

std::shared_ptr<TlsContext> TlsContext::server(const std::string& cert, const std::string& key, std::string* err) {
  auto t = std::shared_ptr<TlsContext>(new TlsContext());
  t->server_ = true;
  t->ctx_ = SSL_CTX_new(TLS_server_method());
  if (!t->ctx_ || SSL_CTX_set_min_proto_version(t->ctx_, TLS1_2_VERSION) != 1 ||
      SSL_CTX_use_certificate_chain_file(t->ctx_, cert.c_str()) != 1 ||
      SSL_CTX_use_PrivateKey_file(t->ctx_, key.c_str(), SSL_FILETYPE_PEM) != 1 ||
      SSL_CTX_check_private_key(t->ctx_) != 1) {
    *err = "TLS server config (" + cert + ", " + key + "): " + ssl_errors();
    return nullptr;
  }
  SSL_CTX_set_mode(t->ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  SSL_CTX_set_alpn_select_cb(t->ctx_, &select_h2, nullptr);
  return t;
}

std::shared_ptr<TlsContext> TlsContext::client(const std::string& ca, const std::string& domain, std::string* err) {
  auto t = std::shared_ptr<TlsContext>(new TlsContext());
  t->domain_ = domain;
  t->ctx_ = SSL_CTX_new(TLS_client_method());
  if (!t->ctx_ || SSL_CTX_set_min_proto_version(t->ctx_, TLS1_2_VERSION) != 1) {
    *err = "TLS client config: " + ssl_errors();
    return nullptr;
  }
  if ((ca.empty() ? SSL_CTX_set_default_verify_paths(t->ctx_) : SSL_CTX_load_verify_locations(t->ctx_, ca.c_str(),
                                                                                                nullptr)) != 1) {
    *err = "TLS CA (" + ca + "): " + ssl_errors();
    return nullptr;
  }
  SSL_CTX_set_verify(t->ctx_, SSL_VERIFY_PEER, nullptr);
  SSL_CTX_set_mode(t->ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  if (SSL_CTX_set_alpn_protos(t->ctx_, kAlpnH2, sizeof kAlpnH2) != 0) {
    *err = "TLS ALPN: " + ssl_errors();
    return nullptr;
  }
  return t;
}

std::shared_ptr<TlsContext> TlsContext::client_http1(const std::string& ca, std::string* err) {
  auto t = std::shared_ptr<TlsContext>(new TlsContext());
  t->http1_ = true;
  t->ctx_ = SSL_CTX_new(TLS_client_method());
  if (!t->ctx_ || SSL_CTX_set_min_proto_version(t->ctx_, TLS1_2_VERSION) != 1) {
    *err = "TLS client config: " + ssl_errors();
    return nullptr;
  }
  if ((ca.empty() ? SSL_CTX_set_default_verify_paths(t->ctx_) : SSL_CTX_load_verify_locations(t->ctx_, ca.c_str(),
                                                                                                nullptr)) != 1) {
    *err = "TLS CA (" + ca + "): " + ssl_errors();
    return nullptr;
  }
  SSL_CTX_set_verify(t->ctx_, SSL_VERIFY_PEER, nullptr);
  SSL_CTX_set_mode(t->ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  return t;
}

TlsConn::TlsConn(std::shared_ptr<TlsContext> ctx, int fd) : ctx_(std::move(ctx)), fd_(fd) {
  ssl_ = SSL_new(ctx_->ctx());
  if (ssl_) SSL_set_fd(ssl_, fd);
}

TlsConn::~TlsConn() {
  if (ssl_) {
    SSL_shutdown(ssl_);  // best effort close_notify; never waits for the peer's
    SSL_free(ssl_);
  }
}

bool TlsConn::wait(int ssl_err, Deadline deadline) {
  short ev = ssl_err == SSL_ERROR_WANT_READ ? POLLIN : ssl_err == SSL_ERROR_WANT_WRITE ? POLLOUT : 0;
  if (!ev) return false;
  for (;;) {
    int ms = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
    if (ms <= 0) return false;
    pollfd p{fd_, ev, 0};
    int r = ::poll(&p, 1, ms);
    if (r < 0 && errno == EINTR) continue;
    return r > 0;
  }
}

bool TlsConn::handshake(const std::string& host, Deadline deadline, std::string* err) {
  if (!ssl_) {
    *err = "SSL_new failed";
    return false;
  }
  if (!ctx_->is_server()) {
    const std::string& name = ctx_->domain().empty() ? host : ctx_->domain();
    SSL_set_tlsext_host_name(ssl_, name.c_str());
    X509_VERIFY_PARAM* vp = SSL_get0_param(ssl_);
    unsigned char ip[16];
    if (inet_pton(AF_INET, name.c_str(), ip) == 1 || inet_pton(AF_INET6, name.c_str(), ip) == 1)
      X509_VERIFY_PARAM_set1_ip_asc(vp, name.c_str());
    else
      SSL_set1_host(ssl_, name.c_str());
  }
  for (;;) {
    ERR_clear_error();
    int r = ctx_->is_server() ? SSL_accept(ssl_) : SSL_connect(ssl_);
    if (r == 1) break;
    int e = SSL_get_error(ssl_, r);
    if ((e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) && wait(e, deadline)) continue;
    *err = std::string("TLS handshake: ") + (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE ? "timed out"
                                                                                                  : ssl_errors());
    return false;
  }
  const unsigned char* proto = nullptr;
  unsigned int plen = 0;
  SSL_get0_alpn_selected(ssl_, &proto, &plen);
  if (ctx_->http1()) return true;
  if (plen != 2 || std::memcmp(proto, "h2", 2) != 0) {
    *err = "TLS peer did not negotiate h2 (ALPN)";
    return false;
  }
  return true;
}

long TlsConn::read(void* buf, size_t n) {
  for (;;) {
    ERR_clear_error();
    int r = SSL_read(ssl_, buf, static_cast<int>(std::min<size_t>(n, 1 << 30)));
    if (r > 0) return r;
    int e = SSL_get_error(ssl_, r);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return 0;
    if (e == SSL_ERROR_SYSCALL && errno == EINTR) continue;
    return -1;
  }
}

bool TlsConn::write_all(const void* buf, size_t n, Deadline deadline) {
  const auto* p = static_cast<const uint8_t*>(buf);
  while (n) {
    ERR_clear_error();
    int r = SSL_write(ssl_, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
    if (r > 0) {
      p += r;
      n -= static_cast<size_t>(r);
      continue;
    }
    int e = SSL_get_error(ssl_, r);
    if ((e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) && wait(e, deadline)) continue;
    if (e == SSL_ERROR_SYSCALL && errno == EINTR) continue;
    return false;
  }
  return true;
}

bool TlsConn::pending() const { return ssl_ && SSL_pending(ssl_) > 0; }

}  // namespace dfs
