// Minimal native gRPC client: unary calls over HTTP/2 (h2c, or TLS + ALPN h2) on nghttp2 —
// the client half of grpc_server.h, used by the native remote client (client_remote.h).
//
// One call owns one connection for its duration (connections are pooled per target and
// reused, so a client with C concurrent calls keeps C connections per server). Windows are
// opened wide (64 MiB per stream, 1 GiB per connection) and we accept 1 MiB frames, so a
// 1-100 MiB block moves without WINDOW_UPDATE round trips. A transport error or a timeout
// drops the connection; the caller sees transport_ok == false and may retry elsewhere.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace dfs {

class TlsContext;

struct GrpcResult {
  bool transport_ok = false;  // false: connect / protocol / timeout failure (no status)
  int status = -1;            // grpc status code
  std::string message;        // serialized response (status 0) or grpc-message text
};

class GrpcChannelPool {
 public:
  // `tls`: client TLS context (https targets, ALPN h2); nullptr = h2c.
  explicit GrpcChannelPool(int timeout_ms = 120000, std::shared_ptr<TlsContext> tls = nullptr);
  ~GrpcChannelPool();
  GrpcChannelPool(const GrpcChannelPool&) = delete;
  GrpcChannelPool& operator=(const GrpcChannelPool&) = delete;

  // `target`: "host:port" or "http://host:port"; `path`: "/dfs.Service/Method".
  GrpcResult call(const std::string& target, const std::string& path, const std::string& request,
                  const std::string& request_id, int timeout_ms = -1);
  uint64_t connects() const;
  // Host aliases (the client library's add_host_alias): a target containing `alias` is
  // dialled at `real` instead (first match, as client.py resolve_url).
  void set_host_aliases(std::vector<std::pair<std::string, std::string>> aliases);

 private:
  std::string resolve(const std::string& target) const;
  struct Conn;
  std::unique_ptr<Conn> take(const std::string& target, int timeout_ms, std::string* err);
  void give(const std::string& target, std::unique_ptr<Conn> c);

  int timeout_ms_;
  std::shared_ptr<TlsContext> tls_;
  mutable std::mutex mu_;
  std::map<std::string, std::vector<std::unique_ptr<Conn>>> idle_;
  std::vector<std::pair<std::string, std::string>> aliases_;  // mu_
  uint64_t connects_ = 0;
};

}  // namespace dfs
