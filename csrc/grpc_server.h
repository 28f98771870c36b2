// Minimal native gRPC server: unary RPCs over HTTP/2 on nghttp2 — h2c (prior knowledge), or
// TLS with ALPN h2 when set_tls() is given the server's certificate (tls.h).
//
// grpc++ is not in this toolchain, nghttp2 is. The wire is plain gRPC —
// HEADERS (:path /dfs.<Service>/<Method>, content-type application/grpc, te: trailers), one
// length-prefixed message in DATA, and grpc-status / grpc-message trailers — so reference
// clients (tonic) and Python grpcio talk to it unchanged (tests/test_native_grpc.py).
//
// Threading: one thread per connection owns its nghttp2 session (the library is not
// thread-safe); complete requests are handed to a worker pool, so the many concurrent streams
// a pooled client channel multiplexes run in parallel; finished responses come back to the
// connection thread through an eventfd. Flow-control windows are opened wide (64 MiB per
// stream, 1 GiB per connection) so a 1-100 MiB block never waits on WINDOW_UPDATE round trips.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

class TlsContext;

struct GrpcCall {
  std::string path;        // "/dfs.ChunkServerService/WriteBlock"
  std::string request_id;  // x-request-id metadata ("" if absent)
  std::string message;     // the serialized request (empty when `body` is set)
  // A large request received into a buffer from the server's body allocator (registered
  // host memory on a chunkserver) instead of `message`; `body_keep` owns it.
  const uint8_t* body = nullptr;
  size_t body_len = 0;
  std::shared_ptr<const void> body_keep;
  const uint8_t* data() const { return body ? body : reinterpret_cast<const uint8_t*>(message.data()); }
  size_t size() const { return body ? body_len : message.size(); }
};

struct GrpcReply {
  int status = 0;          // grpc status code
  std::string message;     // serialized response (status 0) or grpc-message text
  // status 0 alternative to `message`: the serialized response lives in a buffer the
  // handler owns (e.g. registered memory a GPU read landed in); `keep` holds it until the
  // last byte is handed to nghttp2
  std::shared_ptr<const void> keep;
  const uint8_t* ext = nullptr;
  size_t ext_len = 0;
};

class GrpcServer {
 public:
  using Handler = std::function<GrpcReply(const GrpcCall&)>;
  GrpcServer(std::string host, int port, Handler handler, int workers = 32);
  ~GrpcServer();
  GrpcServer(const GrpcServer&) = delete;
  // Serve TLS (ALPN h2) instead of h2c; call before start().
  void set_tls(std::shared_ptr<TlsContext> tls) { tls_ = std::move(tls); }
  // Requests of at least `min_bytes` are received into buffers from `alloc` (nullptr from it:
  // the default std::string). A chunkserver hands out registered host memory here, so a
  // WriteBlock payload is DMA'd (or copied by the fused write kernel) straight from where
  // the socket put it. Call before start().
  using BodyAlloc = std::function<std::shared_ptr<uint8_t>(size_t n)>;
  void set_body_allocator(BodyAlloc alloc, size_t min_bytes) {
    body_alloc_ = std::move(alloc);
    body_min_ = min_bytes;
  }
  bool start(std::string* err);
  void stop();
  int port() const { return port_; }
  bool tls() const { return tls_ != nullptr; }
  uint64_t calls() const { return calls_.load(); }

 private:
  struct Conn;
  void accept_loop();
  void serve(int fd);
  void worker_loop();

  std::string host_;
  int port_;
  Handler handler_;
  BodyAlloc body_alloc_;
  size_t body_min_ = 0;
  int nworkers_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> jobs_;
  std::vector<int> conns_;
  int live_conns_ = 0;
  std::condition_variable conns_cv_;
  std::atomic<uint64_t> calls_{0};
  std::shared_ptr<TlsContext> tls_;
};

}  // namespace dfs
