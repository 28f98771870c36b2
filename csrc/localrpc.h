// Same-host RPC listener of the metadata services (native side of utils/localrpc.py).
//
// A Python gRPC round trip costs ~350 µs of HTTP/2 + grpc-core work per side, which
// dominates metadata latency when the client and the master share a node (every GPU rank
// of the benchmark has its own co-located metadata shard). Servers therefore also listen
// on an abstract UNIX socket named after their TCP port and speak a minimal framing of
// the *same* protobuf messages:
//     request  = u32 body_len | u16 len, path "/dfs.Service/Method" | u16 len, request id | payload
//     response = u32 body_len | u8 grpc status code | payload (OK) or utf-8 status message
// One thread per connection (clients keep a few persistent connections); the handler runs
// on that thread and may block on a Raft commit without stalling other connections.
#pragma once
#include <atomic>
#include <functional>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

class LocalRpcServer {
 public:
  // (path, request id, payload, *out) -> grpc status code; *out = response or message
  using Handler = std::function<int(const std::string&, const std::string&, const std::string&, std::string*)>;

  LocalRpcServer(std::string name, Handler handler);
  ~LocalRpcServer();
  bool start(std::string* err);
  void stop();
  const std::string& name() const { return name_; }
  uint64_t requests() const { return requests_.load(); }

 private:
  void accept_loop();
  void serve(int fd);

  std::string name_;
  Handler handler_;
  int lfd_ = -1;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> requests_{0};
  std::thread acceptor_;
  std::mutex mu_;
  std::set<int> conns_;
  std::vector<std::thread> workers_;
};

}  // namespace dfs
