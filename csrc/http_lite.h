// Small HTTP/1.1 server and client for the control-plane processes' side channel: /health,
// /metrics, /raft/state, the Raft peer endpoints /raft/{vote,append,snapshot,timeout_now},
// /shard_map, /debug/* (reference bin/master.rs:186-226 and bin/config_server.rs:120-160
// serve the same routes over axum). Requests and replies carry Content-Length bodies
// (no chunked transfer); connections are kept alive; one thread per connection, since
// a Raft handler may block on the node for a while and the peers of a shard are few.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

struct HttpRequest {
  std::string method, path, query, body;
  std::map<std::string, std::string> headers;  // lower-cased names
};

struct HttpResponse {
  int status = 200;
  std::string content_type = "text/plain";
  std::string body;
};

class HttpLiteServer {
 public:
  using Handler = std::function<HttpResponse(const HttpRequest&)>;
  HttpLiteServer(std::string host, int port, Handler handler);
  ~HttpLiteServer();
  HttpLiteServer(const HttpLiteServer&) = delete;
  bool start(std::string* err);
  void stop();
  int port() const { return port_; }

 private:
  void accept_loop();
  void serve(int fd);
  std::string host_;
  int port_;
  Handler handler_;
  int lfd_ = -1;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::set<int> conns_;
  struct Worker {
    std::thread t;
    std::shared_ptr<std::atomic<bool>> done;
  };
  std::vector<Worker> workers_;  // finished ones are joined on the next accept
};

// One request over a fresh connection (control-plane traffic is sparse; the Raft data path
// uses the native HTTP/2 peer transport). `url` = http://host:port/path. Returns the HTTP
// status (0 on a transport failure or timeout, with *err set).
int http_request(const std::string& method, const std::string& url, const std::string& body,
                 const std::string& content_type, int timeout_ms, std::string* reply, std::string* err = nullptr);

}  // namespace dfs
