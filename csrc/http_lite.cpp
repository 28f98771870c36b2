// HTTP/1.1 side channel of the control-plane processes (see http_lite.h).
#include "http_lite.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>

namespace dfs {

namespace {

constexpr size_t kMaxHeader = 64 << 10;
constexpr size_t kMaxBody = 1ull << 30;  // snapshots travel here

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t\r");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// Reads until `buf` holds at least `want` bytes; false on EOF / error / timeout.
bool fill(int fd, std::string& buf, size_t want, int timeout_ms) {
  char tmp[65536];
  while (buf.size() < want) {
    pollfd p{fd, POLLIN, 0};
    int r = ::poll(&p, 1, timeout_ms);
    if (r <= 0) return false;
    ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    buf.append(tmp, static_cast<size_t>(n));
  }
  return true;
}

// Reads one header block (through the blank line) into *head; the bytes after it stay in buf.
bool read_head(int fd, std::string& buf, std::string* head, int timeout_ms) {
  for (;;) {
    size_t e = buf.find("\r\n\r\n");
    if (e != std::string::npos) {
      *head = buf.substr(0, e);
      buf.erase(0, e + 4);
      return true;
    }
    if (buf.size() > kMaxHeader || !fill(fd, buf, buf.size() + 1, timeout_ms)) return false;
  }
}

bool send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    off += static_cast<size_t>(n);
  }
  return true;
}

void parse_headers(const std::string& head, size_t from, std::map<std::string, std::string>* out) {
  size_t pos = from;
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string::npos) e = head.size();
    std::string line = head.substr(pos, e - pos);
    size_t c = line.find(':');
    if (c != std::string::npos) (*out)[lower(trim(line.substr(0, c)))] = trim(line.substr(c + 1));
    pos = e + 2;
  }
}

const char* reason(int status) {
  switch (status) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

}  // namespace

HttpLiteServer::HttpLiteServer(std::string host, int port, Handler handler)
    : host_(std::move(host)), port_(port), handler_(std::move(handler)) {}

HttpLiteServer::~HttpLiteServer() { stop(); }

bool HttpLiteServer::start(std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  const std::string h = host_ == "localhost" ? "127.0.0.1" : host_;
  if (::getaddrinfo(h.empty() ? nullptr : h.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res) {
    *err = "cannot resolve " + host_;
    return false;
  }
  lfd_ = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  bool ok = lfd_ >= 0 && ::bind(lfd_, res->ai_addr, res->ai_addrlen) == 0 && ::listen(lfd_, 128) == 0;
  ::freeaddrinfo(res);
  if (!ok) {
    *err = "http bind " + host_ + ":" + std::to_string(port_) + ": " + std::strerror(errno);
    if (lfd_ >= 0) ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  sockaddr_storage sa{};
  socklen_t sl = sizeof(sa);
  if (::getsockname(lfd_, reinterpret_cast<sockaddr*>(&sa), &sl) == 0)
    port_ = ntohs(sa.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&sa)->sin6_port
                                           : reinterpret_cast<sockaddr_in*>(&sa)->sin_port);
  running_ = true;
  acceptor_ = std::thread([this] { accept_loop(); });
  return true;
}

void HttpLiteServer::stop() {
  if (!running_.exchange(false)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  std::vector<Worker> ws;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    ws.swap(workers_);
  }
  for (auto& w : ws)
    if (w.t.joinable()) w.t.join();
}

void HttpLiteServer::accept_loop() {
  while (running_) {
    pollfd p{lfd_, POLLIN, 0};
    if (::poll(&p, 1, 200) <= 0) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = workers_.begin(); it != workers_.end();) {
      if (it->done->load()) {
        it->t.join();
        it = workers_.erase(it);
      } else {
        ++it;
      }
    }
    conns_.insert(fd);
    auto done = std::make_shared<std::atomic<bool>>(false);
    workers_.push_back(Worker{std::thread([this, fd, done] {
                                serve(fd);
                                done->store(true);
                              }),
                              done});
  }
}

void HttpLiteServer::serve(int fd) {
  std::string buf;
  while (running_) {
    std::string head;
    if (!read_head(fd, buf, &head, 60000)) break;
    HttpRequest req;
    size_t e = head.find("\r\n");
    std::string line = head.substr(0, e);
    size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) break;
    req.method = line.substr(0, s1);
    std::string target = line.substr(s1 + 1, s2 - s1 - 1);
    size_t q = target.find('?');
    req.path = target.substr(0, q);
    if (q != std::string::npos) req.query = target.substr(q + 1);
    parse_headers(head, e == std::string::npos ? head.size() : e + 2, &req.headers);
    size_t len = 0;
    auto it = req.headers.find("content-length");
    if (it != req.headers.end()) len = std::strtoull(it->second.c_str(), nullptr, 10);
    if (len > kMaxBody || !fill(fd, buf, len, 60000)) break;
    req.body = buf.substr(0, len);
    buf.erase(0, len);
    HttpResponse r;
    try {
      r = handler_(req);
    } catch (const std::exception& ex) {
      r.status = 500;
      r.body = "Internal server error";
    }
    const bool close = lower(req.headers["connection"]) == "close";
    std::string out = "HTTP/1.1 " + std::to_string(r.status) + " " + reason(r.status) + "\r\nContent-Type: " +
                      r.content_type + "\r\nContent-Length: " + std::to_string(r.body.size()) +
                      (close ? "\r\nConnection: close" : "") + "\r\n\r\n";
    out += r.body;
    if (!send_all(fd, out) || close) break;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    conns_.erase(fd);
  }
  ::close(fd);
}

int http_request(const std::string& method, const std::string& url, const std::string& body,
                 const std::string& content_type, int timeout_ms, std::string* reply, std::string* err) {
  std::string e_;
  std::string& e = err ? *err : e_;
  std::string rest = url;
  if (rest.compare(0, 7, "http://") == 0) rest = rest.substr(7);
  else if (rest.find("://") != std::string::npos) return (e = "unsupported scheme: " + url, 0);
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash), path = slash == std::string::npos ? "/" : rest.substr(slash);
  size_t colon = hostport.rfind(':');
  std::string host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  std::string port = colon == std::string::npos ? "80" : hostport.substr(colon + 1);
  if (host == "localhost") host = "127.0.0.1";
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return (e = "cannot resolve " + host, 0);
  int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) {
    ::freeaddrinfo(res);
    return (e = std::strerror(errno), 0);
  }
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    e = std::string("connect: ") + std::strerror(errno);
    ::close(fd);
    return 0;
  }
  pollfd p{fd, POLLOUT, 0};
  int so = 0;
  socklen_t sl = sizeof(so);
  if (rc != 0 && (::poll(&p, 1, timeout_ms) <= 0 || ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl) != 0 || so)) {
    e = std::string("connect: ") + (so ? std::strerror(so) : "timeout");
    ::close(fd);
    return 0;
  }
  ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) & ~O_NONBLOCK);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + hostport + "\r\nConnection: close\r\n";
  if (!body.empty() || method == "POST" || method == "PUT")
    req += "Content-Type: " + content_type + "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  req += "\r\n";
  req += body;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  auto left = [&] {
    return static_cast<int>(std::max<int64_t>(
        1, std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count()));
  };
  std::string buf, head;
  int status = 0;
  if (!send_all(fd, req) || !read_head(fd, buf, &head, left())) {
    e = "request to " + url + " failed";
  } else {
    size_t sp = head.find(' ');
    status = sp == std::string::npos ? 0 : std::atoi(head.c_str() + sp + 1);
    std::map<std::string, std::string> hs;
    size_t eol = head.find("\r\n");
    parse_headers(head, eol == std::string::npos ? head.size() : eol + 2, &hs);
    auto it = hs.find("content-length");
    if (it != hs.end()) {
      size_t len = std::strtoull(it->second.c_str(), nullptr, 10);
      if (!fill(fd, buf, len, left())) {
        e = "short reply from " + url;
        status = 0;
      } else {
        buf.resize(len);
      }
    } else {
      while (fill(fd, buf, buf.size() + 1, left())) {
      }
    }
    if (reply) *reply = std::move(buf);
  }
  ::close(fd);
  return status;
}

}  // namespace dfs
