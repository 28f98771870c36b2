#include "localrpc.h"

#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <cstddef>
#include <cstring>

namespace dfs {

namespace {

bool read_full(int fd, void* buf, size_t n) {
  auto* p = static_cast<char*>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool write_full(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

}  // namespace

LocalRpcServer::LocalRpcServer(std::string name, Handler handler) : name_(std::move(name)), handler_(std::move(handler)) {}

LocalRpcServer::~LocalRpcServer() { stop(); }

bool LocalRpcServer::start(std::string* err) {
  lfd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) {
    *err = std::string("socket: ") + std::strerror(errno);
    return false;
  }
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  if (name_.size() + 1 > sizeof(sa.sun_path)) {
    *err = "socket name too long";
    return false;
  }
  std::memcpy(sa.sun_path + 1, name_.data(), name_.size());  // abstract namespace
  socklen_t len = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name_.size());
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&sa), len) != 0 || ::listen(lfd_, 128) != 0) {
    *err = std::string("bind/listen ") + name_ + ": " + std::strerror(errno);
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  running_ = true;
  acceptor_ = std::thread([this] { accept_loop(); });
  return true;
}

void LocalRpcServer::stop() {
  if (!running_.exchange(false)) return;
  ::shutdown(lfd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  ::close(lfd_);
  lfd_ = -1;
  std::vector<std::thread> workers;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    workers.swap(workers_);
  }
  for (auto& t : workers)
    if (t.joinable()) t.join();
}

void LocalRpcServer::accept_loop() {
  while (running_) {
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR) continue;
      if (!running_) return;
      continue;
    }
    // The abstract namespace has no file permissions: only processes of our own user (or
    // root) may skip the network listener — which is what keeps a TLS deployment's metadata
    // traffic off plaintext sockets for anyone else on the host.
    ucred cred{};
    socklen_t cl = sizeof(cred);
    if (::getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cred, &cl) != 0 || (cred.uid != ::geteuid() && cred.uid != 0)) {
      ::close(fd);
      continue;
    }
    std::lock_guard<std::mutex> g(mu_);
    if (!running_) {
      ::close(fd);
      return;
    }
    conns_.insert(fd);
    workers_.emplace_back([this, fd] { serve(fd); });
  }
}

void LocalRpcServer::serve(int fd) {
  std::string body, out, path, rid, payload, resp;
  for (;;) {
    uint32_t n;
    if (!read_full(fd, &n, 4) || n < 4 || n > (1u << 30)) break;
    body.resize(n);
    if (!read_full(fd, body.data(), n)) break;
    uint16_t pl, rl;
    std::memcpy(&pl, body.data(), 2);
    if (2u + pl + 2u > n) break;
    path.assign(body, 2, pl);
    std::memcpy(&rl, body.data() + 2 + pl, 2);
    if (4u + pl + rl > n) break;
    rid.assign(body, 4 + pl, rl);
    payload.assign(body, 4 + pl + rl, std::string::npos);
    out.clear();
    int code;
    try {
      code = handler_(path, rid, payload, &out);
    } catch (const std::exception& e) {
      code = 13;  // INTERNAL
      out = e.what();
    }
    requests_++;
    uint32_t len = static_cast<uint32_t>(out.size() + 1);
    resp.assign(reinterpret_cast<const char*>(&len), 4);
    resp.push_back(static_cast<char>(code));
    resp += out;
    if (!write_full(fd, resp.data(), resp.size())) break;
  }
  std::lock_guard<std::mutex> g(mu_);
  conns_.erase(fd);
  ::close(fd);
}

}  // namespace dfs
