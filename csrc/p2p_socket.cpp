// Host-memory P2PTransport over abstract UNIX stream sockets (contract in p2p_transport.h).
//
// Each directed channel is one connected socket plus one worker thread that executes the
// channel's posted ops strictly in post order (send: write the bytes; recv: read exactly
// the posted size) — the same FIFO matching rule as an RCCL p2p communicator. A "dropped"
// send (debug hook) wedges the channel exactly like an RCCL send whose receive is never
// posted: it and everything behind it stay pending until close().
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <thread>

#include "p2p_transport.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;

socklen_t abstract_addr(const std::string& name, sockaddr_un* a) {
  std::memset(a, 0, sizeof(*a));
  a->sun_family = AF_UNIX;
  size_t n = std::min(name.size(), sizeof(a->sun_path) - 2);
  std::memcpy(a->sun_path + 1, name.data(), n);
  return static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + n);
}

bool io_full(int fd, uint8_t* p, uint64_t n, bool send) {
  while (n > 0) {
    ssize_t r = send ? ::send(fd, p, n, MSG_NOSIGNAL) : ::recv(fd, p, n, 0);
    if (r > 0) {
      p += r;
      n -= static_cast<uint64_t>(r);
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

class SocketTransport final : public P2PTransport {
 public:
  SocketTransport(int rank, std::string ns) : rank_(rank), ns_(std::move(ns)) {}
  ~SocketTransport() override {
    std::vector<int> peers;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : links_) peers.push_back(kv.first);
    }
    for (int p : peers) close(p);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : listeners_) ::close(kv.second);
  }

  const char* name() const override { return "socket"; }
  bool device_buffers() const override { return false; }

  std::string make_token(int peer, uint64_t gen, std::string* err) override {
    static std::atomic<uint64_t> nonce{std::random_device{}()};
    std::string name = "dfs_p2p_" + ns_ + "_" + std::to_string(rank_) + "_" + std::to_string(peer) + "_" +
                       std::to_string(gen) + "_" + std::to_string(nonce.fetch_add(1));
    int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    socklen_t len = abstract_addr(name, &a);
    if (fd < 0 || ::bind(fd, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(fd, 4) != 0) {
      *err = std::string("p2p listen: ") + std::strerror(errno);
      if (fd >= 0) ::close(fd);
      return {};
    }
    std::lock_guard<std::mutex> g(mu_);
    auto it = listeners_.find(peer);
    if (it != listeners_.end()) ::close(it->second);
    listeners_[peer] = fd;
    return name;
  }

  bool open(int peer, uint64_t, const std::string& tok_out, const std::string& tok_in, int timeout_ms,
            std::string* err) override {
    close(peer);
    int lfd = -1;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = listeners_.find(peer);
      if (it == listeners_.end()) {
        *err = "no listener for our channel token " + tok_out;
        return false;
      }
      lfd = it->second;
      listeners_.erase(it);
    }
    auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    // connect to the peer's listener first (a listening socket accepts the connection into
    // its backlog before accept()), then accept ours: both ranks do the same, no wait cycle
    int in_fd = -1;
    while (in_fd < 0) {
      int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
      sockaddr_un a;
      socklen_t len = abstract_addr(tok_in, &a);
      if (fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr*>(&a), len) == 0) {
        in_fd = fd;
        break;
      }
      if (fd >= 0) ::close(fd);
      if (Clock::now() > deadline) {
        ::close(lfd);
        *err = "p2p connect to " + tok_in + " timed out";
        return false;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    int out_fd = -1;
    for (;;) {
      int left = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
      pollfd p{lfd, POLLIN, 0};
      if (left <= 0 || ::poll(&p, 1, left) <= 0) break;
      out_fd = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      break;
    }
    ::close(lfd);
    if (out_fd < 0) {
      ::close(in_fd);
      *err = "p2p accept for " + tok_out + " timed out";
      return false;
    }
    auto link = std::make_shared<Link>();
    link->out.fd = out_fd;
    link->in.fd = in_fd;
    link->out.send = true;
    link->out.worker = std::thread([c = &link->out] { run(c); });
    link->in.worker = std::thread([c = &link->in] { run(c); });
    std::lock_guard<std::mutex> g(mu_);
    links_[peer] = std::move(link);
    return true;
  }

  void close(int peer) override {
    std::shared_ptr<Link> l;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = links_.find(peer);
      if (it == links_.end()) return;
      l = it->second;
      links_.erase(it);
    }
    for (Chan* c : {&l->out, &l->in}) {
      {
        std::lock_guard<std::mutex> g(c->mu);
        c->stop = true;
      }
      ::shutdown(c->fd, SHUT_RDWR);
      c->cv.notify_all();
    }
    for (Chan* c : {&l->out, &l->in}) {
      if (c->worker.joinable()) c->worker.join();
      ::close(c->fd);
      for (auto& op : c->q) op.st->store(-1);  // never executed
      c->q.clear();
    }
  }

  bool post_send(int peer, const void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, true, const_cast<void*>(buf), n, op, err);
  }
  bool post_recv(int peer, void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, false, buf, n, op, err);
  }
  int test(P2POp* op) override { return op->state ? op->state->load() : -1; }
  void release(P2POp* op) override { op->state.reset(); }

  void debug_drop_sends(int peer, int n) override {
    if (auto l = find(peer)) {
      std::lock_guard<std::mutex> g(l->out.mu);
      l->out.drop += n;
    }
  }
  void debug_stall(int peer, int ms) override {
    if (auto l = find(peer)) {
      std::lock_guard<std::mutex> g(l->out.mu);
      l->out.stall_ms = ms;
    }
  }

 private:
  struct Op {
    uint8_t* buf;
    uint64_t n;
    std::shared_ptr<std::atomic<int>> st;
  };
  struct Chan {
    int fd = -1;
    bool send = false;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Op> q;
    bool stop = false;
    int drop = 0;
    int stall_ms = 0;
    std::thread worker;
  };
  struct Link {
    Chan out, in;
  };

  std::shared_ptr<Link> find(int peer) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = links_.find(peer);
    return it == links_.end() ? nullptr : it->second;
  }

  bool post(int peer, bool send, void* buf, uint64_t n, P2POp* op, std::string* err) {
    auto l = find(peer);
    if (!l) {
      *err = "p2p channel down";
      return false;
    }
    Chan& c = send ? l->out : l->in;
    op->state = std::make_shared<std::atomic<int>>(0);
    std::lock_guard<std::mutex> g(c.mu);
    if (c.stop) {
      *err = "p2p channel closed";
      return false;
    }
    c.q.push_back(Op{static_cast<uint8_t*>(buf), n, op->state});
    c.cv.notify_all();
    return true;
  }

  static void run(Chan* c) {
    bool wedged = false;
    for (;;) {
      Op op;
      int stall = 0;
      {
        std::unique_lock<std::mutex> lk(c->mu);
        c->cv.wait(lk, [&] { return c->stop || (!wedged && !c->q.empty()); });
        if (c->stop) return;
        if (c->send && c->drop > 0) {
          // the send "vanishes": it and every later op of this channel stay pending
          c->drop--;
          wedged = true;
          continue;
        }
        op = c->q.front();
        c->q.pop_front();
        stall = c->stall_ms;
        c->stall_ms = 0;
      }
      if (stall) std::this_thread::sleep_for(std::chrono::milliseconds(stall));
      bool ok = io_full(c->fd, op.buf, op.n, c->send);
      op.st->store(ok ? 1 : -1);
      if (!ok) {
        std::lock_guard<std::mutex> g(c->mu);
        for (auto& o : c->q) o.st->store(-1);
        c->q.clear();
        c->stop = true;
        return;
      }
    }
  }

  int rank_;
  std::string ns_;
  std::mutex mu_;
  std::map<int, std::shared_ptr<Link>> links_;
  std::map<int, int> listeners_;  // peer -> listening fd of our pending out-channel token
};

}  // namespace

std::unique_ptr<P2PTransport> make_socket_transport(int rank, const std::string& ns) {
  return std::make_unique<SocketTransport>(rank, ns);
}

}  // namespace dfs
