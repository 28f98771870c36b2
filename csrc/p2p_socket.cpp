// Host-memory P2PTransport over abstract UNIX stream sockets (contract in p2p_transport.h).
//
// Each directed channel (`channels` per direction of a pair) is one connected socket plus one worker thread that executes the
// channel's posted ops strictly in post order (send: write the bytes; recv: read exactly
// the posted size) — the same FIFO matching rule as an RCCL p2p communicator. A "dropped"
// send (debug hook) wedges the channel exactly like an RCCL send whose receive is never
// posted: it and everything behind it stay pending until close().
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
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
  SocketTransport(int rank, std::string ns, int channels) : rank_(rank), ns_(std::move(ns)), channels_(channels) {}
  ~SocketTransport() override {
    std::vector<int> peers;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : links_) peers.push_back(kv.first);
    }
    for (int p : peers) close(p);
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : listeners_)
      for (int fd : kv.second) ::close(fd);
  }

  const char* name() const override { return "socket"; }
  bool device_buffers() const override { return false; }
  int channels() const override { return channels_; }

  // one listening socket per channel of our direction; the token is their names, one a line
  std::string make_token(int peer, uint64_t gen, std::string* err) override {
    static std::atomic<uint64_t> nonce{std::random_device{}()};
    std::string tok;
    std::vector<int> fds;
    for (int ch = 0; ch < channels_; ++ch) {
      std::string name = "dfs_p2p_" + ns_ + "_" + std::to_string(rank_) + "_" + std::to_string(peer) + "_" +
                         std::to_string(gen) + "_" + std::to_string(ch) + "_" + std::to_string(nonce.fetch_add(1));
      int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
      sockaddr_un a;
      socklen_t len = abstract_addr(name, &a);
      if (fd < 0 || ::bind(fd, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(fd, 4) != 0) {
        *err = std::string("p2p listen: ") + std::strerror(errno);
        if (fd >= 0) ::close(fd);
        for (int f : fds) ::close(f);
        return {};
      }
      fds.push_back(fd);
      tok += (ch ? "\n" : "") + name;
    }
    std::lock_guard<std::mutex> g(mu_);
    auto it = listeners_.find(peer);
    if (it != listeners_.end())
      for (int fd : it->second) ::close(fd);
    listeners_[peer] = std::move(fds);
    return tok;
  }

  bool open(int peer, uint64_t, const std::string& tok_out, const std::string& tok_in, int timeout_ms,
            std::string* err) override {
    close(peer);
    std::vector<int> lfds;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = listeners_.find(peer);
      if (it == listeners_.end()) {
        *err = "no listener for our channel token " + tok_out;
        return false;
      }
      lfds = std::move(it->second);
      listeners_.erase(it);
    }
    std::vector<std::string> in_names;
    for (size_t pos = 0;;) {
      size_t nl = tok_in.find('\n', pos);
      in_names.push_back(tok_in.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos));
      if (nl == std::string::npos) break;
      pos = nl + 1;
    }
    auto fail = [&](const std::string& e, std::vector<int>& opened) {
      for (int fd : lfds) ::close(fd);
      for (int fd : opened) ::close(fd);
      *err = e;
      return false;
    };
    std::vector<int> in_fds, out_fds;
    if (static_cast<int>(in_names.size()) != channels_ || static_cast<int>(lfds.size()) != channels_)
      return fail("p2p peers disagree on the channel count", in_fds);
    auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    // connect to every listener of the peer first (a listening socket accepts the connection
    // into its backlog before accept()), then accept ours: both ranks do the same, no wait cycle
    for (const auto& nm : in_names) {
      int in_fd = -1;
      while (in_fd < 0) {
        int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
        sockaddr_un a;
        socklen_t len = abstract_addr(nm, &a);
        if (fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr*>(&a), len) == 0) {
          in_fd = fd;
          break;
        }
        if (fd >= 0) ::close(fd);
        if (Clock::now() > deadline) return fail("p2p connect to " + nm + " timed out", in_fds);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
      in_fds.push_back(in_fd);
    }
    for (int lfd : lfds) {
      int out_fd = -1;
      int left = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count());
      pollfd p{lfd, POLLIN, 0};
      if (left > 0 && ::poll(&p, 1, left) > 0) out_fd = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (out_fd < 0) {
        for (int fd : out_fds) ::close(fd);
        return fail("p2p accept for " + tok_out + " timed out", in_fds);
      }
      out_fds.push_back(out_fd);
    }
    for (int fd : lfds) ::close(fd);
    auto link = std::make_shared<Link>();
    for (int ch = 0; ch < channels_; ++ch) {
      for (int dir = 0; dir < 2; ++dir) {
        auto c = std::make_unique<Chan>();
        c->fd = dir == 0 ? out_fds[ch] : in_fds[ch];
        c->send = dir == 0;
        c->link = link.get();
        (dir == 0 ? link->out : link->in).push_back(std::move(c));
      }
    }
    for (auto* v : {&link->out, &link->in})
      for (auto& c : *v) c->worker = std::thread([cp = c.get()] { run(cp); });
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
    for (auto* v : {&l->out, &l->in})
      for (auto& c : *v) {
        {
          std::lock_guard<std::mutex> g(c->mu);
          c->stop = true;
        }
        ::shutdown(c->fd, SHUT_RDWR);
        c->cv.notify_all();
      }
    for (auto* v : {&l->out, &l->in})
      for (auto& c : *v) {
        if (c->worker.joinable()) c->worker.join();
        ::close(c->fd);
        for (auto& op : c->q) op.st->store(-1);  // never executed
        c->q.clear();
      }
  }

  bool post_send(int peer, int ch, const void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, ch, true, const_cast<void*>(buf), n, op, err);
  }
  bool post_recv(int peer, int ch, void* buf, uint64_t n, P2POp* op, std::string* err) override {
    return post(peer, ch, false, buf, n, op, err);
  }
  int test(P2POp* op) override { return op->state ? op->state->load() : -1; }
  void release(P2POp* op) override { op->state.reset(); }

  // the next `n` sends to the peer vanish, whichever channel carries them
  void debug_drop_sends(int peer, int n) override {
    if (auto l = find(peer)) l->drop += n;
  }
  void debug_stall(int peer, int ms) override {
    if (auto l = find(peer)) l->stall_ms = ms;
  }

 private:
  struct Op {
    uint8_t* buf;
    uint64_t n;
    std::shared_ptr<std::atomic<int>> st;
  };
  struct Link;
  struct Chan {
    int fd = -1;
    bool send = false;
    Link* link = nullptr;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Op> q;
    bool stop = false;
    std::thread worker;
  };
  struct Link {
    std::vector<std::unique_ptr<Chan>> out, in;  // one per channel
    std::atomic<int> drop{0}, stall_ms{0};        // test hooks, shared by the out channels
  };

  std::shared_ptr<Link> find(int peer) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = links_.find(peer);
    return it == links_.end() ? nullptr : it->second;
  }

  bool post(int peer, int ch, bool send, void* buf, uint64_t n, P2POp* op, std::string* err) {
    auto l = find(peer);
    if (!l) {
      *err = "p2p channel down";
      return false;
    }
    if (ch < 0 || ch >= channels_) {
      *err = "p2p channel out of range";
      return false;
    }
    Chan& c = send ? *l->out[ch] : *l->in[ch];
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
        int d = c->send ? c->link->drop.load() : 0;
        if (d > 0 && c->link->drop.compare_exchange_strong(d, d - 1)) {
          // the send "vanishes": it and every later op of this channel stay pending
          wedged = true;
          continue;
        }
        op = c->q.front();
        c->q.pop_front();
        if (c->send) stall = c->link->stall_ms.exchange(0);
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
  int channels_;
  std::mutex mu_;
  std::map<int, std::shared_ptr<Link>> links_;
  std::map<int, std::vector<int>> listeners_;  // peer -> listening fds of our pending out-channel token
};

}  // namespace

std::unique_ptr<P2PTransport> make_socket_transport(int rank, const std::string& ns, int channels) {
  return std::make_unique<SocketTransport>(rank, ns, std::max(1, std::min(channels, kMaxP2PChannels)));
}

}  // namespace dfs
