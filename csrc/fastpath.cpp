// Native local data path of a ChunkServer; see fastpath.h for protocol and scope.
#include "fastpath.h"
#include "gf256.h"
#include "trace.h"
#include "thread_name.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <future>

namespace dfs {

namespace {

constexpr uint32_t kMaxBody = 1 << 16;
// Largest single transfer the fast path accepts (the reference caps gRPC messages, and so
// blocks, at 100 MiB: dfs/chunkserver/src/chunkserver.rs:15; large-object extents stay below).
constexpr uint64_t kMaxTransfer = 1ull << 30;
constexpr const char* kShmDir = "/dev/shm/";
constexpr const char* kShmPrefix = "dfs_sc_";

bool read_full(int fd, void* buf, size_t n) {
  auto* p = static_cast<uint8_t*>(buf);
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r > 0) {
      p += r;
      n -= static_cast<size_t>(r);
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

bool write_full(int fd, const void* buf, size_t n) {
  const auto* p = static_cast<const uint8_t*>(buf);
  while (n > 0) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r > 0) {
      p += r;
      n -= static_cast<size_t>(r);
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <class T>
  T get() {
    T v{};
    if (end - p < static_cast<ptrdiff_t>(sizeof(T))) {
      ok = false;
      return v;
    }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint16_t n = get<uint16_t>();
    if (!ok || end - p < n) {
      ok = false;
      return {};
    }
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
};

bool send_response(int fd, FpStatus st, uint64_t total, uint64_t bytes, const std::string& msg) {
  std::string m = msg.size() > 4000 ? msg.substr(0, 4000) : msg;
  uint32_t body = static_cast<uint32_t>(1 + 8 + 8 + 2 + m.size());
  std::vector<uint8_t> out(4 + body);
  uint8_t* q = out.data();
  std::memcpy(q, &body, 4);
  q[4] = static_cast<uint8_t>(st);
  std::memcpy(q + 5, &total, 8);
  std::memcpy(q + 13, &bytes, 8);
  uint16_t ml = static_cast<uint16_t>(m.size());
  std::memcpy(q + 21, &ml, 2);
  std::memcpy(q + 23, m.data(), m.size());
  return write_full(fd, out.data(), out.size());
}

void put_str(std::vector<uint8_t>& b, const std::string& s) {
  uint16_t n = static_cast<uint16_t>(s.size());
  const auto* q = reinterpret_cast<const uint8_t*>(&n);
  b.insert(b.end(), q, q + 2);
  b.insert(b.end(), s.begin(), s.end());
}

template <class T>
void put(std::vector<uint8_t>& b, T v) {
  const auto* q = reinterpret_cast<const uint8_t*>(&v);
  b.insert(b.end(), q, q + sizeof(T));
}

std::vector<std::string> read_list(Reader& rd, bool optional) {
  std::vector<std::string> out;
  if (optional && rd.p == rd.end) return out;
  uint16_t n = rd.get<uint16_t>();
  for (uint16_t i = 0; rd.ok && i < n; ++i) out.push_back(rd.str());
  return out;
}

// [off, off+len) inside an object of `size` bytes, without the wrap-around of off+len.
bool range_ok(uint64_t off, uint64_t len, uint64_t size) { return off <= size && len <= size - off; }

bool valid_shm_path(const std::string& path) {
  // only our client arenas: /dev/shm/dfs_sc_<...> with no path tricks
  if (path.rfind(kShmDir, 0) != 0) return false;
  std::string base = path.substr(std::strlen(kShmDir));
  return base.rfind(kShmPrefix, 0) == 0 && base.find('/') == std::string::npos && base.find("..") == std::string::npos;
}

}  // namespace

FastPathServer::FastPathServer(ChunkStore* store, std::string name) : store_(store), name_(std::move(name)) {}

FastPathServer::~FastPathServer() { stop(); }

bool FastPathServer::start(std::string* err) {
  lfd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) {
    *err = std::string("socket: ") + std::strerror(errno);
    return false;
  }
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (name_.size() + 1 >= sizeof(addr.sun_path)) {
    *err = "socket name too long";
    return false;
  }
  // abstract namespace: no filesystem entry to clean up after a crash
  addr.sun_path[0] = '\0';
  std::memcpy(addr.sun_path + 1, name_.data(), name_.size());
  socklen_t len = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name_.size());
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&addr), len) != 0 || ::listen(lfd_, 256) != 0) {
    *err = std::string("bind/listen: ") + std::strerror(errno);
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  acceptor_ = std::thread([this] {
    name_thread("fp-accept");
    accept_loop();
  });
  return true;
}

void FastPathServer::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  std::unique_lock<std::mutex> g(mu_);
  for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
  workers_cv_.wait(g, [this] { return live_workers_ == 0 && pending_regs_ == 0; });
  for (auto& kv : maps_) {
    if (kv.second.registered) store_->unregister_host(kv.second.p);
    ::munmap(kv.second.p, kv.second.size);
  }
  maps_.clear();
  for (auto& m : retired_) {
    if (m.registered) store_->unregister_host(m.p);
    ::munmap(m.p, m.size);
  }
  retired_.clear();
  std::lock_guard<std::mutex> pg(peers_mu_);
  for (auto& kv : peers_)
    for (int fd : kv.second->idle) ::close(fd);
  peers_.clear();
}

bool FastPathServer::fence(uint64_t term, uint64_t* known) {
  uint64_t cur = term_.load();
  while (true) {
    if (term > 0 && term < cur) {
      *known = cur;
      return false;
    }
    if (term <= cur) {
      *known = cur;
      return true;
    }
    if (term_.compare_exchange_weak(cur, term)) {
      *known = term;
      return true;
    }
  }
}

void FastPathServer::adopt_term(uint64_t term) {
  uint64_t known;
  fence(term, &known);
}

std::vector<std::string> FastPathServer::drain_suspects() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  out.swap(suspects_);
  return out;
}

namespace {
constexpr size_t kRecentRids = 64;
}

void FastPathServer::note_rid(const std::string& rid) {
  if (rid.empty()) return;
  std::lock_guard<std::mutex> g(mu_);
  if (recent_rids_.size() < kRecentRids) recent_rids_.push_back(rid);
  else recent_rids_[recent_pos_++ % kRecentRids] = rid;
}

std::vector<std::string> FastPathServer::recent_request_ids() {
  std::lock_guard<std::mutex> g(mu_);
  if (recent_rids_.size() < kRecentRids) return recent_rids_;
  std::vector<std::string> out;
  for (size_t i = 0; i < kRecentRids; ++i) out.push_back(recent_rids_[(recent_pos_ + i) % kRecentRids]);
  return out;
}

FpStats FastPathServer::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

void FastPathServer::accept_loop() {
  while (!stop_.load()) {
    pollfd p{lfd_, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    // The abstract namespace has no file permissions: only processes of our own user
    // (or root) may hand this server shared-memory offsets.
    ucred cred{};
    socklen_t cl = sizeof(cred);
    if (::getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cred, &cl) != 0 ||
        (cred.uid != ::geteuid() && cred.uid != 0)) {
      ::close(fd);
      std::lock_guard<std::mutex> g(mu_);
      st_.rejected_peers++;
      continue;
    }
    std::lock_guard<std::mutex> g(mu_);
    if (stop_.load()) {
      ::close(fd);
      break;
    }
    conns_.push_back(fd);
    st_.connections++;
    live_workers_++;
    // detached: a finished connection frees its thread at once; stop() waits on the count
    std::thread([this, fd] {
      name_thread("fp-serve");
      serve(fd);
    }).detach();
  }
}

uint8_t* FastPathServer::map_shm(const std::string& path, uint64_t off, uint64_t len, std::string* err) {
  if (!valid_shm_path(path)) {
    *err = "refusing shared-memory path " + path;
    return nullptr;
  }
  if (len > kMaxTransfer || off > (1ull << 62)) {
    *err = "transfer out of bounds";
    return nullptr;
  }
  const uint64_t need = off + len;  // cannot wrap after the bounds above
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = maps_.find(path);
    if (it != maps_.end() && range_ok(off, len, it->second.size)) return it->second.p;
    if (it != maps_.end()) {
      // the client recreated a bigger arena under the same name: map it again but keep
      // the old mapping alive (another connection may still be copying from it)
      retired_.push_back(it->second);
      maps_.erase(it);
    }
  }
  int fd = ::open(path.c_str(), O_RDWR | O_CLOEXEC | O_NOFOLLOW);
  if (fd < 0) {
    *err = "open " + path + ": " + std::strerror(errno);
    return nullptr;
  }
  struct stat sb {};
  if (::fstat(fd, &sb) != 0 || sb.st_size < 0 || !range_ok(off, len, static_cast<uint64_t>(sb.st_size))) {
    ::close(fd);
    *err = "shared-memory arena too small";
    return nullptr;
  }
  void* p = ::mmap(nullptr, static_cast<size_t>(sb.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) {
    *err = std::string("mmap: ") + std::strerror(errno);
    return nullptr;
  }
  std::lock_guard<std::mutex> g(mu_);
  auto& m = maps_[path];
  if (m.p != nullptr) {  // raced with another connection of the same client
    ::munmap(p, static_cast<size_t>(sb.st_size));
    if (!range_ok(off, len, m.size)) {
      *err = "shared-memory arena too small";
      return nullptr;
    }
    return m.p;
  }
  m.p = static_cast<uint8_t*>(p);
  m.size = static_cast<uint64_t>(sb.st_size);
  // pin the client's arena for the GPU copy engines: blocks then move slot <-> HBM in one
  // DMA, with no bounce through staging buffers and no CPU memcpy. Pinning a 256 MiB arena
  // takes tens of ms, so it runs on its own thread, off mu_: until it lands, this client's
  // ops take the staged path (store_->host_registered says which) and nobody else waits.
  if (store_->gpu()) {
    ++pending_regs_;
    uint8_t* base = m.p;
    const uint64_t size = m.size;
    std::thread([this, base, size] {
      bool ok = store_->register_host(base, size);
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& kv : maps_)
        if (kv.second.p == base) kv.second.registered = ok;
      for (auto& r : retired_)
        if (r.p == base) r.registered = ok;
      --pending_regs_;
      workers_cv_.notify_all();
    }).detach();
  }
  return m.p;
}

void FastPathServer::set_replication(ReplicationEngine* engine) { repl_ = engine; }

void FastPathServer::set_peer(const std::string& addr, int rank, const std::string& fp_name) {
  std::lock_guard<std::mutex> g(peers_mu_);
  auto& p = peers_[addr];
  if (!p) p = std::make_unique<Peer>();
  p->rank = rank;
  if (!fp_name.empty()) p->name = fp_name;
}

namespace {

int connect_abstract(const std::string& name) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  addr.sun_path[0] = '\0';
  std::memcpy(addr.sun_path + 1, name.data(), std::min(name.size(), sizeof(addr.sun_path) - 2));
  socklen_t len = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name.size());
  timeval tv{120, 0};  // bounded like every other wait on the replication path
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), len) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

}  // namespace

namespace {

// One request/response exchange on a pooled peer connection.
bool exchange(int fd, const std::vector<uint8_t>& req, std::vector<uint8_t>* resp) {
  uint32_t n = 0;
  if (!write_full(fd, req.data(), req.size())) return false;
  if (!read_full(fd, &n, 4) || n < 19 || n > kMaxBody) return false;
  resp->resize(n);
  return read_full(fd, resp->data(), n);
}

std::string resp_msg(const std::vector<uint8_t>& r) {
  uint16_t ml = 0;
  std::memcpy(&ml, r.data() + 17, 2);
  return std::string(reinterpret_cast<const char*>(r.data() + 19), std::min<size_t>(ml, r.size() - 19));
}

void finish_frame(std::vector<uint8_t>& req) {
  uint32_t body = static_cast<uint32_t>(req.size() - 4);
  std::memcpy(req.data(), &body, 4);
}

}  // namespace

void FastPathServer::set_self_host(const std::string& host) {
  std::lock_guard<std::mutex> g(peers_mu_);
  self_host_ = host;
}

FastPathServer::Peer* FastPathServer::local_peer(const std::string& addr) {
  // same-host peers are reachable at the deterministic socket "dfs_fp_<port>"
  auto colon = addr.rfind(':');
  if (colon == std::string::npos) return nullptr;
  std::string host = addr.substr(0, colon), port = addr.substr(colon + 1);
  std::lock_guard<std::mutex> g(peers_mu_);
  auto it = peers_.find(addr);
  if (it != peers_.end()) return it->second.get();
  bool local = host == "127.0.0.1" || host == "localhost" || host == "::1" || (!self_host_.empty() && host == self_host_);
  if (!local || port.empty()) return nullptr;
  auto& p = peers_[addr];
  p = std::make_unique<Peer>();
  p->name = "dfs_fp_" + port;
  return p.get();
}

bool FastPathServer::exchange_with(Peer* p, const std::vector<uint8_t>& req, std::vector<uint8_t>* resp) {
  int fd = -1;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (!p->idle.empty()) {
      fd = p->idle.back();
      p->idle.pop_back();
    }
  }
  if (fd < 0 && (fd = connect_abstract(p->name)) < 0) return false;
  if (!exchange(fd, req, resp)) {
    ::close(fd);
    return false;
  }
  std::lock_guard<std::mutex> g(p->mu);
  p->idle.push_back(fd);
  return true;
}

bool FastPathServer::control(int rank, const std::string& blob, std::string* reply) {
  Peer* p = nullptr;
  {
    std::lock_guard<std::mutex> g(peers_mu_);
    for (auto& kv : peers_)
      if (kv.second->rank == rank && !kv.second->name.empty()) p = kv.second.get();
  }
  if (!p) return false;
  std::vector<uint8_t> req(4, 0), resp;
  req.push_back(5);
  put_str(req, blob);
  finish_frame(req);
  if (!exchange_with(p, req, &resp) || static_cast<FpStatus>(resp[0]) != FpStatus::Ok) return false;
  *reply = resp_msg(resp);
  return true;
}

std::vector<std::string> FastPathServer::drain_healed() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  out.swap(healed_);
  return out;
}

int FastPathServer::replicate_block(const std::string& id, const std::vector<std::string>& targets, uint64_t term,
                                    std::vector<std::string>* done) {
  TraceRange tr("dfs.fp.heal_copy");
  if (repl_ == nullptr || !store_->exists(id)) return 0;
  const uint32_t crc = store_->block_crc(id);
  std::vector<uint8_t> host;
  if (!store_->gpu()) {  // host store: the socket transport sends from host memory
    ReadResult st = store_->stat(id, 0, 0);
    if (st.status != ReadStatus::Ok) return 0;
    host.resize(st.bytes);
    ReadResult rr = store_->read_into(id, 0, st.bytes, host.data());
    if (rr.status != ReadStatus::Ok || rr.partial_corrupt) return 0;
  }
  int total = 0;
  for (const auto& t : targets) {
    Peer* p = local_peer(t);
    if (p == nullptr || p->rank < 0 || !repl_->pair_ok(p->rank)) continue;
    int n = replicate_one(t, id, crc, term, ShmSrc{}, host.empty() ? nullptr : host.data(), host.size(), true);
    if (n > 0) {
      done->push_back(t);
      std::lock_guard<std::mutex> g(mu_);
      st_.heals_out++;
    }
    total += n;
  }
  return total;
}

int FastPathServer::replicate_one(const std::string& addr, const std::string& id, uint32_t crc, uint64_t term,
                                  const ShmSrc& src, const uint8_t* host, uint64_t n, bool heal,
                                  const StagedSource* staged, bool ephemeral) {
  Peer* p = local_peer(addr);
  if (p == nullptr) return 0;
  std::vector<uint8_t> resp;
  auto count_ok = [&](uint64_t FpStats::*field) {
    uint64_t down = 0;
    std::memcpy(&down, resp.data() + 9, 8);
    std::lock_guard<std::mutex> g(mu_);
    (st_.*field)++;
    return static_cast<int>(down);
  };
  bool tried_p2p = false;
  if (repl_ != nullptr && p->rank >= 0 && repl_->pair_ok(p->rank)) {
    // payload over the P2P transport (RCCL: HBM -> HBM over xGMI), descriptor on the socket
    ReplTicket t;
    std::string err;
    auto descriptor = [&](const ReplTicket& tk) {
      std::vector<uint8_t> req(4, 0);
      req.push_back(3);
      put<uint64_t>(req, term);
      put<uint32_t>(req, crc);
      put<int32_t>(req, repl_->rank());
      put<uint64_t>(req, tk.gen);
      put<int64_t>(req, tk.seq);
      put<uint64_t>(req, tk.size);
      put<uint64_t>(req, tk.slice);
      put_str(req, id);
      put<uint16_t>(req, 0);  // fan-out: the replica forwards nowhere
      put_str(req, t_request_id);
      put<uint8_t>(req, heal ? 1 : 0);  // a heal copy: the receiver reports the new location
      put<uint8_t>(req, ephemeral ? 1 : 0);  // an EC gather copy: held in HBM only, never persisted
      put<uint8_t>(req, static_cast<uint8_t>(tk.ch));  // the pair's channel the transfer is sequenced on
      finish_frame(req);
      return req;
    };
    // A staged (still landing) block announces itself before its first slice is posted, so
    // the replica posts its receives while the head's later slices still cross PCIe; the
    // reply is read after the posts. Otherwise: post, then one descriptor round trip.
    int early_fd = -1;
    auto announce = [&](const ReplTicket& tk) {
      std::vector<uint8_t> req = descriptor(tk);
      {
        std::lock_guard<std::mutex> g(p->mu);
        if (!p->idle.empty()) {
          early_fd = p->idle.back();
          p->idle.pop_back();
        }
      }
      if (early_fd < 0) early_fd = connect_abstract(p->name);
      if (early_fd >= 0 && write_full(early_fd, req.data(), req.size())) return true;
      if (early_fd >= 0) ::close(early_fd);
      early_fd = -1;
      return false;
    };
    std::function<bool(const ReplTicket&)> ann;
    if (staged) ann = announce;
    const bool posted = repl_->send(p->rank, id, host, n, &t, &err, staged, ann);
    if (!posted && early_fd >= 0) {  // announced, then failed: the pair is failed, the peer gives up
      ::close(early_fd);
      early_fd = -1;
    }
    if (posted) {
      tried_p2p = true;
      const auto d0 = std::chrono::steady_clock::now();
      bool io_ok;
      int drop = drop_descriptors_.load();
      if (staged) {
        uint32_t rn = 0;
        io_ok = read_full(early_fd, &rn, 4) && rn >= 19 && rn <= kMaxBody;
        if (io_ok) {
          resp.resize(rn);
          io_ok = read_full(early_fd, resp.data(), rn);
        }
        if (io_ok) {
          std::lock_guard<std::mutex> g(p->mu);
          p->idle.push_back(early_fd);
        } else {
          ::close(early_fd);
        }
      } else if (drop > 0 && drop_descriptors_.compare_exchange_strong(drop, drop - 1)) {
        io_ok = false;  // test hook
      } else {
        io_ok = exchange_with(p, descriptor(t), &resp);
      }
      if (!io_ok) {
        // the posted sends can never be matched now: abort the pair (it is rebuilt under a
        // new generation) and move this replica to shared memory below
        repl_->cancel_send(&t, "descriptor to " + addr + " failed");
      } else {
        {
          std::lock_guard<std::mutex> g(mu_);
          st_.desc_calls++;
          st_.desc_ns += static_cast<uint64_t>(
              std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - d0).count());
        }
        std::string werr;
        bool sent = repl_->wait_send(&t, &werr);
        FpStatus st = static_cast<FpStatus>(resp[0]);
        if (st == FpStatus::Ok) return count_ok(&FpStats::rccl_forwards);
        if (st == FpStatus::Fenced) return 0;
        (void)sent;  // a failed transfer already failed the pair inside the engine
      }
    }
  }
  if (src.path.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    st_.replica_failures++;
    return 0;
  }
  // same-host hop without a P2P pair: the replica stages straight from the client's slot
  std::vector<uint8_t> req(4, 0);
  req.push_back(4);
  put<uint64_t>(req, term);
  put<uint32_t>(req, crc);
  put<uint64_t>(req, src.off);
  put<uint64_t>(req, src.len);
  put_str(req, id);
  put_str(req, src.path);
  put<uint16_t>(req, 0);
  put_str(req, t_request_id);
  finish_frame(req);
  if (exchange_with(p, req, &resp) && static_cast<FpStatus>(resp[0]) == FpStatus::Ok) {
    if (tried_p2p) {
      std::lock_guard<std::mutex> g(mu_);
      st_.p2p_fallbacks++;
    }
    return count_ok(&FpStats::shm_forwards);
  }
  std::lock_guard<std::mutex> g(mu_);
  st_.replica_failures++;
  return 0;
}

bool FastPathServer::all_local(const std::vector<std::string>& next) {
  for (auto& a : next)
    if (local_peer(a) == nullptr) return false;
  return true;
}

bool FastPathServer::p2p_ready(const std::vector<std::string>& next) {
  for (auto& a : next) {
    Peer* p = local_peer(a);
    if (p == nullptr || repl_ == nullptr || p->rank < 0 || !repl_->pair_ok(p->rank)) return false;
  }
  return true;
}

void FastPathServer::add_suspect(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  suspects_.push_back(id);
}

bool FastPathServer::persist_and_replicate(const std::string& id, const uint8_t* host, uint64_t n, uint32_t crc,
                                           uint64_t term, const std::vector<std::string>& next, int* downstream,
                                           std::string* err) {
  // no shared-memory source: replicas go over the P2P transport (the block is staged in HBM)
  // or, without a pair, fail and are not counted — as a downstream failure in the reference
  const std::string rid = t_request_id;
  auto fut = pool_.submit([&] {
    RequestScope rs(rid);
    replicate(id, crc, term, next, ShmSrc{}, host, n, downstream);
  });
  bool ok = store_->persist(id, host, n, err);
  fut.get();
  return ok;
}

void FastPathServer::replicate(const std::string& id, uint32_t crc, uint64_t term, const std::vector<std::string>& next,
                               const ShmSrc& src, const uint8_t* host, uint64_t n, int* replicas,
                               const StagedSource* staged) {
  *replicas = 0;
  if (next.empty()) return;
  // every replica at once: each has its own xGMI link from this GPU
  std::vector<std::future<int>> futs;
  const std::string rid = t_request_id;
  for (size_t i = 1; i < next.size(); ++i)
    futs.push_back(pool_.submit([&, i] {
      RequestScope rs(rid);
      return replicate_one(next[i], id, crc, term, src, host, n, false, staged);
    }));
  int total = replicate_one(next[0], id, crc, term, src, host, n, false, staged);
  for (auto& f : futs) total += f.get();
  *replicas = total;
}

// Pipelined head write: the store stages the block slice by slice
// (one fused copy+checksum kernel per engine slice) and every replica send posts slice k
// as soon as it is in HBM, so the links carry slice k while slice k+1 crosses PCIe; the
// store verifies the whole block from the slice partials while the tail is still in flight.
// The replicas verify what they receive against the client's CRC on their own, so a block
// the head rejects is rejected downstream too.
bool FastPathServer::write_sliced(int fd, const std::string& id, const uint8_t* host, uint64_t len, uint32_t crc,
                                  uint64_t term, const std::vector<std::string>& next, const ShmSrc& src, bool* sent) {
  static const uint64_t min_bytes = [] {  // DFS_SLICED_WRITE_MIN_MIB (0 = off)
    const char* e = std::getenv("DFS_SLICED_WRITE_MIN_MIB");
    return (e ? std::strtoull(e, nullptr, 10) : 16ull) << 20;
  }();
  if (min_bytes == 0 || len < min_bytes || repl_ == nullptr || !store_->gpu() || !repl_->transport()->device_buffers() ||
      !p2p_ready(next))
    return false;
  const uint64_t slice = repl_->slice_for(len);
  if (len <= slice) return false;  // a single slice: nothing to overlap
  ChunkStore::SliceStage ss;
  std::string err;
  if (!store_->stage_slices_begin(host, len, slice, &ss, &err)) return false;
  StagedSource staged{ss.ext.ptr, slice, &ss.done};
  int down = 0;
  const std::string rid = t_request_id;
  auto fut = pool_.submit([&] {
    RequestScope rs(rid);
    replicate(id, crc, term, next, src, host, len, &down, &staged);
  });
  WriteResult wr = store_->stage_slices_finish(id, &ss, crc, 1);  // pinned while the sends read it
  std::string perr;
  const bool pok = wr.ok && store_->persist(id, host, len, &perr);
  fut.get();
  if (wr.ok) store_->unpin(id);
  store_->stage_slices_end(&ss);
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.sliced_writes++;
    if (wr.ok) st_.writes++;
  }
  if (!wr.ok) *sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
  else if (!pok) *sent = send_response(fd, FpStatus::IoError, 0, 0, perr);
  else *sent = send_response(fd, FpStatus::Ok, len, 1 + static_cast<uint64_t>(down), "");
  return true;
}

void FastPathServer::serve(int fd) {
  std::vector<uint8_t> body;
  auto bump = [this](uint64_t FpStats::*field) {
    std::lock_guard<std::mutex> g(mu_);
    (st_.*field)++;
  };
  auto fenced = [&](uint64_t term, std::string* msg) {
    uint64_t known = 0;
    if (fence(term, &known)) return false;
    bump(&FpStats::fenced);
    *msg = "Stale master term: request has " + std::to_string(term) + " but known term is " + std::to_string(known);
    return true;
  };
  // Local persist and the downstream fan-out run concurrently; the ack waits for both.
  auto persist_and_forward = [&](const std::string& id, const uint8_t* host, uint64_t len, uint32_t crc,
                                 uint64_t term, const std::vector<std::string>& next, const ShmSrc& src) -> bool {
    int down = 0;
    std::string perr;
    const std::string rid = t_request_id;
    auto fut = pool_.submit([&] {
      RequestScope rs(rid);
      replicate(id, crc, term, next, src, host, len, &down);
    });
    bool pok = store_->persist(id, host, host ? len : 0, &perr);
    fut.get();
    if (!pok) return send_response(fd, FpStatus::IoError, 0, 0, perr);
    return send_response(fd, FpStatus::Ok, len, 1 + static_cast<uint64_t>(down), "");
  };
  while (!stop_.load()) {
    uint32_t n = 0;
    if (!read_full(fd, &n, 4) || n == 0 || n > kMaxBody) break;
    body.resize(n);
    if (!read_full(fd, body.data(), n)) break;
    Reader rd{body.data() + 1, body.data() + n};
    uint8_t op = body[0];
    bool sent = false;
    std::string msg;
    if (op == 1) {  // WRITE from a co-located client (optionally the head of a chain)
      uint64_t term = rd.get<uint64_t>();
      uint32_t crc = rd.get<uint32_t>();
      uint64_t off = rd.get<uint64_t>(), len = rd.get<uint64_t>();
      std::string id = rd.str(), path = rd.str();
      std::vector<std::string> next = read_list(rd, true);
      std::string rid = rd.p < rd.end ? rd.str() : std::string();  // request id (after the list)
      RequestScope rs(rid);
      note_rid(rid);
      TraceRange tr("dfs.fp.write");
      std::string err;
      uint8_t* base = nullptr;
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed write request");
      } else if (fenced(term, &msg)) {
        sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
      } else if (!all_local(next)) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "no native route for a replica");
      } else if ((base = map_shm(path, off, len, &err)) == nullptr) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "short-circuit unavailable: " + err);
      } else if (next.empty()) {
        WriteResult wr = store_->write(id, base + off, len, crc);
        if (wr.ok) bump(&FpStats::writes);
        sent = wr.ok ? send_response(fd, FpStatus::Ok, len, 1, "") : send_response(fd, FpStatus::IoError, 0, 0, wr.error);
      } else if (!write_sliced(fd, id, base + off, len, crc, term, next, ShmSrc{path, off, len}, &sent)) {
        const auto c0 = std::chrono::steady_clock::now();
        WriteResult wr = store_->stage(id, base + off, len, crc);  // HBM + CRC verify, not yet durable
        if (!wr.ok) {
          sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
        } else {
          bump(&FpStats::writes);
          const auto c1 = std::chrono::steady_clock::now();
          sent = persist_and_forward(id, base + off, len, crc, term, next, ShmSrc{path, off, len});
          const auto c2 = std::chrono::steady_clock::now();
          std::lock_guard<std::mutex> g(mu_);
          st_.chain_writes++;
          st_.chain_stage_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count());
          st_.chain_forward_ns += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(c2 - c1).count());
        }
      }
    } else if (op == 3) {  // REPL: block arrives over the P2P transport from the head
      uint64_t term = rd.get<uint64_t>();
      uint32_t crc = rd.get<uint32_t>();
      int32_t src = rd.get<int32_t>();
      uint64_t gen = rd.get<uint64_t>();
      int64_t seq = rd.get<int64_t>();
      uint64_t size = rd.get<uint64_t>();
      uint64_t slice = rd.get<uint64_t>();
      std::string id = rd.str();
      std::vector<std::string> next = read_list(rd, false);
      std::string rid = rd.p < rd.end ? rd.str() : std::string();
      const bool heal = rd.p < rd.end && rd.get<uint8_t>() == 1;
      const bool ephemeral = rd.p < rd.end && rd.get<uint8_t>() == 1;
      const int ch = rd.p < rd.end ? rd.get<uint8_t>() : 0;
      RequestScope rs(rid);
      note_rid(rid);
      if (!rd.ok || id.empty() || repl_ == nullptr || size > kMaxTransfer) {
        if (repl_ && rd.ok && src >= 0) repl_->fail_pair_gen(src, gen, "malformed descriptor");
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, repl_ ? "malformed replicate request" : "replication disabled");
      } else {
        // The receive is posted even for a fenced request — refusing it would leave the
        // sender's transfer unmatched and cost the pair a rebuild; the block is dropped after.
        bool last = next.empty();
        bool stale = fenced(term, &msg);
        WriteResult wr = repl_->recv(src, gen, ch, seq, id, size, slice, crc, last && !stale && !ephemeral);
        if (stale) {
          if (wr.ok) store_->remove(id);
          sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
        } else if (!wr.ok) {
          sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
        } else {
          bump(&FpStats::replicas_in);
          if (heal) {
            std::lock_guard<std::mutex> g(mu_);
            healed_.push_back(id);
            st_.heals_in++;
          }
          sent = last ? send_response(fd, FpStatus::Ok, size, 1, "")
                      : persist_and_forward(id, nullptr, size, crc, term, next, ShmSrc{});
        }
      }
    } else if (op == 4) {  // REPL_SHM: a same-host hop; stage from the client's slot
      uint64_t term = rd.get<uint64_t>();
      uint32_t crc = rd.get<uint32_t>();
      uint64_t off = rd.get<uint64_t>(), len = rd.get<uint64_t>();
      std::string id = rd.str(), path = rd.str();
      std::vector<std::string> next = read_list(rd, false);
      std::string rid = rd.p < rd.end ? rd.str() : std::string();
      RequestScope rs(rid);
      note_rid(rid);
      TraceRange tr("dfs.fp.replicate_shm");
      std::string err;
      uint8_t* base = nullptr;
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed replicate request");
      } else if (fenced(term, &msg)) {
        sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
      } else if ((base = map_shm(path, off, len, &err)) == nullptr) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "short-circuit unavailable: " + err);
      } else if (next.empty()) {
        WriteResult wr = store_->write(id, base + off, len, crc);
        if (wr.ok) bump(&FpStats::replicas_in);
        sent = wr.ok ? send_response(fd, FpStatus::Ok, len, 1, "") : send_response(fd, FpStatus::IoError, 0, 0, wr.error);
      } else {
        WriteResult wr = store_->stage(id, base + off, len, crc);
        if (!wr.ok) {
          sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
        } else {
          bump(&FpStats::replicas_in);
          sent = persist_and_forward(id, base + off, len, crc, term, next, ShmSrc{path, off, len});
        }
      }
    } else if (op == 6) {  // EC: GF(2^8) matrix x shards on this server's GPU, in the client's slot
      uint16_t k = rd.get<uint16_t>(), rows = rd.get<uint16_t>();
      uint64_t len = rd.get<uint64_t>(), in_off = rd.get<uint64_t>(), out_off = rd.get<uint64_t>();
      std::string mat = rd.str(), path = rd.str();
      std::string rid = rd.p < rd.end ? rd.str() : std::string();
      // optional: the k inputs sit at in_off + idx[c] * stride (a degraded read decodes
      // straight from the shard layout it fetched, survivors need not be adjacent)
      std::vector<uint16_t> idx;
      if (rd.p < rd.end) {
        uint16_t ni = rd.get<uint16_t>();
        for (uint16_t i = 0; rd.ok && i < ni && i <= kMaxShards * 2; ++i) idx.push_back(rd.get<uint16_t>());
        if (idx.size() != k) rd.ok = false;
      }
      RequestScope rs(rid);
      note_rid(rid);
      TraceRange tr("dfs.fp.ec");
      const uint64_t stride = (len + 15) / 16 * 16;
      std::string err;
      uint8_t* base = nullptr;
      uint64_t span = k;
      for (uint16_t v : idx) span = std::max<uint64_t>(span, uint64_t(v) + 1);
      if (span > 2 * kMaxShards) rd.ok = false;
      // Each region is bounded on its own before any pointer is formed: offsets near 2^64
      // must not wrap into a small span (len <= kMaxTransfer and k, rows <= kMaxShards keep
      // stride * k far below 2^62, so only the offsets need checking).
      const uint64_t in_len = stride * span, out_len = stride * rows;
      const bool regions_ok = in_off <= (1ull << 62) && out_off <= (1ull << 62);
      if (!rd.ok || k == 0 || rows == 0 || k > kMaxShards || rows > kMaxShards || mat.size() != size_t(k) * rows ||
          len > kMaxTransfer || !regions_ok) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed ec request");
      } else if (!store_->gpu()) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "no GPU on this chunkserver");
      } else if ((base = map_shm(path, in_off, in_len, &err)) == nullptr ||
                 map_shm(path, out_off, out_len, &err) != base) {
        if (base != nullptr && err.empty()) err = "ec regions outside the arena";
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "short-circuit unavailable: " + err);
      } else {
        std::vector<std::vector<uint8_t>> M(rows, std::vector<uint8_t>(k));
        for (int r = 0; r < rows; ++r)
          for (int c = 0; c < k; ++c) M[r][c] = static_cast<uint8_t>(mat[r * k + c]);
        std::vector<const uint8_t*> in(k);
        std::vector<uint8_t*> out(rows);
        for (int c = 0; c < k; ++c) in[c] = base + in_off + (idx.empty() ? c : idx[c]) * stride;
        for (int r = 0; r < rows; ++r) out[r] = base + out_off + r * stride;
        bool ok = store_->gf_matmul_gpu(M, in, out, len);
        if (ok) bump(&FpStats::ec_ops);
        sent = ok ? send_response(fd, FpStatus::Ok, len, rows, "")
                  : send_response(fd, FpStatus::Unsupported, 0, 0, "GPU erasure coding failed");
      }
    } else if (op == 7) {  // EC_WRITE: encode in HBM, scatter the shards over the engine
      sent = ec_write(fd, body.data() + 1, body.data() + n);
    } else if (op == 8) {  // EC_READ: gather the surviving shards into HBM, decode there
      sent = ec_read(fd, body.data() + 1, body.data() + n);
    } else if (op == 9) {  // PUSH: a local block to a peer over the engine (EC gathers)
      sent = push_block(fd, body.data() + 1, body.data() + n);
    } else if (op == 5) {  // CTRL: replication pair bring-up / rebuild
      std::string blob = rd.str();
      if (!rd.ok || repl_ == nullptr) sent = send_response(fd, FpStatus::Unsupported, 0, 0, "replication disabled");
      else sent = send_response(fd, FpStatus::Ok, 0, 0, repl_->handle_control(blob));
    } else if (op == 2) {  // READ into the client's slot
      uint64_t offset = rd.get<uint64_t>(), length = rd.get<uint64_t>();
      uint64_t shm_off = rd.get<uint64_t>(), cap = rd.get<uint64_t>();
      std::string id = rd.str(), path = rd.str();
      std::string rid = rd.p < rd.end ? rd.str() : std::string();
      RequestScope rs(rid);
      note_rid(rid);
      TraceRange tr("dfs.fp.read");
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed read request");
      } else {
        ReadResult st = store_->stat(id, offset, length);
        std::string err;
        uint8_t* base = nullptr;
        if (st.status != ReadStatus::Ok) {
          sent = send_response(fd, static_cast<FpStatus>(st.status), st.total_size, 0, st.error);
        } else if (st.bytes > cap) {
          sent = send_response(fd, FpStatus::Unsupported, st.total_size, 0, "slot too small");
        } else if ((base = map_shm(path, shm_off, cap, &err)) == nullptr) {
          sent = send_response(fd, FpStatus::Unsupported, st.total_size, 0, "short-circuit unavailable: " + err);
        } else {
          ReadResult rr = store_->read_into(id, offset, st.bytes, base + shm_off);
          if (rr.status == ReadStatus::Ok && !rr.partial_corrupt) {
            bump(&FpStats::reads);
            sent = send_response(fd, FpStatus::Ok, rr.total_size, rr.bytes, "");
          } else if (rr.status == ReadStatus::Ok) {
            {
              std::lock_guard<std::mutex> g(mu_);
              suspects_.push_back(id);
              st_.reads++;
            }
            sent = send_response(fd, FpStatus::PartialCorrupt, rr.total_size, rr.bytes, rr.error);
          } else {
            bump(&FpStats::punts);
            sent = send_response(fd, static_cast<FpStatus>(rr.status), rr.total_size, 0, rr.error);
          }
        }
      }
    } else {
      sent = send_response(fd, FpStatus::Unsupported, 0, 0, "unknown op");
    }
    if (!sent) break;
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = conns_.begin(); it != conns_.end(); ++it) {
    if (*it == fd) {
      conns_.erase(it);
      break;
    }
  }
  ::close(fd);
  if (--live_workers_ == 0) workers_cv_.notify_all();
}


// ------------------------------------------------------------------ device erasure coding
void FastPathServer::set_self_addr(const std::string& addr) { self_addr_ = addr; }

bool FastPathServer::is_self(const std::string& addr) const { return !self_addr_.empty() && addr == self_addr_; }

FastPathServer::EcGather::~EcGather() {
  if (!fp) return;
  for (auto& id : pinned) fp->store_->unpin(id);
  for (auto& id : temps) fp->store_->remove(id);
}

bool FastPathServer::ec_gather(const std::string& id, const std::vector<std::string>& locations, uint64_t shard_len,
                               int skip, int want, EcGather* g, std::string* err) {
  g->fp = this;
  g->ptrs.assign(locations.size(), nullptr);
  if (!store_->gpu() || repl_ == nullptr || !repl_->transport()->device_buffers()) {
    *err = "no device transport";
    return false;
  }
  std::vector<uint64_t> sizes(locations.size(), 0);
  int have = 0;
  // our own shard in place, once its slices verify against its .meta (K1b): a corrupt local
  // shard counts as lost
  std::vector<int> peers;
  for (size_t i = 0; i < locations.size(); ++i) {
    if (static_cast<int>(i) == skip || locations[i].empty()) continue;
    if (!is_self(locations[i])) {
      peers.push_back(static_cast<int>(i));
      continue;
    }
    uint64_t size = 0;
    const uint8_t* d = store_->pin_device(id, &size);
    if (!d) continue;
    if ((shard_len == 0 || size == shard_len) && store_->scrub_resident({id}).empty()) {
      g->ptrs[i] = d;
      g->pinned.push_back(id);
      sizes[i] = size;
      ++have;
    } else {
      store_->unpin(id);
    }
  }
  // then the peers', pushed over the engine (checksummed as they land), in rounds of just
  // as many as are still needed: a dead or corrupt holder is replaced by the next candidate
  std::mutex gm;
  const std::string rid = t_request_id;
  size_t next = 0;
  while (have < want && next < peers.size()) {
    std::vector<std::future<void>> futs;
    for (int need = want - have; need > 0 && next < peers.size(); ++next) {
      const int i = peers[next];
      Peer* p = local_peer(locations[i]);
      if (p == nullptr || p->rank < 0 || !repl_->pair_ok(p->rank)) {
        g->unreachable++;
        continue;
      }
      --need;
      const std::string tmp = id + ".g" + std::to_string(i) + "." + std::to_string(tmp_seq_.fetch_add(1));
      futs.push_back(pool_.submit([this, p, id, tmp, i, shard_len, rid, g, &gm, &have, &sizes] {
        RequestScope rs(rid);
        std::vector<uint8_t> req(4, 0), resp;
        req.push_back(9);
        put_str(req, id);
        put_str(req, tmp);
        put_str(req, self_addr_);
        put_str(req, rid);
        finish_frame(req);
        const bool ok = exchange_with(p, req, &resp) && static_cast<FpStatus>(resp[0]) == FpStatus::Ok;
        uint64_t size = 0;
        const uint8_t* d = ok ? store_->pin_device(tmp, &size) : nullptr;
        std::lock_guard<std::mutex> lk(gm);
        if (store_->exists(tmp)) g->temps.push_back(tmp);
        if (d && (shard_len == 0 || size == shard_len)) {
          g->ptrs[i] = d;
          g->pinned.push_back(tmp);
          sizes[i] = size;
          ++have;
        } else {
          if (d) store_->unpin(tmp);
          g->unreachable++;
        }
      }));
    }
    for (auto& f : futs) f.get();
  }
  // every shard of a block has the same length: without a given one, keep the shards that
  // agree with the first (a stale shard of another length is treated as lost)
  g->len = shard_len;
  for (size_t i = 0; i < g->ptrs.size(); ++i) {
    if (!g->ptrs[i]) continue;
    if (g->len == 0) g->len = sizes[i];
    if (sizes[i] != g->len) g->ptrs[i] = nullptr;
  }
  std::lock_guard<std::mutex> lk(mu_);
  st_.ec_gathered += g->temps.size();
  return true;
}

bool FastPathServer::push_block(int fd, const uint8_t* body, const uint8_t* end) {
  Reader rd{body, end};
  std::string id = rd.str(), as_id = rd.str(), dst = rd.str();
  std::string rid = rd.p < rd.end ? rd.str() : std::string();
  RequestScope rs(rid);
  note_rid(rid);
  TraceRange tr("dfs.fp.ec_push");
  if (!rd.ok || id.empty() || as_id.empty() || repl_ == nullptr || !store_->gpu() ||
      !repl_->transport()->device_buffers())
    return send_response(fd, FpStatus::Unsupported, 0, 0, "no device transport");
  uint64_t size = 0;
  const uint8_t* d = store_->pin_device(id, &size);
  if (!d) return send_response(fd, FpStatus::NotFound, 0, 0, "Block not found");
  const uint32_t crc = store_->block_crc(id);
  // the block is resident and complete: every slice is "landed" at once
  hipEvent_t ready = nullptr;
  (void)hipSetDevice(store_->config().device);
  bool ok = hipEventCreateWithFlags(&ready, hipEventDisableTiming) == hipSuccess;
  int n = 0;
  if (ok) {
    const uint64_t slice = repl_->slice_for(size);
    std::vector<hipEvent_t> done(std::max<uint64_t>(1, (size + slice - 1) / slice), ready);
    StagedSource staged{d, slice, &done};
    n = replicate_one(dst, as_id, crc, 0, ShmSrc{}, nullptr, size, false, &staged, true);
    (void)hipEventDestroy(ready);
  }
  store_->unpin(id);
  return n > 0 ? send_response(fd, FpStatus::Ok, size, 1, "")
               : send_response(fd, FpStatus::IoError, 0, 0, "push over the replication engine failed");
}

bool FastPathServer::ec_write(int fd, const uint8_t* body, const uint8_t* end) {
  Reader rd{body, end};
  uint64_t term = rd.get<uint64_t>();
  uint16_t k = rd.get<uint16_t>(), m = rd.get<uint16_t>();
  uint64_t sl = rd.get<uint64_t>(), off = rd.get<uint64_t>(), hstride = rd.get<uint64_t>();
  std::string id = rd.str(), path = rd.str();
  std::vector<std::string> targets = read_list(rd, false);
  std::string rid = rd.p < rd.end ? rd.str() : std::string();
  RequestScope rs(rid);
  note_rid(rid);
  TraceRange tr("dfs.fp.ec_write");
  auto fallback = [&](const std::string& why) {
    std::lock_guard<std::mutex> g(mu_);
    st_.ec_device_fallbacks++;
    return send_response(fd, FpStatus::Unsupported, 0, 0, why);
  };
  if (!rd.ok || id.empty() || k == 0 || m == 0 || k + m > kMaxShards || targets.size() != size_t(k) + m ||
      sl == 0 || sl > kMaxTransfer || hstride < sl || hstride > kMaxTransfer)
    return send_response(fd, FpStatus::BadRequest, 0, 0, "malformed ec write");
  std::string msg;
  uint64_t known = 0;
  if (!fence(term, &known)) {
    std::lock_guard<std::mutex> g(mu_);
    st_.fenced++;
    return send_response(fd, FpStatus::Fenced, known, 0,
                         "Stale master term: request has " + std::to_string(term) + " but known term is " +
                             std::to_string(known));
  }
  if (!store_->gpu() || repl_ == nullptr || !repl_->transport()->device_buffers())
    return fallback("no device transport");
  for (auto& t : targets) {
    if (is_self(t)) continue;
    Peer* p = local_peer(t);
    if (p == nullptr || p->rank < 0 || !repl_->pair_ok(p->rank)) return fallback("a shard target has no P2P pair");
  }
  std::string err;
  uint8_t* base = map_shm(path, off, hstride * k, &err);
  if (base == nullptr) return fallback("short-circuit unavailable: " + err);
  gf::Matrix full = gf::rs_matrix(k, m), parity(full.begin() + k, full.end());
  ChunkStore::EcBuffers enc;
  if (!store_->ec_encode(base + off, hstride, sl, k, parity, &enc, &err)) return fallback(err);
  const uint64_t slice = repl_->slice_for(sl);
  std::vector<hipEvent_t> done(std::max<uint64_t>(1, (sl + slice - 1) / slice), enc.done);
  std::vector<std::future<std::string>> futs;
  const std::string rid_s = t_request_id;
  for (int i = 0; i < k + m; ++i) {
    futs.push_back(pool_.submit([&, i]() -> std::string {
      RequestScope scope(rid_s);
      if (is_self(targets[i])) {
        WriteResult w = store_->commit_copy(id, enc.shard(i), sl, enc.crc[i], true);
        return w.ok ? std::string() : w.error;
      }
      StagedSource staged{enc.shard(i), slice, &done};
      const int n = replicate_one(targets[i], id, enc.crc[i], term, ShmSrc{}, nullptr, sl, false, &staged);
      if (n > 0) {
        std::lock_guard<std::mutex> g(mu_);
        st_.ec_shard_forwards++;
        return std::string();
      }
      return "replica did not accept the shard";
    }));
  }
  std::string first_err;
  int failed_at = -1;
  for (int i = 0; i < k + m; ++i) {
    std::string e = futs[i].get();
    if (!e.empty() && failed_at < 0) {
      failed_at = i;
      first_err = e;
    }
  }
  const std::vector<uint32_t> crcs = enc.crc;
  store_->ec_free(&enc);
  if (failed_at >= 0)  // the reference's try_join_all: one failed shard fails the write
    return send_response(fd, FpStatus::IoError, 0, 0, "Shard " + std::to_string(failed_at) + " write failed: " + first_err);
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.ec_device_writes++;
  }
  // the shard CRCs travel back in the message: the client records nothing per shard, but
  // tests compare them with the CPU codec
  std::string crc_list;
  for (uint32_t c : crcs) crc_list += std::to_string(c) + ",";
  return send_response(fd, FpStatus::Ok, sl, static_cast<uint64_t>(k + m), crc_list);
}

bool FastPathServer::ec_read(int fd, const uint8_t* body, const uint8_t* end) {
  Reader rd{body, end};
  uint64_t offset = rd.get<uint64_t>(), length = rd.get<uint64_t>();
  uint16_t k = rd.get<uint16_t>(), m = rd.get<uint16_t>();
  uint64_t sl = rd.get<uint64_t>(), orig = rd.get<uint64_t>(), shm_off = rd.get<uint64_t>(), cap = rd.get<uint64_t>();
  std::string id = rd.str(), path = rd.str();
  std::vector<std::string> locs = read_list(rd, false);
  std::string rid = rd.p < rd.end ? rd.str() : std::string();
  RequestScope rs(rid);
  note_rid(rid);
  TraceRange tr("dfs.fp.ec_read");
  auto fallback = [&](const std::string& why) {
    std::lock_guard<std::mutex> g(mu_);
    st_.ec_device_fallbacks++;
    return send_response(fd, FpStatus::Unsupported, 0, 0, why);
  };
  if (!rd.ok || id.empty() || k == 0 || m == 0 || k + m > kMaxShards || locs.size() != size_t(k) + m || sl == 0 ||
      sl > kMaxTransfer || orig == 0 || orig > sl * k || (length > 0 && offset >= orig))
    return send_response(fd, FpStatus::BadRequest, 0, 0, "malformed ec read");
  const uint64_t from = length > 0 ? offset : 0, want = length > 0 ? std::min<uint64_t>(length, orig - offset) : orig;
  std::string err;
  uint8_t* base = want > cap ? nullptr : map_shm(path, shm_off, cap, &err);
  if (base == nullptr) return fallback(want > cap ? "slot too small" : "short-circuit unavailable: " + err);
  EcGather g;
  if (!ec_gather(id, locs, sl, -1, k, &g, &err)) return fallback(err);
  std::vector<int> present, missing;
  for (int i = 0; i < k + m; ++i)
    if (g.ptrs[i]) present.push_back(i);
    else if (i < k) missing.push_back(i);
  if (static_cast<int>(present.size()) < k) {
    if (g.unreachable > 0) return fallback("surviving shards not reachable over the engine");
    return send_response(fd, FpStatus::IoError, 0, 0, "RS reconstruct error: TooFewShardsPresent");
  }
  present.resize(k);
  ChunkStore::EcBuffers dec;
  if (!missing.empty()) {
    std::vector<const uint8_t*> in;
    for (int i : present) in.push_back(g.ptrs[i]);
    gf::Matrix rows = gf::rs_decode_rows(k, m, present, missing);
    if (!store_->ec_decode(rows, in, sl, &dec, &err)) return fallback(err);
  }
  // the requested range of the original bytes, stripe by stripe, HBM -> the client's slot
  bool ok = true;
  for (int c = 0; ok && c < k; ++c) {
    const uint64_t lo = std::max<uint64_t>(from, c * sl), hi = std::min<uint64_t>(from + want, (c + 1) * sl);
    if (lo >= hi) continue;
    const uint8_t* src = g.ptrs[c];
    if (!src) {
      auto it = std::find(missing.begin(), missing.end(), c);
      src = dec.shard(static_cast<int>(it - missing.begin()));
    }
    ok = store_->device_to_host(base + shm_off + (lo - from), src + (lo - c * sl), hi - lo);
  }
  store_->ec_free(&dec);
  {
    std::lock_guard<std::mutex> lk(mu_);
    st_.ec_device_reads++;
    if (!missing.empty()) st_.ec_device_decodes++;
  }
  return ok ? send_response(fd, FpStatus::Ok, orig, want, "") : send_response(fd, FpStatus::IoError, 0, 0, "copy out failed");
}

}  // namespace dfs
