// Native local data path of a ChunkServer; see fastpath.h for protocol and scope.
#include "fastpath.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <future>

namespace dfs {

namespace {

constexpr uint32_t kMaxBody = 1 << 16;
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
  acceptor_ = std::thread([this] { accept_loop(); });
  return true;
}

void FastPathServer::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  std::vector<std::thread> ws;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    ws.swap(workers_);
  }
  for (auto& t : ws)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : maps_) ::munmap(kv.second.p, kv.second.size);
  maps_.clear();
  for (auto& m : retired_) ::munmap(m.p, m.size);
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
    std::lock_guard<std::mutex> g(mu_);
    if (stop_.load()) {
      ::close(fd);
      break;
    }
    conns_.push_back(fd);
    st_.connections++;
    workers_.emplace_back([this, fd] { serve(fd); });
  }
}

uint8_t* FastPathServer::map_shm(const std::string& path, uint64_t need, std::string* err) {
  if (!valid_shm_path(path)) {
    *err = "refusing shared-memory path " + path;
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = maps_.find(path);
    if (it != maps_.end() && it->second.size >= need) return it->second.p;
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
  if (::fstat(fd, &sb) != 0 || static_cast<uint64_t>(sb.st_size) < need) {
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
    return m.p;
  }
  m.p = static_cast<uint8_t*>(p);
  m.size = static_cast<uint64_t>(sb.st_size);
  return m.p;
}

void FastPathServer::set_rccl(RcclEngine* engine) { rccl_ = engine; }

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

bool FastPathServer::forward(const std::string& id, uint32_t crc, uint64_t term, const std::vector<std::string>& next,
                             const ShmSrc& src, int* replicas, std::string* err) {
  *replicas = 0;
  Peer* p = next.empty() ? nullptr : local_peer(next[0]);
  if (p == nullptr) {
    *err = "no native route to " + (next.empty() ? std::string("?") : next[0]);
    return false;
  }
  bool use_rccl = rccl_ != nullptr && p->rank >= 0 && rccl_->pair_ok(rccl_->rank(), p->rank);
  bool use_shm = !use_rccl && !src.path.empty();
  if (!use_rccl && !use_shm) {
    *err = "no RCCL pair and no shared-memory source for " + next[0];
    return false;
  }
  int fd = -1;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (!p->idle.empty()) {
      fd = p->idle.back();
      p->idle.pop_back();
    }
  }
  if (fd < 0 && (fd = connect_abstract(p->name)) < 0) {
    *err = "cannot reach fast path of " + next[0];
    return false;
  }
  auto put_next = [&](std::vector<uint8_t>& req) {
    put<uint16_t>(req, static_cast<uint16_t>(next.size() - 1));
    for (size_t i = 1; i < next.size(); ++i) put_str(req, next[i]);
  };
  std::vector<uint8_t> req(4, 0), resp;
  bool io_ok;
  if (use_rccl) {
    // payload GPU->GPU over xGMI (ncclSend from HBM), descriptor over the socket
    uint64_t size = 0;
    int64_t seq = rccl_->send(p->rank, id, &size, err);
    if (seq < 0) {
      std::lock_guard<std::mutex> g(p->mu);
      p->idle.push_back(fd);
      return false;
    }
    req.push_back(3);
    put<uint64_t>(req, term);
    put<uint32_t>(req, crc);
    put<int32_t>(req, rccl_->rank());
    put<int64_t>(req, seq);
    put<uint64_t>(req, size);
    put_str(req, id);
    put_next(req);
    finish_frame(req);
    io_ok = exchange(fd, req, &resp);
    std::string werr;
    bool sent = rccl_->wait_send(p->rank, seq, &werr);
    if (!io_ok || !sent) {
      ::close(fd);
      // an unmatched send would wedge this pair's stream: retire it; the next block on
      // this hop uses the shared-memory route (or the client's gRPC fallback)
      rccl_->abort_pair(rccl_->rank(), p->rank);
      *err = !io_ok ? "descriptor to " + next[0] + " failed" : "RCCL send failed: " + werr;
      return false;
    }
  } else {
    // same-host hop without RCCL: the next server stages straight from the client's
    // shared-memory slot (H2D on its own GPU) — no payload on any socket
    req.push_back(4);
    put<uint64_t>(req, term);
    put<uint32_t>(req, crc);
    put<uint64_t>(req, src.off);
    put<uint64_t>(req, src.len);
    put_str(req, id);
    put_str(req, src.path);
    put_next(req);
    finish_frame(req);
    io_ok = exchange(fd, req, &resp);
    if (!io_ok) {
      ::close(fd);
      *err = "forward to " + next[0] + " failed";
      return false;
    }
  }
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->idle.push_back(fd);
  }
  if (static_cast<FpStatus>(resp[0]) != FpStatus::Ok) {
    *err = "downstream " + next[0] + ": " + resp_msg(resp);
    return false;
  }
  uint64_t downstream = 0;
  std::memcpy(&downstream, resp.data() + 9, 8);
  *replicas = static_cast<int>(downstream);
  std::lock_guard<std::mutex> g(mu_);
  if (use_rccl) st_.rccl_forwards++;
  else st_.shm_forwards++;
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
  // Local persist and downstream forward run concurrently; the ack waits for both.
  auto persist_and_forward = [&](const std::string& id, const uint8_t* host, uint64_t len, uint32_t crc,
                                 uint64_t term, const std::vector<std::string>& next, const ShmSrc& src) -> bool {
    int down = 0;
    std::string ferr, perr;
    auto fut = std::async(std::launch::async, [&] { return forward(id, crc, term, next, src, &down, &ferr); });
    bool pok = store_->persist(id, host, host ? len : 0, &perr);
    bool fok = fut.get();
    if (!pok) return send_response(fd, FpStatus::IoError, 0, 0, perr);
    if (!fok) {
      bump(&FpStats::forward_failures);
      return send_response(fd, FpStatus::Unsupported, 0, 0, "native forward failed: " + ferr);
    }
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
      std::string err;
      uint8_t* base = nullptr;
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed write request");
      } else if (fenced(term, &msg)) {
        sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
      } else if (!next.empty() && local_peer(next[0]) == nullptr) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "no native route for the chain");
      } else if ((base = map_shm(path, off + len, &err)) == nullptr) {
        sent = send_response(fd, FpStatus::Unsupported, 0, 0, "short-circuit unavailable: " + err);
      } else if (next.empty()) {
        WriteResult wr = store_->write(id, base + off, len, crc);
        if (wr.ok) bump(&FpStats::writes);
        sent = wr.ok ? send_response(fd, FpStatus::Ok, len, 1, "") : send_response(fd, FpStatus::IoError, 0, 0, wr.error);
      } else {
        WriteResult wr = store_->stage(id, base + off, len, crc);  // HBM + CRC verify, not yet durable
        if (!wr.ok) {
          sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
        } else {
          bump(&FpStats::writes);
          sent = persist_and_forward(id, base + off, len, crc, term, next, ShmSrc{path, off, len});
        }
      }
    } else if (op == 3) {  // REPL: block arrives over RCCL from the previous hop
      uint64_t term = rd.get<uint64_t>();
      uint32_t crc = rd.get<uint32_t>();
      int32_t src = rd.get<int32_t>();
      int64_t seq = rd.get<int64_t>();
      uint64_t size = rd.get<uint64_t>();
      std::string id = rd.str();
      std::vector<std::string> next = read_list(rd, false);
      if (!rd.ok || id.empty() || rccl_ == nullptr) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, rccl_ ? "malformed replicate request" : "RCCL disabled");
      } else {
        // The recv must be posted even when the request is refused, or the sender's
        // ncclSend never completes; recv first, then judge the request.
        bool last = next.empty();
        bool stale = fenced(term, &msg);
        WriteResult wr = rccl_->recv(src, seq, id, size, crc, last && !stale);
        if (stale) {
          sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
        } else if (!wr.ok) {
          sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
        } else {
          bump(&FpStats::replicas_in);
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
      std::string err;
      uint8_t* base = nullptr;
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed replicate request");
      } else if (fenced(term, &msg)) {
        sent = send_response(fd, FpStatus::Fenced, term_.load(), 0, msg);
      } else if ((base = map_shm(path, off + len, &err)) == nullptr) {
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
    } else if (op == 2) {  // READ into the client's slot
      uint64_t offset = rd.get<uint64_t>(), length = rd.get<uint64_t>();
      uint64_t shm_off = rd.get<uint64_t>(), cap = rd.get<uint64_t>();
      std::string id = rd.str(), path = rd.str();
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
        } else if ((base = map_shm(path, shm_off + cap, &err)) == nullptr) {
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
}

}  // namespace dfs
