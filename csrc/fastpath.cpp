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
    if (it != maps_.end()) {  // the client recreated a bigger arena: remap
      ::munmap(it->second.p, it->second.size);
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

void FastPathServer::serve(int fd) {
  std::vector<uint8_t> body;
  while (!stop_.load()) {
    uint32_t n = 0;
    if (!read_full(fd, &n, 4) || n == 0 || n > kMaxBody) break;
    body.resize(n);
    if (!read_full(fd, body.data(), n)) break;
    Reader rd{body.data() + 1, body.data() + n};
    uint8_t op = body[0];
    bool sent = false;
    if (op == 1) {  // WRITE (no downstream replicas)
      uint64_t term = rd.get<uint64_t>();
      uint32_t crc = rd.get<uint32_t>();
      uint64_t off = rd.get<uint64_t>(), len = rd.get<uint64_t>();
      std::string id = rd.str(), path = rd.str();
      if (!rd.ok || id.empty()) {
        sent = send_response(fd, FpStatus::BadRequest, 0, 0, "malformed write request");
      } else {
        uint64_t known = 0;
        std::string err;
        uint8_t* base = nullptr;
        if (!fence(term, &known)) {
          {
            std::lock_guard<std::mutex> g(mu_);
            st_.fenced++;
          }
          sent = send_response(fd, FpStatus::Fenced, known, 0,
                               "Stale master term: request has " + std::to_string(term) + " but known term is " +
                                   std::to_string(known));
        } else if ((base = map_shm(path, off + len, &err)) == nullptr) {
          sent = send_response(fd, FpStatus::Unsupported, 0, 0, "short-circuit unavailable: " + err);
        } else {
          WriteResult wr = store_->write(id, base + off, len, crc);
          if (wr.ok) {
            {
              std::lock_guard<std::mutex> g(mu_);
              st_.writes++;
            }
            sent = send_response(fd, FpStatus::Ok, len, len, "");
          } else {
            sent = send_response(fd, FpStatus::IoError, 0, 0, wr.error);
          }
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
            {
              std::lock_guard<std::mutex> g(mu_);
              st_.reads++;
            }
            sent = send_response(fd, FpStatus::Ok, rr.total_size, rr.bytes, "");
          } else if (rr.status == ReadStatus::Ok) {
            {
              std::lock_guard<std::mutex> g(mu_);
              suspects_.push_back(id);
              st_.reads++;
            }
            sent = send_response(fd, FpStatus::PartialCorrupt, rr.total_size, rr.bytes, rr.error);
          } else {
            {
              std::lock_guard<std::mutex> g(mu_);
              st_.punts++;
            }
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
