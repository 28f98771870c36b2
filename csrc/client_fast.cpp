#include "client_fast.h"
#include "gf256.h"
#include "trace.h"

#include <fcntl.h>
#include <openssl/evp.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstddef>
#include <cstring>
#include <future>
#include <random>

#include "crc32.h"
#include "dfs_pb.h"

namespace dfs {

namespace {

// 128 random bits as 32 hex digits, like the Python client's uuid4().hex
std::string new_request_id() {
  thread_local std::mt19937_64 rng{std::random_device{}() ^ (static_cast<uint64_t>(::getpid()) << 32)};
  char buf[33];
  std::snprintf(buf, sizeof buf, "%016llx%016llx", static_cast<unsigned long long>(rng()),
                static_cast<unsigned long long>(rng()));
  return buf;
}


using Clock = std::chrono::steady_clock;

double since(Clock::time_point& t) {
  auto now = Clock::now();
  double d = std::chrono::duration<double>(now - t).count();
  t = now;
  return d;
}

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

std::string strip_scheme(const std::string& a) {
  auto p = a.find("://");
  std::string s = p == std::string::npos ? a : a.substr(p + 3);
  while (!s.empty() && s.back() == '/') s.pop_back();
  return s;
}

// "http://127.0.0.1:50051" -> "dfs_rpc_50051" for loopback targets, else "".
std::string local_rpc_name(const std::string& addr) {
  if (addr.rfind("https://", 0) == 0) return "";
  std::string a = strip_scheme(addr);
  auto colon = a.rfind(':');
  if (colon == std::string::npos) return "";
  std::string host = a.substr(0, colon), port = a.substr(colon + 1);
  if (host != "127.0.0.1" && host != "localhost" && host != "::1" && host != "[::1]") return "";
  if (port.empty() || port.find_first_not_of("0123456789") != std::string::npos) return "";
  return "dfs_rpc_" + port;
}

int connect_abstract(const std::string& name) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  if (name.size() + 1 > sizeof(sa.sun_path)) {
    ::close(fd);
    return -1;
  }
  std::memcpy(sa.sun_path + 1, name.data(), name.size());
  socklen_t len = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name.size());
  if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), len) != 0) {
    ::close(fd);
    return -1;
  }
  timeval tv{120, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  return fd;
}

bool send_all(int fd, const std::string& s) {
  const char* p = s.data();
  size_t n = s.size();
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

bool recv_all(int fd, void* buf, size_t n) {
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

template <class T>
void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof v);
}

void put_str(std::string& s, const std::string& v) {
  put<uint16_t>(s, static_cast<uint16_t>(v.size()));
  s += v;
}

std::string md5_hex(const uint8_t* p, size_t n) {
  unsigned char d[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_Digest(p, n, d, &len, EVP_md5(), nullptr);
  static const char* hx = "0123456789abcdef";
  std::string out;
  for (unsigned i = 0; i < len; ++i) {
    out.push_back(hx[d[i] >> 4]);
    out.push_back(hx[d[i] & 15]);
  }
  return out;
}

constexpr int kOutOfRange = 11, kFailedPrecondition = 9, kUnavailable = 14, kNotFound = 5;

}  // namespace

FastClient::FastClient(std::string fastpath_socket, std::string local_chunkserver, size_t arena_bytes,
                       size_t slot_bytes, int hash_threads)
    : fp_socket_(std::move(fastpath_socket)), local_cs_(strip_scheme(local_chunkserver)), slot_bytes_(slot_bytes) {
  arena_bytes_ = std::max(slot_bytes, arena_bytes / slot_bytes * slot_bytes);
  std::random_device rd;
  char name[96];
  std::snprintf(name, sizeof name, "/dev/shm/dfs_sc_%d_n%08x", static_cast<int>(::getpid()), rd());
  int fd = ::open(name, O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0600);
  if (fd >= 0) {
    if (::ftruncate(fd, static_cast<off_t>(arena_bytes_)) == 0) {
      // populated up front: a slot's first use in a timed loop must not take 256 page faults
      // (each allocating and zeroing a shmem page) inside its copy
      void* p = ::mmap(nullptr, arena_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, 0);
      if (p != MAP_FAILED) {
        base_ = static_cast<uint8_t*>(p);
        arena_path_ = name;
      }
    }
    ::close(fd);
    if (!base_) ::unlink(name);
  }
  for (int64_t off = 0; off + static_cast<int64_t>(slot_bytes_) <= static_cast<int64_t>(arena_bytes_);
       off += static_cast<int64_t>(slot_bytes_))
    free_slots_.push_back(off);
  for (int i = 0; i < std::max(1, hash_threads); ++i) hashers_.emplace_back([this] { hash_loop(); });
  {
    // the ETag hashes: AVX-512 lanes under a small CPU budget, else 2 messages interleaved per
    // scalar thread (DFS_MD5_LANES), enough engines for hash_threads messages in flight
    const auto kind = Md5MultiBuffer::wanted();
    const char* ln = std::getenv("DFS_MD5_LANES");
    const int lanes = ln && *ln ? std::atoi(ln) : 2;
    if (kind == Md5MultiBuffer::Kind::Avx512)
      md5mb_ = std::make_unique<Md5MultiBuffer>(std::max(1, (hash_threads + 15) / 16), kind);
    else if (kind == Md5MultiBuffer::Kind::Scalar)
      md5mb_ = std::make_unique<Md5MultiBuffer>(std::max(1, (hash_threads + lanes - 1) / lanes), kind, lanes);
  }
}

FastClient::~FastClient() {
  {
    std::lock_guard<std::mutex> g(q_mu_);
    stop_ = true;
  }
  q_cv_.notify_all();
  for (auto& t : hashers_) t.join();
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (auto& kv : idle_)
      for (int fd : kv.second) ::close(fd);
    idle_.clear();
  }
  if (base_) {
    ::munmap(base_, arena_bytes_);
    ::unlink(arena_path_.c_str());
  }
}

void FastClient::hash_loop() {
  for (;;) {
    std::function<void()> job;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
      if (queue_.empty()) return;
      job = std::move(queue_.front());
      queue_.pop_front();
    }
    job();
  }
}

void FastClient::set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters) {
  ShardMap m = shard_map_json.empty() ? ShardMap::new_range() : ShardMap::from_json(Json::parse(shard_map_json));
  std::lock_guard<std::mutex> g(route_mu_);
  map_ = std::move(m);
  have_map_ = !shard_map_json.empty();
  masters_ = masters;
}

std::string FastClient::master_socket(const std::string& path) {
  std::lock_guard<std::mutex> g(route_mu_);
  std::string addr;
  if (have_map_) {
    std::string shard = map_.get_shard(path);
    const auto* peers = shard.empty() ? nullptr : map_.peers(shard);
    if (peers && !peers->empty()) addr = peers->front();
  }
  if (addr.empty() && !masters_.empty()) addr = masters_.front();
  return addr.empty() ? std::string() : local_rpc_name(addr);
}

int64_t FastClient::acquire(size_t n) {
  if (!base_ || n > slot_bytes_) return -1;
  std::unique_lock<std::mutex> lk(slot_mu_);
  if (!slot_cv_.wait_for(lk, std::chrono::seconds(5), [&] { return !free_slots_.empty(); })) return -1;
  int64_t s = free_slots_.back();
  free_slots_.pop_back();
  return s;
}

void FastClient::release(int64_t slot) {
  slot -= slot % static_cast<int64_t>(slot_bytes_);  // a range read hands out slot + shift
  {
    std::lock_guard<std::mutex> g(slot_mu_);
    free_slots_.push_back(slot);
  }
  slot_cv_.notify_one();
}

int FastClient::take_conn(const std::string& name) {
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    auto& v = idle_[name];
    if (!v.empty()) {
      int fd = v.back();
      v.pop_back();
      return fd;
    }
  }
  return connect_abstract(name);
}

void FastClient::give_conn(const std::string& name, int fd) {
  std::lock_guard<std::mutex> g(conn_mu_);
  idle_[name].push_back(fd);
}

bool FastClient::call(const std::string& sock, const std::string& method_path, const std::string& rid,
                      const std::string& req, int* code, std::string* resp) {
  int fd = take_conn(sock);
  if (fd < 0) return false;
  std::string msg;
  msg.reserve(8 + method_path.size() + rid.size() + req.size());
  put<uint32_t>(msg, static_cast<uint32_t>(2 + method_path.size() + 2 + rid.size() + req.size()));
  put_str(msg, method_path);
  put_str(msg, rid);  // x-request-id: the master's handlers and logs see the client's id
  msg += req;
  uint32_t n = 0;
  if (!send_all(fd, msg) || !recv_all(fd, &n, 4) || n == 0 || n > (1u << 30)) {
    ::close(fd);
    return false;
  }
  resp->resize(n);
  if (!recv_all(fd, resp->data(), n)) {
    ::close(fd);
    return false;
  }
  give_conn(sock, fd);
  *code = static_cast<uint8_t>((*resp)[0]);
  resp->erase(0, 1);
  return true;
}

bool FastClient::fp_call(uint8_t op, const std::string& body, uint8_t* status, uint64_t* total, uint64_t* nbytes,
                         std::string* msg) {
  return fp_call_to(fp_socket_, op, body, status, total, nbytes, msg);
}

bool FastClient::fp_call_to(const std::string& sock, uint8_t op, const std::string& body, uint8_t* status,
                            uint64_t* total, uint64_t* nbytes, std::string* msg) {
  const std::string& fp_socket_ = sock;  // the connection pool is keyed by socket name
  int fd = take_conn(fp_socket_);
  if (fd < 0) return false;
  std::string req;
  put<uint32_t>(req, static_cast<uint32_t>(body.size() + 1));
  req.push_back(static_cast<char>(op));
  req += body;
  uint32_t n = 0;
  std::string resp;
  if (!send_all(fd, req) || !recv_all(fd, &n, 4) || n < 19 || n > (1u << 20)) {
    ::close(fd);
    return false;
  }
  resp.resize(n);
  if (!recv_all(fd, resp.data(), n)) {
    ::close(fd);
    return false;
  }
  give_conn(fp_socket_, fd);
  *status = static_cast<uint8_t>(resp[0]);
  std::memcpy(total, resp.data() + 1, 8);
  std::memcpy(nbytes, resp.data() + 9, 8);
  uint16_t ml;
  std::memcpy(&ml, resp.data() + 17, 2);
  msg->assign(resp, 19, std::min<size_t>(ml, resp.size() - 19));
  return true;
}

FastClient::Status FastClient::write(const std::string& path, const uint8_t* data, size_t n, int* replicas,
                                     std::string* msg, Times* t, const std::string& rid_in,
                                     const std::map<std::string, std::string>* attrs) {
  if (!base_ || n > slot_bytes_) return NotHandled;
  auto c0 = Clock::now();
  int64_t slot = acquire(n);
  if (slot < 0) return NotHandled;
  t->acquire = std::chrono::duration<double>(Clock::now() - c0).count();
  // the MD5 and the CRC read the caller's buffer while it is copied into the slot, so neither
  // waits for the copy (the MD5, ~1 ms per MiB, is the write's longest chain)
  Hashes h;
  struct Join {
    Hashes& h;
    ~Join() { h.wait(); }
  } join{h};
  start_hashes(data, n, true, &h);
  std::memcpy(base_ + slot, data, n);
  t->copy = since(c0);
  std::string md5;
  Status st = write_slot_impl(path, slot, n, replicas, msg, t, rid_in, attrs, nullptr, &md5, &h);
  h.wait();
  release(slot);
  return st;
}

void FastClient::start_hashes(const uint8_t* p, size_t n, bool with_crc, Hashes* h) {
  std::shared_ptr<std::packaged_task<std::string()>> md5_task;
  if (md5mb_) {
    h->md5 = md5mb_->submit(p, n);  // a lane of the multi-buffer engine
  } else {
    md5_task = std::make_shared<std::packaged_task<std::string()>>([p, n] { return md5_hex(p, n); });
    h->md5 = md5_task->get_future();
  }
  std::shared_ptr<std::packaged_task<uint32_t()>> crc_task;
  if (with_crc) {
    crc_task = std::make_shared<std::packaged_task<uint32_t()>>([p, n] { return crc32(p, n); });
    h->crc = crc_task->get_future();
  }
  if (!md5_task && !crc_task) return;
  {
    std::lock_guard<std::mutex> g(q_mu_);
    if (md5_task) queue_.emplace_back([md5_task] { (*md5_task)(); });
    if (crc_task) queue_.emplace_front([crc_task] { (*crc_task)(); });
  }
  if (md5_task && crc_task) q_cv_.notify_all();
  else q_cv_.notify_one();
}

int64_t FastClient::acquire_slot(size_t n) { return acquire(n); }

FastClient::Status FastClient::write_slot(const std::string& path, int64_t slot, size_t n, int* replicas,
                                          std::string* msg, Times* t, const std::string& rid_in,
                                          const std::map<std::string, std::string>* attrs, const char* etag_attr,
                                          std::string* md5_out) {
  return write_slot_impl(path, slot, n, replicas, msg, t, rid_in, attrs, etag_attr, md5_out, nullptr);
}

FastClient::Status FastClient::write_slot_impl(const std::string& path, int64_t slot, size_t n, int* replicas,
                                               std::string* msg, Times* t, const std::string& rid_in,
                                               const std::map<std::string, std::string>* attrs,
                                               const char* etag_attr, std::string* md5_out, Hashes* pre) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.client.write");
  if (!base_ || n > slot_bytes_ || slot < 0) return NotHandled;
  std::string sock = master_socket(path);
  if (sock.empty()) return NotHandled;
  const uint8_t* data = base_ + slot;
  auto clk = Clock::now();
  // MD5 (the ETag) is a sequential chain and only CompleteFile needs it: hash on a worker
  // while the create RPC, the CRC and the block transfer run here (write() started it, and
  // the CRC, on its own buffer already)
  Hashes own;
  struct Join {  // never return while the worker still reads the buffer
    Hashes& h;
    ~Join() { h.wait(); }
  } join{own};
  Hashes& h = pre ? *pre : own;
  if (!pre) start_hashes(data, n, false, &own);
  std::future<std::string>& md5 = h.md5;
  uint32_t crc = 0;
  bool have_crc = false;
  if (!h.crc.valid()) {
    crc = crc32(data, n);
    have_crc = true;
  }
  t->crc = since(clk);

  pb::CreateFileRequest creq;
  creq.path = path;
  creq.allocate_block = true;
  creq.defer_create = true;
  creq.preferred_chunk_server = local_cs_;
  int code;
  std::string raw;
  if (!call(sock, "/dfs.MasterService/CreateFile", rid, creq.str(), &code, &raw)) return NotHandled;
  if (code == kOutOfRange || code == kFailedPrecondition || code == kUnavailable) return NotHandled;
  if (code != 0) {
    *msg = "Failed to create file: " + raw;
    return Failed;
  }
  pb::CreateFileResponse cresp;
  if (!cresp.decode(raw)) return NotHandled;
  if (!cresp.success) {
    if (cresp.error_message == "Not Leader") return NotHandled;
    *msg = "Failed to create file: " + cresp.error_message;
    return Failed;
  }
  if (!cresp.has_allocation || !cresp.allocation.has_block) return NotHandled;
  const pb::AllocateBlockResponse& alloc = cresp.allocation;
  if (alloc.chunk_server_addresses.empty()) {
    *msg = "No chunk servers available";
    return Failed;
  }
  if (!cresp.deferred || strip_scheme(alloc.chunk_server_addresses[0]) != local_cs_)
    return NotHandled;  // nothing was recorded yet: the Python path redoes it
  if (!have_crc) crc = h.crc.get();  // computed beside the copy and the create RPC
  t->create = since(clk);

  std::string body;
  put<uint64_t>(body, alloc.master_term);
  put<uint32_t>(body, crc);
  put<uint64_t>(body, static_cast<uint64_t>(slot));
  put<uint64_t>(body, n);
  put_str(body, alloc.block.block_id);
  put_str(body, arena_path_);
  put<uint16_t>(body, static_cast<uint16_t>(alloc.chunk_server_addresses.size() - 1));
  for (size_t i = 1; i < alloc.chunk_server_addresses.size(); ++i)
    put_str(body, strip_scheme(alloc.chunk_server_addresses[i]));
  put_str(body, rid);
  uint8_t st;
  uint64_t total, written;
  std::string fmsg;
  bool sent = fp_call(1, body, &st, &total, &written, &fmsg);
  if (!sent) return NotHandled;
  if (st == 5 || st == 4) {  // fenced / I/O error: what the gRPC path would report
    *msg = "Failed to write block: " + fmsg;
    return Failed;
  }
  if (st != 0) return NotHandled;
  *replicas = static_cast<int>(written);
  t->write = since(clk);

  pb::CompleteFileRequest done;
  done.path = path;
  done.size = n;
  done.etag_md5 = md5.get();
  *md5_out = done.etag_md5;
  t->md5_wait = since(clk);
  done.created_at_ms = static_cast<uint64_t>(now_ms());
  pb::BlockChecksumInfo sum;
  sum.block_id = alloc.block.block_id;
  sum.checksum_crc32c = crc;
  sum.actual_size = n;
  done.block_checksums.push_back(sum);
  done.create = true;
  done.ec_data_shards = alloc.ec_data_shards;
  done.ec_parity_shards = alloc.ec_parity_shards;
  done.blocks.push_back(alloc.block);
  if (attrs) done.attributes = *attrs;
  if (etag_attr) done.attributes[etag_attr] = "\"" + done.etag_md5 + "\"";
  if (!call(sock, "/dfs.MasterService/CompleteFile", rid, done.str(), &code, &raw)) {
    *msg = "Failed to complete file: master connection lost";
    return Failed;
  }
  if (code != 0) {
    *msg = "Failed to complete file: " + raw;
    return Failed;
  }
  pb::CompleteFileResponse dresp;
  dresp.decode(raw);
  if (!dresp.success) {
    *msg = dresp.error_message.empty() ? "Failed to complete file" : "Failed to create file: " + dresp.error_message;
    return Failed;
  }
  t->complete = since(clk);
  writes_++;
  return Ok;
}

FastClient::Status FastClient::list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
                                    const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.client.list");
  std::vector<std::string> socks;
  {
    std::lock_guard<std::mutex> g(route_mu_);
    if (have_map_) {
      for (const auto& shard : map_.shards()) {
        const auto* peers = map_.peers(shard);
        if (!peers || peers->empty()) return NotHandled;
        socks.push_back(local_rpc_name(peers->front()));
      }
    } else if (!masters_.empty()) {
      socks.push_back(local_rpc_name(masters_.front()));
    }
  }
  if (socks.empty()) return NotHandled;
  pb::ListFilesRequest req;
  req.path = prefix;
  req.with_metadata = true;
  const std::string body = req.str();
  out->clear();
  for (const auto& sock : socks) {
    int code = 0;
    std::string raw;
    if (!call(sock, "/dfs.MasterService/ListFiles", rid, body, &code, &raw) || code != 0) return NotHandled;
    pb::ListFilesResponse resp;
    if (!resp.decode(raw) || resp.metadata.size() != resp.files.size()) return NotHandled;
    for (size_t i = 0; i < resp.files.size(); ++i) out->emplace_back(resp.files[i], std::move(resp.metadata[i]));
  }
  std::sort(out->begin(), out->end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  return Ok;
}

FastClient::Status FastClient::list_components(const std::string& prefix, std::set<std::string>* out,
                                               const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  std::vector<std::string> socks;
  {
    std::lock_guard<std::mutex> g(route_mu_);
    if (have_map_) {
      for (const auto& shard : map_.shards()) {
        const auto* peers = map_.peers(shard);
        if (!peers || peers->empty()) return NotHandled;
        socks.push_back(local_rpc_name(peers->front()));
      }
    } else if (!masters_.empty()) {
      socks.push_back(local_rpc_name(masters_.front()));
    }
  }
  if (socks.empty()) return NotHandled;
  pb::ListFilesRequest req;
  req.path = prefix;
  req.delimiter = "/";
  const std::string body = req.str();
  auto component = [&](const std::string& p) {  // the next path component after `prefix`
    if (p.compare(0, prefix.size(), prefix) != 0) return;
    const size_t e = p.find('/', prefix.size());
    if (e != std::string::npos && e > prefix.size()) out->insert(p.substr(prefix.size(), e - prefix.size()));
  };
  for (const auto& sock : socks) {
    int code = 0;
    std::string raw;
    if (!call(sock, "/dfs.MasterService/ListFiles", rid, body, &code, &raw) || code != 0) return NotHandled;
    pb::ListFilesResponse resp;
    if (!resp.decode(raw)) return NotHandled;
    for (const auto& cp : resp.common_prefixes) component(cp);
    for (const auto& f : resp.files) component(f);  // (a master without the extension lists every path)
  }
  return Ok;
}

FastClient::Status FastClient::stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
                                    const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  std::string sock = master_socket(path);
  if (sock.empty()) return NotHandled;
  pb::GetFileInfoRequest req;
  req.path = path;
  int code;
  std::string raw;
  if (!call(sock, "/dfs.MasterService/GetFileInfo", rid, req.str(), &code, &raw)) return NotHandled;
  if (code == kNotFound) {
    *found = false;
    return Ok;
  }
  if (code != 0) {
    *msg = raw;
    return NotHandled;  // redirect / not leader / unavailable: the Python path follows it
  }
  pb::GetFileInfoResponse info;
  if (!info.decode(raw)) return NotHandled;
  *found = info.found;
  if (info.found) *meta_pb = info.metadata.str();
  return Ok;
}

FastClient::Status FastClient::remove(const std::string& path, std::string* msg, const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  std::string sock = master_socket(path);
  if (sock.empty()) return NotHandled;
  pb::DeleteFileRequest req;
  req.path = path;
  int code;
  std::string raw;
  if (!call(sock, "/dfs.MasterService/DeleteFile", rid, req.str(), &code, &raw)) return NotHandled;
  if (code != 0) {
    *msg = raw;
    return code == kNotFound ? Failed : NotHandled;
  }
  pb::DeleteFileResponse r;
  if (!r.decode(raw)) return NotHandled;
  if (!r.success) {
    if (r.error_message == "Not Leader") return NotHandled;
    *msg = r.error_message;
    return Failed;
  }
  return Ok;
}

FastClient::Status FastClient::rename(const std::string& src, const std::string& dst, std::string* msg,
                                      const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  std::string sock = master_socket(src);
  if (sock.empty()) return NotHandled;
  pb::RenameRequest req;
  req.source_path = src;
  req.dest_path = dst;
  int code;
  std::string raw;
  if (!call(sock, "/dfs.MasterService/Rename", rid, req.str(), &code, &raw)) return NotHandled;
  if (code != 0) {
    *msg = raw;
    return NotHandled;  // redirect / not leader / safe mode: the caller's slower path retries
  }
  pb::RenameResponse r;
  if (!r.decode(raw)) return NotHandled;
  if (!r.success) {
    if (r.error_message == "Not Leader") return NotHandled;
    *msg = r.error_message;
    return Failed;
  }
  return Ok;
}

FastClient::Status FastClient::read(const std::string& path, int64_t* slot, uint64_t* n, std::string* msg,
                                    Times* t, const std::string& rid_in, uint64_t offset, uint64_t length) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.client.read");
  if (!base_) return NotHandled;
  auto clk = Clock::now();
  bool found = false;
  std::string meta;
  Status st = stat(path, &found, &meta, msg, rid);
  if (st != Ok) return st;
  if (!found) {
    *msg = "File not found";
    return Failed;
  }
  t->getinfo = since(clk);
  return read_known(meta, slot, n, msg, t, rid, offset, length);
}

FastClient::Status FastClient::read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg,
                                          Times* t, const std::string& rid_in, uint64_t offset, uint64_t length) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  if (!base_) return NotHandled;
  auto clk = Clock::now();
  pb::FileMetadata m;
  if (!m.decode(meta_pb)) return NotHandled;
  if (m.size == 0) {
    *slot = -1;
    *n = 0;
    return Ok;
  }
  if (m.blocks.size() == 1 && m.blocks[0].ec_data_shards > 0) return read_ec(meta_pb, slot, n, msg, rid, offset, length);
  if (m.blocks.size() != 1) return NotHandled;
  if (length > 0) {
    if (offset >= m.size) return NotHandled;  // the Python path reports the range error
    length = std::min<uint64_t>(length, m.size - offset);
  } else {
    offset = 0;
  }
  const uint64_t want = length > 0 ? length : m.size;
  // a range lands at slot + offset % 16, so the chunkserver's fused verify+copy kernel can
  // store it with aligned 16 B writes (whole blocks start at offset 0 anyway)
  const uint64_t shift = length > 0 ? offset % 16 : 0;
  if (want + shift > slot_bytes_) return NotHandled;
  const pb::BlockInfo& b = m.blocks[0];
  bool local = false;
  for (auto& l : b.locations) local |= strip_scheme(l) == local_cs_;
  if (!local) return NotHandled;
  int64_t s = acquire(slot_bytes_);
  if (s < 0) return NotHandled;
  std::string body;
  put<uint64_t>(body, offset);
  put<uint64_t>(body, length);  // 0 = the whole block
  put<uint64_t>(body, static_cast<uint64_t>(s) + shift);
  put<uint64_t>(body, slot_bytes_ - shift);
  put_str(body, b.block_id);
  put_str(body, arena_path_);
  put_str(body, rid);
  uint8_t st;
  uint64_t total, got;
  std::string fmsg;
  if (!fp_call(2, body, &st, &total, &got, &fmsg) || (st != 0 && st != 8)) {
    release(s);
    return NotHandled;  // corrupt / missing here: the Python path recovers from a replica
  }
  t->read += since(clk);
  *slot = s + static_cast<int64_t>(shift);
  *n = got;
  reads_++;
  return Ok;
}


std::string FastClient::peer_fastpath(const std::string& addr) const {
  // chunkservers listen on the deterministic abstract socket dfs_fp_<grpc port> (same host)
  const std::string a = strip_scheme(addr);
  size_t c = a.rfind(':'), lc = local_cs_.rfind(':');
  if (c == std::string::npos || lc == std::string::npos) return {};
  const std::string host = a.substr(0, c), lhost = local_cs_.substr(0, lc);
  const bool local = host == lhost || host == "127.0.0.1" || host == "localhost" || host == "::1";
  return local ? "dfs_fp_" + a.substr(c + 1) : std::string();
}

bool FastClient::ec_matmul(const std::vector<std::vector<uint8_t>>& mat, int k, uint64_t len, uint64_t in_off,
                           uint64_t out_off, const std::vector<uint16_t>* idx, const std::string& rid) {
  std::string body, flat;
  for (auto& row : mat) flat.append(reinterpret_cast<const char*>(row.data()), row.size());
  put<uint16_t>(body, static_cast<uint16_t>(k));
  put<uint16_t>(body, static_cast<uint16_t>(mat.size()));
  put<uint64_t>(body, len);
  put<uint64_t>(body, in_off);
  put<uint64_t>(body, out_off);
  put_str(body, flat);
  put_str(body, arena_path_);
  put_str(body, rid);
  if (idx) {
    put<uint16_t>(body, static_cast<uint16_t>(idx->size()));
    for (uint16_t v : *idx) put<uint16_t>(body, v);
  }
  uint8_t st;
  uint64_t total, got;
  std::string fmsg;
  if (fp_call(6, body, &st, &total, &got, &fmsg) && st == 0) {
    ec_gpu_++;
    return true;
  }
  // no GPU behind the fast path (host store) or no room: the CPU codec, same bytes
  const uint64_t stride = (len + 15) / 16 * 16;
  std::vector<const uint8_t*> in(k);
  std::vector<uint8_t*> out(mat.size());
  for (int c = 0; c < k; ++c) in[c] = base_ + in_off + (idx ? (*idx)[c] : c) * stride;
  for (size_t r = 0; r < mat.size(); ++r) out[r] = base_ + out_off + r * stride;
  gf::matmul_cpu(mat, in.data(), out.data(), len);
  ec_cpu_++;
  return true;
}

FastClient::Status FastClient::write_ec(const std::string& path, const uint8_t* data, size_t n, int k, int m,
                                        std::string* msg, const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? new_request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.client.write_ec");
  if (!base_ || k <= 0 || m <= 0 || k + m > 32 || n == 0) return NotHandled;
  std::string sock = master_socket(path);
  if (sock.empty()) return NotHandled;
  const uint64_t sl = (n + k - 1) / k, stride = (sl + 15) / 16 * 16;
  if (stride * (k + m) > slot_bytes_) return NotHandled;
  pb::CreateFileRequest creq;
  creq.path = path;
  creq.ec_data_shards = k;
  creq.ec_parity_shards = m;
  creq.allocate_block = true;
  creq.defer_create = true;
  creq.preferred_chunk_server = local_cs_;
  int code;
  std::string raw;
  if (!call(sock, "/dfs.MasterService/CreateFile", rid, creq.str(), &code, &raw)) return NotHandled;
  if (code == kOutOfRange || code == kFailedPrecondition || code == kUnavailable) return NotHandled;
  if (code != 0) {
    *msg = "Failed to create file: " + raw;
    return Failed;
  }
  pb::CreateFileResponse cresp;
  if (!cresp.decode(raw)) return NotHandled;
  if (!cresp.success) {
    if (cresp.error_message == "Not Leader") return NotHandled;
    *msg = "Failed to create file: " + cresp.error_message;
    return Failed;
  }
  if (!cresp.has_allocation || !cresp.allocation.has_block || !cresp.deferred) return NotHandled;
  const pb::AllocateBlockResponse& alloc = cresp.allocation;
  if (alloc.ec_data_shards != k || alloc.ec_parity_shards != m) {
    *msg = "Master returned non-EC policy (data=" + std::to_string(alloc.ec_data_shards) + ", parity=" +
           std::to_string(alloc.ec_parity_shards) + ") for EC file";
    return Failed;
  }
  if (alloc.chunk_server_addresses.size() != static_cast<size_t>(k + m)) {
    *msg = "Expected " + std::to_string(k + m) + " chunk servers for EC(" + std::to_string(k) + "," +
           std::to_string(m) + "), got " + std::to_string(alloc.chunk_server_addresses.size());
    return Failed;
  }
  int64_t slot = acquire(stride * (k + m));
  if (slot < 0) return NotHandled;
  struct Rel {
    FastClient* c;
    int64_t s;
    ~Rel() { c->release(s); }
  } rel{this, slot};
  uint8_t* b = base_ + slot;
  for (int c = 0; c < k; ++c) {  // zero-padded stripes (erasure.rs:7-24)
    const uint64_t off = c * sl, have = off < n ? std::min<uint64_t>(sl, n - off) : 0;
    if (have) std::memcpy(b + c * stride, data + off, have);
    if (have < sl) std::memset(b + c * stride + have, 0, sl - have);
  }
  // Device path: the co-located chunkserver takes the k stripes up once, computes the parity
  // in HBM, checksums every shard there and scatters them HBM -> HBM over its replication
  // engine (fast-path op 7); no parity crosses PCIe and no target re-reads our slot.
  bool device_done = false;
  {
    std::string body;
    put<uint64_t>(body, alloc.master_term);
    put<uint16_t>(body, static_cast<uint16_t>(k));
    put<uint16_t>(body, static_cast<uint16_t>(m));
    put<uint64_t>(body, sl);
    put<uint64_t>(body, static_cast<uint64_t>(slot));
    put<uint64_t>(body, stride);
    put_str(body, alloc.block.block_id);
    put_str(body, arena_path_);
    put<uint16_t>(body, static_cast<uint16_t>(k + m));
    for (auto& a : alloc.chunk_server_addresses) put_str(body, strip_scheme(a));
    put_str(body, rid);
    uint8_t st = 0;
    uint64_t total = 0, got = 0;
    std::string fmsg;
    if (fp_call(7, body, &st, &total, &got, &fmsg)) {
      if (st == 0) {
        device_done = true;
        ec_dev_writes_++;
      } else if (st == 4 || st == 5) {
        *msg = fmsg;
        return Failed;
      }
    }
    if (!device_done) ec_host_++;
  }
  std::vector<std::future<std::pair<int, std::string>>> futs;  // (0 ok, 1 not handled, 2 failed)
  if (!device_done) {
  gf::Matrix full = gf::rs_matrix(k, m), parity(full.begin() + k, full.end());
  ec_matmul(parity, k, sl, static_cast<uint64_t>(slot), static_cast<uint64_t>(slot) + k * stride, nullptr, rid);
  for (int i = 0; i < k + m; ++i) {
    futs.push_back(shard_pool_.submit([this, i, b, slot, stride, sl, &alloc, rid]() -> std::pair<int, std::string> {
      RequestScope scope(rid);
      const std::string addr = strip_scheme(alloc.chunk_server_addresses[i]);
      const uint8_t* p = b + i * stride;
      const uint32_t crc = crc32(p, sl);
      const std::string fps = peer_fastpath(addr);
      if (!fps.empty()) {
        std::string body;
        put<uint64_t>(body, alloc.master_term);
        put<uint32_t>(body, crc);
        put<uint64_t>(body, static_cast<uint64_t>(slot) + i * stride);
        put<uint64_t>(body, sl);
        put_str(body, alloc.block.block_id);
        put_str(body, arena_path_);
        put<uint16_t>(body, 0);
        put_str(body, rid);
        uint8_t st;
        uint64_t total, written;
        std::string fmsg;
        if (fp_call_to(fps, 1, body, &st, &total, &written, &fmsg)) {
          if (st == 0) return {0, ""};
          if (st == 4 || st == 5) return {2, "Shard " + std::to_string(i) + " write failed: " + fmsg};
        }
      }
      pb::WriteBlockRequest req;
      req.block_id = alloc.block.block_id;
      req.expected_checksum_crc32c = crc;
      req.shard_index = i;
      req.master_term = alloc.master_term;
      GrpcResult r = grpc_.call(addr, "/dfs.ChunkServerService/WriteBlock", encode_with_payload(req, p, sl), rid);
      if (!r.transport_ok) return {1, r.message};
      pb::WriteBlockResponse resp;
      if (r.status != 0 || !resp.decode(r.message) || !resp.success)
        return {2, "Shard " + std::to_string(i) + " write failed: " + (r.status ? r.message : resp.error_message)};
      return {0, ""};
    }));
  }
  }  // host path
  int worst = 0;
  std::string why;
  for (auto& f : futs) {
    auto r = f.get();
    if (r.first > worst) {
      worst = r.first;
      why = r.second;
    }
  }
  if (worst == 1) return NotHandled;  // a server we cannot reach natively: the Python path redoes it
  if (worst == 2) {
    *msg = why;
    return Failed;
  }
  pb::CompleteFileRequest done;
  done.path = path;
  done.size = n;
  done.etag_md5 = "";  // the reference leaves EC files without an ETag
  done.created_at_ms = static_cast<uint64_t>(now_ms());
  pb::BlockChecksumInfo sum;
  sum.block_id = alloc.block.block_id;
  sum.checksum_crc32c = crc32(data, n);
  sum.actual_size = n;
  done.block_checksums.push_back(sum);
  done.create = true;
  done.ec_data_shards = k;
  done.ec_parity_shards = m;
  done.blocks.push_back(alloc.block);
  if (!call(sock, "/dfs.MasterService/CompleteFile", rid, done.str(), &code, &raw) || code != 0) {
    *msg = "Failed to complete file: " + (code ? raw : std::string("master connection lost"));
    return Failed;
  }
  pb::CompleteFileResponse dresp;
  dresp.decode(raw);
  if (!dresp.success) {
    *msg = dresp.error_message.empty() ? "Failed to complete file" : "Failed to create file: " + dresp.error_message;
    return Failed;
  }
  writes_++;
  return Ok;
}

FastClient::Status FastClient::read_ec(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg,
                                       const std::string& rid, uint64_t offset, uint64_t length) {
  TraceRange tr("dfs.client.read_ec");
  pb::FileMetadata m;
  if (!m.decode(meta_pb) || m.blocks.size() != 1) return NotHandled;
  const pb::BlockInfo& b = m.blocks[0];
  const int k = b.ec_data_shards, mm = b.ec_parity_shards;
  const uint64_t orig = b.original_size ? b.original_size : m.size;
  if (k <= 0 || mm <= 0 || b.locations.size() != static_cast<size_t>(k + mm) || orig == 0) return NotHandled;
  const uint64_t sl = (orig + k - 1) / k, stride = (sl + 15) / 16 * 16;
  if (stride * (2 * k + mm) > slot_bytes_) return NotHandled;
  if (length > 0 && offset >= orig) return NotHandled;
  int64_t s = acquire(slot_bytes_);
  if (s < 0) return NotHandled;
  uint8_t* base = base_ + s;
  // Data shards first (each straight into the slot by its holder); parity only when one is
  // missing, and then the co-located chunkserver gathers the survivors into its HBM and
  // decodes there (fast-path op 8), falling back to fetching parity here.
  std::vector<std::future<bool>> futs(k + mm);
  auto fetch = [this, s, base, stride, sl, &b, rid](int i) -> bool {
      RequestScope scope(rid);
      const std::string addr = strip_scheme(b.locations[i]);
      if (addr.empty()) return false;  // a shard known lost
      const std::string fps = peer_fastpath(addr);
      if (!fps.empty()) {
        std::string body;
        put<uint64_t>(body, 0);
        put<uint64_t>(body, 0);
        put<uint64_t>(body, static_cast<uint64_t>(s) + i * stride);
        put<uint64_t>(body, stride);
        put_str(body, b.block_id);
        put_str(body, arena_path_);
        put_str(body, rid);
        uint8_t st;
        uint64_t total, got;
        std::string fmsg;
        if (fp_call_to(fps, 2, body, &st, &total, &got, &fmsg) && st == 0 && got == sl) return true;
      }
      pb::ReadBlockRequest req;
      req.block_id = b.block_id;
      GrpcResult r = grpc_.call(addr, "/dfs.ChunkServerService/ReadBlock", req.str(), rid);
      pb::ReadBlockResponse resp;
      if (!r.transport_ok || r.status != 0 || !resp.decode(r.message) || resp.data.size() != sl) return false;
      std::memcpy(base + i * stride, resp.data.data(), sl);
      return true;
  };
  for (int i = 0; i < k; ++i) futs[i] = shard_pool_.submit([&fetch, i] { return fetch(i); });
  std::vector<int> present, missing;
  for (int i = 0; i < k; ++i)
    if (futs[i].get()) present.push_back(i);
    else missing.push_back(i);
  uint64_t from = 0, want = orig;
  if (length > 0) {
    from = offset;
    want = std::min<uint64_t>(length, orig - offset);
  }
  if (!missing.empty() && !local_cs_.empty()) {
    std::string body;
    put<uint64_t>(body, from);
    put<uint64_t>(body, want);
    put<uint16_t>(body, static_cast<uint16_t>(k));
    put<uint16_t>(body, static_cast<uint16_t>(mm));
    put<uint64_t>(body, sl);
    put<uint64_t>(body, orig);
    put<uint64_t>(body, static_cast<uint64_t>(s));
    put<uint64_t>(body, slot_bytes_);
    put_str(body, b.block_id);
    put_str(body, arena_path_);
    put<uint16_t>(body, static_cast<uint16_t>(k + mm));
    for (auto& a : b.locations) put_str(body, strip_scheme(a));
    put_str(body, rid);
    uint8_t st = 0;
    uint64_t total = 0, got = 0;
    std::string fmsg;
    if (fp_call(8, body, &st, &total, &got, &fmsg) && st == 0 && got == want) {
      ec_dev_reads_++;
      ec_degraded_++;
      *slot = s;
      *n = want;
      reads_++;
      return Ok;
    }
    ec_host_++;
  }
  if (!missing.empty()) {
    for (int i = k; i < k + mm; ++i) futs[i] = shard_pool_.submit([&fetch, i] { return fetch(i); });
    for (int i = k; i < k + mm; ++i)
      if (futs[i].get()) present.push_back(i);
  }
  if (!missing.empty()) {
    if (static_cast<int>(present.size()) < k) {
      release(s);
      *msg = "RS reconstruct error: TooFewShardsPresent";
      return Failed;
    }
    std::vector<int> use(present.begin(), present.begin() + k);
    gf::Matrix rows = gf::rs_decode_rows(k, mm, use, missing);
    std::vector<uint16_t> idx(use.begin(), use.end());
    const uint64_t out_off = static_cast<uint64_t>(s) + (k + mm) * stride;
    ec_matmul(rows, k, sl, static_cast<uint64_t>(s), out_off, &idx, rid);
    for (size_t r = 0; r < missing.size(); ++r)
      std::memcpy(base + missing[r] * stride, base_ + out_off + r * stride, sl);
    ec_degraded_++;
  }
  for (int c = 1; c < k; ++c) std::memmove(base + c * sl, base + c * stride, sl);  // stripes back to back
  *slot = s + static_cast<int64_t>(from);
  *n = want;
  reads_++;
  return Ok;
}

}  // namespace dfs
