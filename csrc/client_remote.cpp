// Native remote client; design notes in client_remote.h.
#include "client_remote.h"
#include "gf256.h"

#include <openssl/evp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <future>
#include <random>

#include "crc32.h"
#include "dfs_pb.h"
#include "json.h"
#include "trace.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;
constexpr int kNotFound = 5, kFailedPrecondition = 9, kOutOfRange = 11;

std::string request_id() {
  thread_local std::mt19937_64 rng{std::random_device{}()};
  char buf[33];
  std::snprintf(buf, sizeof buf, "%016llx%016llx", static_cast<unsigned long long>(rng()),
                static_cast<unsigned long long>(rng()));
  return buf;
}

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

// "Not Leader" / "Not Leader|<hint>" in a status message or a response's error field
bool not_leader(const std::string& m, std::string* hint) {
  if (m.compare(0, 10, "Not Leader") != 0) return false;
  auto bar = m.find('|');
  *hint = bar == std::string::npos ? std::string() : m.substr(bar + 1);
  return true;
}

}  // namespace

RemoteClient::RemoteClient(int hash_threads, int timeout_ms, std::shared_ptr<TlsContext> tls)
    : pool_(timeout_ms, std::move(tls)) {
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

RemoteClient::~RemoteClient() {
  {
    std::lock_guard<std::mutex> g(q_mu_);
    stop_ = true;
  }
  q_cv_.notify_all();
  for (auto& t : hashers_) t.join();
}

void RemoteClient::hash_loop() {
  for (;;) {
    std::function<void()> job;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
      if (queue_.empty()) return;
      job = std::move(queue_.front());
      queue_.pop_front();
    }
    job();
  }
}

void RemoteClient::set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters) {
  ShardMap m = shard_map_json.empty() ? ShardMap::new_range() : ShardMap::from_json(Json::parse(shard_map_json));
  std::lock_guard<std::mutex> g(route_mu_);
  map_ = std::move(m);
  have_map_ = !shard_map_json.empty();
  masters_ = masters;
}

std::vector<std::string> RemoteClient::masters_for(const std::string& path, std::string* shard) {
  std::lock_guard<std::mutex> g(route_mu_);
  std::vector<std::string> out;
  shard->clear();
  if (have_map_) {
    *shard = map_.get_shard(path);
    const auto* peers = shard->empty() ? nullptr : map_.peers(*shard);
    if (peers) out = *peers;
  }
  if (out.empty()) out = masters_;
  auto it = leader_.find(*shard);
  if (it != leader_.end()) {
    auto pos = std::find(out.begin(), out.end(), it->second);
    if (pos != out.end()) std::rotate(out.begin(), pos, pos + 1);
  }
  return out;
}

bool RemoteClient::master_call(const std::string& path, const std::string& method, const std::string& req,
                               const std::string& rid, int* code, std::string* resp) {
  std::string shard;
  std::vector<std::string> cands = masters_for(path, &shard);
  return call_candidates(std::move(cands), shard, method, req, rid, code, resp);
}

bool RemoteClient::call_candidates(std::vector<std::string> cands, const std::string& shard, const std::string& method,
                                   const std::string& req, const std::string& rid, int* code, std::string* resp) {
  const std::string full = "/dfs.MasterService/" + method;
  *code = -1;
  bool redirected = false;
  for (size_t i = 0; i < cands.size() && i < 8; ++i) {
    GrpcResult r = pool_.call(cands[i], full, req, rid);
    if (!r.transport_ok) continue;
    std::string hint;
    // "REDIRECT:<addr>": this master's shard does not own the path (our shard map is stale,
    // e.g. after a split); the owner's address is the next candidate. Its answer is not
    // cached as this shard's leader.
    static const std::string kRedirect = "REDIRECT:";
    if (r.status == kOutOfRange && r.message.compare(0, kRedirect.size(), kRedirect) == 0 &&
        r.message.size() > kRedirect.size()) {
      hint = r.message.substr(kRedirect.size());
      if (hint.find("://") == std::string::npos) {
        const size_t sch = cands[i].find("://");
        if (sch != std::string::npos) hint = cands[i].substr(0, sch + 3) + hint;
      }
      if (std::find(cands.begin() + static_cast<long>(i) + 1, cands.end(), hint) == cands.end())
        cands.insert(cands.begin() + static_cast<long>(i) + 1, hint);
      redirected = true;
      continue;
    }
    bool follower = r.status == kFailedPrecondition && not_leader(r.message, &hint);
    if (!follower && r.status == 0 && (method == "CreateFile" || method == "DeleteFile" || method == "Rename")) {
      // these answer a follower's refusal in the response: fields 1 success, 2 error_message,
      // 3 leader_hint, which DeleteFileResponse is exactly (the decoder skips the rest)
      pb::DeleteFileResponse head;
      if (head.decode(r.message) && !head.success && head.error_message == "Not Leader") {
        follower = true;
        hint = head.leader_hint;
      }
    }
    if (follower) {
      if (!hint.empty() && hint.find("://") == std::string::npos) {
        const size_t sch = cands[i].find("://");
        if (sch != std::string::npos) hint = cands[i].substr(0, sch + 3) + hint;
      }
      if (!hint.empty() && std::find(cands.begin() + static_cast<long>(i) + 1, cands.end(), hint) == cands.end())
        cands.insert(cands.begin() + static_cast<long>(i) + 1, hint);
      continue;
    }
    if (!redirected) {
      std::lock_guard<std::mutex> g(route_mu_);
      leader_[shard] = cands[i];
    }
    *code = r.status;
    *resp = std::move(r.message);
    return true;
  }
  return false;
}

FastClient::Status RemoteClient::write(const std::string& path, const uint8_t* data, size_t n, int* replicas,
                                       std::string* msg, Times* t, const std::string& rid_in,
                                       const std::map<std::string, std::string>* attrs) {
  std::string md5;
  return write_etag(path, data, n, replicas, msg, t, rid_in, attrs, nullptr, &md5);
}

FastClient::Status RemoteClient::write_etag(const std::string& path, const uint8_t* data, size_t n, int* replicas,
                                            std::string* msg, Times* t, const std::string& rid_in,
                                            const std::map<std::string, std::string>* attrs, const char* etag_attr,
                                            std::string* md5_out) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.remote.write");
  auto clk = Clock::now();
  std::future<std::string> md5;
  if (md5mb_) {
    md5 = md5mb_->submit(data, n);  // a lane of the multi-buffer engine (md5_mb.h)
  } else {
    auto md5_task = std::make_shared<std::packaged_task<std::string()>>([data, n] { return md5_hex(data, n); });
    md5 = md5_task->get_future();
    {
      std::lock_guard<std::mutex> g(q_mu_);
      queue_.emplace_back([md5_task] { (*md5_task)(); });
    }
    q_cv_.notify_one();
  }
  struct Join {  // never return while the worker still reads the caller's buffer
    std::future<std::string>& f;
    ~Join() {
      if (f.valid()) f.wait();
    }
  } join{md5};
  const uint32_t crc = crc32(data, n);
  t->crc = since(clk);

  pb::CreateFileRequest creq;
  creq.path = path;
  creq.allocate_block = true;
  creq.defer_create = true;
  int code;
  std::string raw;
  if (!master_call(path, "CreateFile", creq.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code == kOutOfRange || code == kFailedPrecondition || code == 14) return FastClient::NotHandled;
  if (code != 0) {
    *msg = "Failed to create file: " + raw;
    return FastClient::Failed;
  }
  pb::CreateFileResponse cresp;
  if (!cresp.decode(raw)) return FastClient::NotHandled;
  if (!cresp.success) {
    if (cresp.error_message == "Not Leader") return FastClient::NotHandled;
    *msg = "Failed to create file: " + cresp.error_message;
    return FastClient::Failed;
  }
  if (!cresp.has_allocation || !cresp.allocation.has_block || !cresp.deferred) return FastClient::NotHandled;
  const pb::AllocateBlockResponse& alloc = cresp.allocation;
  if (alloc.chunk_server_addresses.empty()) {
    *msg = "No chunk servers available";
    return FastClient::Failed;
  }
  t->create = since(clk);

  pb::WriteBlockRequest w;
  w.block_id = alloc.block.block_id;
  for (size_t i = 1; i < alloc.chunk_server_addresses.size(); ++i) w.next_servers.push_back(alloc.chunk_server_addresses[i]);
  w.expected_checksum_crc32c = crc;
  w.shard_index = -1;
  w.master_term = alloc.master_term;
  std::string wire = encode_with_payload(w, data, n);
  GrpcResult wr = pool_.call(alloc.chunk_server_addresses[0], "/dfs.ChunkServerService/WriteBlock", wire, rid);
  std::string().swap(wire);
  if (!wr.transport_ok) {
    *msg = "Failed to write block: " + wr.message;
    return FastClient::Failed;
  }
  if (wr.status != 0) {
    *msg = "Failed to write block: " + wr.message;
    return FastClient::Failed;
  }
  pb::WriteBlockResponse wresp;
  if (!wresp.decode(wr.message) || !wresp.success) {
    *msg = "Failed to write block: " + wresp.error_message;
    return FastClient::Failed;
  }
  *replicas = wresp.replicas_written;
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
  if (!master_call(path, "CompleteFile", done.str(), rid, &code, &raw)) {
    *msg = "Failed to complete file: master unreachable";
    return FastClient::Failed;
  }
  if (code != 0) {
    *msg = "Failed to complete file: " + raw;
    return FastClient::Failed;
  }
  pb::CompleteFileResponse dresp;
  dresp.decode(raw);
  if (!dresp.success) {
    *msg = dresp.error_message.empty() ? "Failed to complete file" : "Failed to create file: " + dresp.error_message;
    return FastClient::Failed;
  }
  t->complete = since(clk);
  writes_++;
  return FastClient::Ok;
}

FastClient::Status RemoteClient::read(const std::string& path, std::string* out, std::string* msg, Times* t,
                                      const std::string& rid_in, uint64_t offset, uint64_t length) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.remote.read");
  auto clk = Clock::now();
  pb::GetFileInfoRequest req;
  req.path = path;
  int code;
  std::string raw;
  if (!master_call(path, "GetFileInfo", req.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code != 0) return code == kNotFound ? (*msg = raw, FastClient::Failed) : FastClient::NotHandled;
  pb::GetFileInfoResponse info;
  if (!info.decode(raw)) return FastClient::NotHandled;
  if (!info.found) {
    *msg = "File not found";
    return FastClient::Failed;
  }
  t->getinfo = since(clk);
  return read_meta(info.metadata, out, msg, t, rid, offset, length);
}

FastClient::Status RemoteClient::read_meta(const pb::FileMetadata& m, std::string* out, std::string* msg, Times* t,
                                           const std::string& rid, uint64_t offset, uint64_t length) {
  RequestScope rs(rid);
  auto clk = Clock::now();
  if (m.size == 0) {
    out->clear();
    reads_++;
    return FastClient::Ok;
  }
  if (m.blocks.size() == 1 && m.blocks[0].ec_data_shards > 0) {
    FastClient::Status st = read_ec(m, out, msg, rid, offset, length);
    if (st == FastClient::Ok) t->read = since(clk);
    return st;
  }
  if (m.blocks.size() != 1) return FastClient::NotHandled;
  if (length > 0) {
    if (offset >= m.size) return FastClient::NotHandled;  // the Python path reports the range error
    length = std::min<uint64_t>(length, m.size - offset);
  } else {
    offset = 0;
    length = m.size;
  }
  const pb::BlockInfo& b = m.blocks[0];
  pb::ReadBlockRequest rreq;
  rreq.block_id = b.block_id;
  rreq.offset = offset;
  rreq.length = length;
  const std::string wire = rreq.str();
  auto fetch = [this, wire, rid, want = rreq.length](const std::string& loc, std::string* data) {
    GrpcResult r = pool_.call(loc, "/dfs.ChunkServerService/ReadBlock", wire, rid);
    if (!r.transport_ok || r.status != 0) return false;  // corrupt / missing / down
    pb::ReadBlockResponse resp;
    if (!resp.decode(r.message) || resp.data.size() != want) return false;
    *data = std::move(resp.data);
    return true;
  };
  size_t next = 0;
  const int hedge = hedge_ms_.load();
  if (hedge > 0 && b.locations.size() >= 2) {
    // Hedged read (reference mod.rs:948-1107): the primary, and after `hedge` ms without an
    // answer the second replica as well; the first clean answer wins, a late one is dropped.
    struct Race {
      std::mutex mu;
      std::condition_variable cv;
      int finished = 0;
      bool won = false;
      std::string data;
    };
    auto race = std::make_shared<Race>();
    auto launch = [&](const std::string& loc) {
      hedge_pool_.submit([race, fetch, loc] {
        std::string d;
        bool ok = fetch(loc, &d);
        std::lock_guard<std::mutex> g(race->mu);
        race->finished++;
        if (ok && !race->won) {
          race->won = true;
          race->data = std::move(d);
        }
        race->cv.notify_all();
      });
    };
    launch(b.locations[0]);
    int launched = 1;
    std::unique_lock<std::mutex> lk(race->mu);
    if (!race->cv.wait_for(lk, std::chrono::milliseconds(hedge), [&] { return race->won || race->finished == 1; }) ||
        !race->won) {
      lk.unlock();
      launch(b.locations[1]);
      launched = 2;
      hedged_++;
      lk.lock();
    }
    race->cv.wait(lk, [&] { return race->won || race->finished == launched; });
    if (race->won) {
      *out = std::move(race->data);
      t->read = since(clk);
      reads_++;
      return FastClient::Ok;
    }
    next = 2;  // both raced replicas failed: the rest in order
  }
  for (size_t i = next; i < b.locations.size(); ++i) {
    if (!fetch(b.locations[i], out)) continue;  // next replica
    t->read = since(clk);
    reads_++;
    return FastClient::Ok;
  }
  return FastClient::NotHandled;  // no replica answered cleanly: the Python path recovers / reports
}


FastClient::Status RemoteClient::stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg,
                                      const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  pb::GetFileInfoRequest req;
  req.path = path;
  int code;
  std::string raw;
  if (!master_call(path, "GetFileInfo", req.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code == kNotFound) {
    *found = false;
    return FastClient::Ok;
  }
  if (code != 0) {
    *msg = raw;
    return FastClient::NotHandled;
  }
  pb::GetFileInfoResponse info;
  if (!info.decode(raw)) return FastClient::NotHandled;
  *found = info.found;
  if (info.found) *meta_pb = info.metadata.str();
  return FastClient::Ok;
}

FastClient::Status RemoteClient::remove(const std::string& path, std::string* msg, const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  pb::DeleteFileRequest req;
  req.path = path;
  int code;
  std::string raw;
  if (!master_call(path, "DeleteFile", req.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code != 0) {
    *msg = raw;
    return code == kNotFound ? FastClient::Failed : FastClient::NotHandled;
  }
  pb::DeleteFileResponse r;
  if (!r.decode(raw)) return FastClient::NotHandled;
  if (!r.success) {
    if (r.error_message == "Not Leader") return FastClient::NotHandled;
    *msg = r.error_message;
    return FastClient::Failed;
  }
  return FastClient::Ok;
}

FastClient::Status RemoteClient::rename(const std::string& src, const std::string& dst, std::string* msg,
                                        const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  pb::RenameRequest req;
  req.source_path = src;
  req.dest_path = dst;
  int code;
  std::string raw;
  if (!master_call(src, "Rename", req.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code != 0) {
    *msg = raw;
    return FastClient::NotHandled;
  }
  pb::RenameResponse r;
  if (!r.decode(raw)) return FastClient::NotHandled;
  if (!r.success) {
    if (r.error_message == "Not Leader") return FastClient::NotHandled;
    *msg = r.error_message;
    return FastClient::Failed;
  }
  return FastClient::Ok;
}

FastClient::Status RemoteClient::list(const std::string& prefix,
                                      std::vector<std::pair<std::string, pb::FileMetadata>>* out,
                                      const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  RequestScope rs(rid);
  std::vector<std::pair<std::string, std::vector<std::string>>> shards;  // shard -> candidates
  {
    std::lock_guard<std::mutex> g(route_mu_);
    if (have_map_) {
      for (const auto& shard : map_.shards()) {
        const auto* peers = map_.peers(shard);
        if (!peers || peers->empty()) return FastClient::NotHandled;
        std::vector<std::string> c = *peers;
        auto it = leader_.find(shard);
        if (it != leader_.end()) {
          auto pos = std::find(c.begin(), c.end(), it->second);
          if (pos != c.end()) std::rotate(c.begin(), pos, pos + 1);
        }
        shards.emplace_back(shard, std::move(c));
      }
    } else if (!masters_.empty()) {
      std::vector<std::string> c = masters_;
      auto it = leader_.find("");
      if (it != leader_.end()) {
        auto pos = std::find(c.begin(), c.end(), it->second);
        if (pos != c.end()) std::rotate(c.begin(), pos, pos + 1);
      }
      shards.emplace_back("", std::move(c));
    }
  }
  if (shards.empty()) return FastClient::NotHandled;
  pb::ListFilesRequest req;
  req.path = prefix;
  req.with_metadata = true;
  const std::string body = req.str();
  out->clear();
  for (auto& sh : shards) {
    int code = 0;
    std::string raw;
    if (!call_candidates(sh.second, sh.first, "ListFiles", body, rid, &code, &raw) || code != 0)
      return FastClient::NotHandled;
    pb::ListFilesResponse resp;
    if (!resp.decode(raw) || resp.metadata.size() != resp.files.size()) return FastClient::NotHandled;
    for (size_t i = 0; i < resp.files.size(); ++i) out->emplace_back(resp.files[i], std::move(resp.metadata[i]));
  }
  std::sort(out->begin(), out->end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  return FastClient::Ok;
}

FastClient::Status RemoteClient::write_ec(const std::string& path, const uint8_t* data, size_t n, int k, int m,
                                          std::string* msg, const std::string& rid_in) {
  const std::string rid = rid_in.empty() ? request_id() : rid_in;
  RequestScope rs(rid);
  TraceRange tr("dfs.remote.write_ec");
  if (k <= 0 || m <= 0 || k + m > 32 || n == 0) return FastClient::NotHandled;
  pb::CreateFileRequest creq;
  creq.path = path;
  creq.ec_data_shards = k;
  creq.ec_parity_shards = m;
  creq.allocate_block = true;
  creq.defer_create = true;
  int code;
  std::string raw;
  if (!master_call(path, "CreateFile", creq.str(), rid, &code, &raw)) return FastClient::NotHandled;
  if (code == kOutOfRange || code == kFailedPrecondition || code == 14) return FastClient::NotHandled;
  if (code != 0) {
    *msg = "Failed to create file: " + raw;
    return FastClient::Failed;
  }
  pb::CreateFileResponse cresp;
  if (!cresp.decode(raw)) return FastClient::NotHandled;
  if (!cresp.success) {
    if (cresp.error_message == "Not Leader") return FastClient::NotHandled;
    *msg = "Failed to create file: " + cresp.error_message;
    return FastClient::Failed;
  }
  if (!cresp.has_allocation || !cresp.allocation.has_block || !cresp.deferred) return FastClient::NotHandled;
  const pb::AllocateBlockResponse& alloc = cresp.allocation;
  if (alloc.ec_data_shards != k || alloc.ec_parity_shards != m ||
      alloc.chunk_server_addresses.size() != static_cast<size_t>(k + m)) {
    *msg = "Expected " + std::to_string(k + m) + " chunk servers for EC(" + std::to_string(k) + "," +
           std::to_string(m) + "), got " + std::to_string(alloc.chunk_server_addresses.size());
    return FastClient::Failed;
  }
  const uint64_t sl = (n + k - 1) / k;
  std::vector<std::string> shards(k + m, std::string(sl, '\0'));
  for (int c = 0; c < k; ++c) {
    const uint64_t off = c * sl;
    if (off < n) std::memcpy(&shards[c][0], data + off, std::min<uint64_t>(sl, n - off));
  }
  gf::Matrix full = gf::rs_matrix(k, m), parity(full.begin() + k, full.end());
  std::vector<const uint8_t*> in(k);
  std::vector<uint8_t*> outp(m);
  for (int c = 0; c < k; ++c) in[c] = reinterpret_cast<const uint8_t*>(shards[c].data());
  for (int r = 0; r < m; ++r) outp[r] = reinterpret_cast<uint8_t*>(&shards[k + r][0]);
  gf::matmul_cpu(parity, in.data(), outp.data(), sl);
  std::vector<std::future<std::pair<int, std::string>>> futs;
  for (int i = 0; i < k + m; ++i)
    futs.push_back(hedge_pool_.submit([this, i, &shards, &alloc, rid]() -> std::pair<int, std::string> {
      pb::WriteBlockRequest req;
      req.block_id = alloc.block.block_id;
      const auto* sp = reinterpret_cast<const uint8_t*>(shards[i].data());
      req.expected_checksum_crc32c = crc32(sp, shards[i].size());
      req.shard_index = i;
      req.master_term = alloc.master_term;
      GrpcResult r = pool_.call(alloc.chunk_server_addresses[i], "/dfs.ChunkServerService/WriteBlock",
                                encode_with_payload(req, sp, shards[i].size()), rid);
      if (!r.transport_ok) return {1, r.message};
      pb::WriteBlockResponse resp;
      if (r.status != 0 || !resp.decode(r.message) || !resp.success)
        return {2, "Shard " + std::to_string(i) + " write failed: " + (r.status ? r.message : resp.error_message)};
      return {0, ""};
    }));
  int worst = 0;
  std::string why;
  for (auto& f : futs) {
    auto r = f.get();
    if (r.first > worst) {
      worst = r.first;
      why = r.second;
    }
  }
  if (worst == 1) return FastClient::NotHandled;
  if (worst == 2) {
    *msg = why;
    return FastClient::Failed;
  }
  pb::CompleteFileRequest done;
  done.path = path;
  done.size = n;
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
  if (!master_call(path, "CompleteFile", done.str(), rid, &code, &raw) || code != 0) {
    *msg = "Failed to complete file: " + (code > 0 ? raw : std::string("master unreachable"));
    return FastClient::Failed;
  }
  pb::CompleteFileResponse dresp;
  dresp.decode(raw);
  if (!dresp.success) {
    *msg = dresp.error_message.empty() ? "Failed to complete file" : "Failed to create file: " + dresp.error_message;
    return FastClient::Failed;
  }
  writes_++;
  return FastClient::Ok;
}

FastClient::Status RemoteClient::read_ec(const pb::FileMetadata& m, std::string* out, std::string* msg,
                                         const std::string& rid, uint64_t offset, uint64_t length) {
  const pb::BlockInfo& b = m.blocks[0];
  const int k = b.ec_data_shards, mm = b.ec_parity_shards;
  const uint64_t orig = b.original_size ? b.original_size : m.size;
  if (k <= 0 || mm <= 0 || b.locations.size() != static_cast<size_t>(k + mm) || orig == 0) return FastClient::NotHandled;
  if (length > 0 && offset >= orig) return FastClient::NotHandled;
  const uint64_t sl = (orig + k - 1) / k;
  std::vector<std::string> shards(k + mm);
  std::vector<std::future<bool>> futs;
  pb::ReadBlockRequest req;
  req.block_id = b.block_id;
  const std::string wire = req.str();
  for (int i = 0; i < k + mm; ++i)
    futs.push_back(hedge_pool_.submit([this, i, &b, &shards, wire, rid, sl]() -> bool {
      if (b.locations[i].empty()) return false;
      GrpcResult r = pool_.call(b.locations[i], "/dfs.ChunkServerService/ReadBlock", wire, rid);
      pb::ReadBlockResponse resp;
      if (!r.transport_ok || r.status != 0 || !resp.decode(r.message) || resp.data.size() != sl) return false;
      shards[i] = std::move(resp.data);
      return true;
    }));
  std::vector<int> present, missing;
  for (int i = 0; i < k + mm; ++i)
    if (futs[i].get()) present.push_back(i);
    else if (i < k) missing.push_back(i);
  if (!missing.empty()) {
    if (static_cast<int>(present.size()) < k) {
      *msg = "RS reconstruct error: TooFewShardsPresent";
      return FastClient::Failed;
    }
    std::vector<int> use(present.begin(), present.begin() + k);
    gf::Matrix rows = gf::rs_decode_rows(k, mm, use, missing);
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> outp(missing.size());
    for (int c = 0; c < k; ++c) in[c] = reinterpret_cast<const uint8_t*>(shards[use[c]].data());
    for (size_t r = 0; r < missing.size(); ++r) {
      shards[missing[r]].assign(sl, '\0');
      outp[r] = reinterpret_cast<uint8_t*>(&shards[missing[r]][0]);
    }
    gf::matmul_cpu(rows, in.data(), outp.data(), sl);
    ec_degraded_++;
  }
  const uint64_t from = length > 0 ? offset : 0, want = length > 0 ? std::min<uint64_t>(length, orig - offset) : orig;
  out->clear();
  out->reserve(want);
  for (uint64_t pos = from; pos < from + want;) {
    const uint64_t c = pos / sl, o = pos % sl, take = std::min<uint64_t>(sl - o, from + want - pos);
    out->append(shards[c], o, take);
    pos += take;
  }
  reads_++;
  return FastClient::Ok;
}

}  // namespace dfs
