// Native ChunkServer control loop; design notes in cs_agent.h.
#include "cs_agent.h"
#include "thread_name.h"

#include <sys/statvfs.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <future>
#include <random>
#include <cstring>
#include <set>

#include "client_fast.h"
#include "crc32.h"
#include "gf256.h"
#include "trace.h"

namespace dfs {

namespace {

std::string rid() {
  thread_local std::mt19937_64 rng{std::random_device{}()};
  char b[33];
  std::snprintf(b, sizeof b, "%016llx%016llx", static_cast<unsigned long long>(rng()),
                static_cast<unsigned long long>(rng()));
  return b;
}

std::string strip_scheme(const std::string& a) {
  auto p = a.find("://");
  std::string s = p == std::string::npos ? a : a.substr(p + 3);
  while (!s.empty() && s.back() == '/') s.pop_back();
  return s;
}

}  // namespace

CsAgent::CsAgent(CsAgentConfig cfg, ChunkStore* store, FastPathServer* fp, std::shared_ptr<TlsContext> tls)
    : cfg_(std::move(cfg)), store_(store), fp_(fp), pool_(cfg_.rpc_timeout_ms, std::move(tls)) {
  masters_ = cfg_.masters;
}

CsAgent::~CsAgent() { stop(); }

void CsAgent::start() {
  hb_ = std::thread([this] {
    name_thread("cs-heartbeat");
    heartbeat_loop();
  });
  scrub_ = std::thread([this] {
    name_thread("cs-scrub");
    scrub_loop();
  });
}

void CsAgent::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (hb_.joinable()) hb_.join();
  if (scrub_.joinable()) scrub_.join();
}

std::string CsAgent::target(const std::string& addr) const {
  return (cfg_.tls ? "https://" : "http://") + strip_scheme(addr);
}

bool CsAgent::is_me(const std::string& addr) const { return strip_scheme(addr) == strip_scheme(cfg_.advertise); }

void CsAgent::adopt(uint64_t term) {
  if (fp_) {
    fp_->adopt_term(term);
    return;
  }
  uint64_t cur = term_.load();
  while (term > cur && !term_.compare_exchange_weak(cur, term)) {
  }
}

uint64_t CsAgent::known_term() { return fp_ ? fp_->term() : term_.load(); }

std::vector<std::string> CsAgent::masters() {
  std::lock_guard<std::mutex> g(mu_);
  return masters_;
}

CsAgentStats CsAgent::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

void CsAgent::report_new_block(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  new_.push_back(id);
}

void CsAgent::report_bad_block(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  if (std::find(bad_.begin(), bad_.end(), id) == bad_.end()) bad_.push_back(id);
}

// ---------------------------------------------------------------- heartbeat
bool CsAgent::refresh_masters() {
  for (const auto& c : cfg_.config_servers) {
    GrpcResult r = pool_.call(target(c), "/dfs.ConfigService/FetchShardMap", pb::FetchShardMapRequest{}.str(), rid(),
                              5000);
    pb::FetchShardMapResponse resp;
    if (!r.transport_ok || r.status != 0 || !resp.decode(r.message)) continue;
    std::set<std::string> all;
    for (const auto& kv : resp.shards)
      for (const auto& p : kv.second.peers) all.insert(p);
    std::lock_guard<std::mutex> g(mu_);
    if (!all.empty()) masters_.assign(all.begin(), all.end());
    else masters_ = cfg_.masters;
    st_.map_refreshes++;
    return true;
  }
  return false;
}

void CsAgent::heartbeat_once() {
  TraceRange tr("dfs.cs.heartbeat");
  if (!cfg_.config_servers.empty()) refresh_masters();
  if (fp_)
    for (const auto& id : fp_->drain_suspects()) queue_recovery(id);  // partial-read corruption seen natively
  pb::HeartbeatRequest req;
  req.chunk_server_address = cfg_.advertise;
  struct statvfs vs{};
  if (::statvfs(cfg_.storage_dir.c_str(), &vs) == 0) {
    const uint64_t total = static_cast<uint64_t>(vs.f_blocks) * vs.f_frsize;
    req.available_space = static_cast<uint64_t>(vs.f_bavail) * vs.f_frsize;
    req.used_space = total > req.available_space ? total - req.available_space : 0;
  }
  StoreStats ss = store_->stats();
  req.chunk_count = ss.blocks;
  req.rack_id = cfg_.rack_id;
  req.gpu_rank = cfg_.gpu_rank;
  req.hbm_capacity = ss.hbm_capacity;
  req.hbm_used = ss.hbm_used;
  std::vector<std::string> ms;
  {
    std::lock_guard<std::mutex> g(mu_);
    req.bad_blocks.swap(bad_);
    req.new_blocks.swap(new_);
    req.ec_encoded.swap(enc_);
    req.ec_failed.swap(fail_);
    req.ec_rebuilt.swap(rebuilt_);
    ms = masters_;
  }
  if (fp_)
    for (auto& id : fp_->drain_healed()) req.new_blocks.push_back(std::move(id));
  const std::string wire = req.str();
  bool any = false;
  for (const auto& m : ms) {
    GrpcResult r = pool_.call(target(m), "/dfs.MasterService/Heartbeat", wire, rid(), 5000);
    pb::HeartbeatResponse resp;
    if (!r.transport_ok || r.status != 0 || !resp.decode(r.message)) continue;
    any = true;
    adopt(resp.master_term);
    for (const auto& c : resp.commands) {
      {
        std::lock_guard<std::mutex> g(mu_);
        st_.commands++;
      }
      dispatch(c);
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  if (any) {
    st_.heartbeats++;
  } else {
    st_.heartbeat_failures++;
    // nobody heard the reports: keep them for the next round (the reference re-sends its
    // bad-block list every heartbeat too)
    bad_.insert(bad_.end(), req.bad_blocks.begin(), req.bad_blocks.end());
    new_.insert(new_.end(), req.new_blocks.begin(), req.new_blocks.end());
    enc_.insert(enc_.end(), req.ec_encoded.begin(), req.ec_encoded.end());
    fail_.insert(fail_.end(), req.ec_failed.begin(), req.ec_failed.end());
    rebuilt_.insert(rebuilt_.end(), req.ec_rebuilt.begin(), req.ec_rebuilt.end());
  }
}

void CsAgent::heartbeat_loop() {
  // the first round waits for a shard map when config servers are configured
  while (!cfg_.config_servers.empty() && !refresh_masters()) {
    std::unique_lock<std::mutex> lk(mu_);
    if (cv_.wait_for(lk, std::chrono::seconds(2), [this] { return stop_; })) return;
  }
  for (;;) {
    heartbeat_once();
    std::unique_lock<std::mutex> lk(mu_);
    if (cv_.wait_for(lk, std::chrono::milliseconds(cfg_.heartbeat_ms), [this] { return stop_; })) return;
  }
}

void CsAgent::scrub_loop() {
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (cv_.wait_for(lk, std::chrono::milliseconds(cfg_.scrub_ms), [this] { return stop_; })) return;
    }
    scrub_once();
  }
}

std::vector<std::string> CsAgent::scrub_once() {
  TraceRange tr("dfs.cs.scrub");
  std::vector<std::string> bad = store_->scrub();
  {
    std::lock_guard<std::mutex> g(mu_);
    st_.scrubs++;
    st_.scrub_bad += bad.size();
  }
  for (const auto& b : bad) {
    report_bad_block(b);
    queue_recovery(b);
  }
  return bad;
}

// ---------------------------------------------------------------- commands
void CsAgent::submit_command(const std::string& cmd_pb) {
  pb::ChunkServerCommand c;
  if (c.decode(cmd_pb)) dispatch(c);
}

void CsAgent::dispatch(const pb::ChunkServerCommand& c) {
  if (c.master_term) adopt(c.master_term);
  using T = pb::ChunkServerCommand;
  constexpr int kReplicate = T::REPLICATE, kDelete = T::DELETE, kReconstruct = T::RECONSTRUCT_EC_SHARD,
                kMoveToCold = T::MOVE_TO_COLD, kEncodeEc = T::ENCODE_EC;
  const int type = c.type;
  if (type == kDelete) {
    // queued, and removed by a bounded set of drain jobs: concurrent removes still share
    // the journal's group-committed tombstone flushes
    std::lock_guard<std::mutex> g(mu_);
    del_q_.push_back(c.block_id);
    if (del_workers_ < kDeleteWorkers) {
      del_workers_++;
      jobs_.submit([this] {
        RequestScope rs(rid());
        for (;;) {
          std::string id;
          {
            std::lock_guard<std::mutex> g2(mu_);
            if (del_q_.empty()) {
              del_workers_--;
              return;
            }
            id = std::move(del_q_.front());
            del_q_.pop_front();
          }
          store_->remove(id);
          std::lock_guard<std::mutex> g2(mu_);
          st_.deletes++;
        }
      });
    }
    return;
  }
  jobs_.submit([this, c, type] {
    RequestScope rs(rid());
    if (type == kReplicate) {
      replicate_to(c.block_id, c.target_chunk_server_address);
    } else if (type == kMoveToCold) {
      store_->move_to_cold(c.block_id);
      std::lock_guard<std::mutex> g(mu_);
      st_.moves++;
    } else if (type == kReconstruct) {
      bool ok = reconstruct(c);
      std::lock_guard<std::mutex> g(mu_);
      (ok ? st_.reconstructs : st_.reconstruct_failed)++;
      if (ok) rebuilt_.push_back(c.block_id + "/" + std::to_string(c.shard_index));
    } else if (type == kEncodeEc) {
      bool ok = encode_ec(c);
      std::lock_guard<std::mutex> g(mu_);
      (ok ? st_.encodes : st_.encode_failed)++;
      (ok ? enc_ : fail_).push_back(c.block_id);
    }
  });
}

bool CsAgent::read_local(const std::string& id, std::vector<uint8_t>* out) {
  const int64_t n = store_->block_size(id);
  if (n < 0) return false;
  out->resize(static_cast<size_t>(n));
  ReadResult r = store_->read_into(id, 0, static_cast<uint64_t>(n), out->data());
  return r.status == ReadStatus::Ok && r.bytes == static_cast<uint64_t>(n);
}

bool CsAgent::replicate_to(const std::string& block_id, const std::string& tgt) {
  TraceRange tr("dfs.cs.replicate");
  if (!store_->exists(block_id)) {
    std::lock_guard<std::mutex> g(mu_);
    st_.replicate_failed++;
    return false;
  }
  // same-node target with a P2P pair: HBM -> HBM on the replication engine, receipt
  // reported by the receiver (reference chunkserver.rs:462-499 forwards over gRPC)
  if (fp_) {
    std::vector<std::string> done;
    if (fp_->replicate_block(block_id, {strip_scheme(tgt)}, known_term(), &done) > 0) {
      std::lock_guard<std::mutex> g(mu_);
      st_.replicate_engine++;
      return true;
    }
  }
  std::vector<uint8_t> data;
  bool ok = read_local(block_id, &data);
  if (ok) {
    pb::ReplicateBlockRequest q;
    q.block_id = block_id;
    q.data.assign(reinterpret_cast<const char*>(data.data()), data.size());
    q.expected_checksum_crc32c = crc32(data.data(), data.size());
    q.master_term = known_term();
    q.heal = true;
    GrpcResult r = pool_.call(target(tgt), "/dfs.ChunkServerService/ReplicateBlock", q.str(), rid());
    pb::ReplicateBlockResponse resp;
    ok = r.transport_ok && r.status == 0 && resp.decode(r.message) && resp.success;
  }
  std::lock_guard<std::mutex> g(mu_);
  (ok ? st_.replicate_grpc : st_.replicate_failed)++;
  return ok;
}

bool CsAgent::gf_product(const std::vector<std::vector<uint8_t>>& mat, const std::vector<const uint8_t*>& in,
                         const std::vector<uint8_t*>& out, uint64_t len) {
  if (store_->gpu() && store_->gf_matmul_gpu(mat, in, out, len)) {
    std::lock_guard<std::mutex> g(mu_);
    st_.ec_gpu++;
    return true;
  }
  gf::matmul_cpu(mat, in.data(), out.data(), len);
  std::lock_guard<std::mutex> g(mu_);
  st_.ec_cpu++;
  return true;
}

// RECONSTRUCT_EC_SHARD (reference chunkserver.rs:503-640): gather >= k survivors in
// parallel, rebuild shard `shard_index` with the decode rows of the first k present.
bool CsAgent::reconstruct(const pb::ChunkServerCommand& c) {
  TraceRange tr("dfs.cs.reconstruct");
  const int k = c.ec_data_shards, m = c.ec_parity_shards;
  if (k <= 0 || m <= 0 || static_cast<int>(c.ec_shard_sources.size()) != k + m || c.shard_index < 0 ||
      c.shard_index >= k + m)
    return false;
  // Device path: gather k survivors into this GPU over the replication engine (our own
  // shards pinned in place, peers' pushed HBM -> HBM), decode the target shard there and
  // commit it from HBM; shards on other hosts (or a host store) take the gRPC gather below.
  if (fp_ != nullptr && store_->gpu()) {
    FastPathServer::EcGather g;
    std::string err;
    if (fp_->ec_gather(c.block_id, c.ec_shard_sources, 0, c.shard_index, k, &g, &err)) {
      std::vector<int> present;
      for (int i = 0; i < k + m; ++i)
        if (g.ptrs[i] && i != c.shard_index) present.push_back(i);
      if (static_cast<int>(present.size()) >= k) {
        present.resize(k);
        std::vector<const uint8_t*> in;
        for (int i : present) in.push_back(g.ptrs[i]);
        gf::Matrix rows = gf::rs_decode_rows(k, m, present, {c.shard_index});
        ChunkStore::EcBuffers dec;
        if (store_->ec_decode(rows, in, g.len, &dec, &err)) {
          WriteResult w = store_->commit_copy(c.block_id, dec.shard(0), g.len, dec.crc[0], true);
          store_->ec_free(&dec);
          std::lock_guard<std::mutex> lk(mu_);
          st_.ec_gpu++;
          st_.reconstruct_device++;
          return w.ok;
        }
      }
    }
  }
  std::vector<std::string> shards(k + m);
  std::vector<bool> have(k + m, false);
  std::vector<std::future<bool>> futs(k + m);
  for (int i = 0; i < k + m; ++i) {
    const std::string& a = c.ec_shard_sources[i];
    if (a.empty() || i == c.shard_index) continue;
    futs[i] = jobs_.submit([this, a, i, &shards, &c] {
      pb::ReadBlockRequest q;
      q.block_id = c.block_id;
      GrpcResult r = pool_.call(target(a), "/dfs.ChunkServerService/ReadBlock", q.str(), rid());
      pb::ReadBlockResponse resp;
      if (!r.transport_ok || r.status != 0 || !resp.decode(r.message)) return false;
      shards[i] = std::move(resp.data);
      return true;
    });
  }
  std::vector<int> present;
  for (int i = 0; i < k + m; ++i)
    if (futs[i].valid() && futs[i].get()) {
      have[i] = true;
      present.push_back(i);
    }
  if (static_cast<int>(present.size()) < k) return false;
  present.resize(k);
  const uint64_t sl = shards[present[0]].size();
  for (int i : present)
    if (shards[i].size() != sl) return false;
  gf::Matrix rows = gf::rs_decode_rows(k, m, present, {c.shard_index});
  std::vector<const uint8_t*> in;
  for (int i : present) in.push_back(reinterpret_cast<const uint8_t*>(shards[i].data()));
  std::vector<uint8_t> out(sl);
  std::vector<uint8_t*> outp{out.data()};
  gf_product(rows, in, outp, sl);
  WriteResult w = store_->write(c.block_id, out.data(), sl, 0);
  return w.ok;
}

// ENCODE_EC (tiering's EC conversion, C32): RS(k, m) of the verified local replica; shard i
// is written as block `new_block_id` to ec_shard_sources[i] (locally when that is us).
bool CsAgent::encode_ec(const pb::ChunkServerCommand& c) {
  TraceRange tr("dfs.cs.encode_ec");
  const int k = c.ec_data_shards, m = c.ec_parity_shards;
  if (k <= 0 || m <= 0 || static_cast<int>(c.ec_shard_sources.size()) != k + m || c.new_block_id.empty())
    return false;
  std::vector<uint8_t> data;
  if (!read_local(c.block_id, &data) || data.empty()) return false;
  const uint64_t sl = (data.size() + k - 1) / k;
  std::vector<std::vector<uint8_t>> shards(k + m, std::vector<uint8_t>(sl, 0));
  for (int i = 0; i < k; ++i) {
    const uint64_t off = static_cast<uint64_t>(i) * sl;
    if (off < data.size()) std::memcpy(shards[i].data(), data.data() + off, std::min<uint64_t>(sl, data.size() - off));
  }
  gf::Matrix full = gf::rs_matrix(k, m), parity(full.begin() + k, full.end());
  std::vector<const uint8_t*> in;
  std::vector<uint8_t*> out;
  for (int i = 0; i < k; ++i) in.push_back(shards[i].data());
  for (int r = 0; r < m; ++r) out.push_back(shards[k + r].data());
  gf_product(parity, in, out, sl);
  std::vector<std::future<bool>> futs;
  for (int i = 0; i < k + m; ++i)
    futs.push_back(jobs_.submit([this, i, &shards, &c] {
      const uint32_t crc = crc32(shards[i].data(), shards[i].size());
      if (is_me(c.ec_shard_sources[i])) return store_->write(c.new_block_id, shards[i].data(), shards[i].size(), crc).ok;
      pb::WriteBlockRequest q;
      q.block_id = c.new_block_id;
      q.expected_checksum_crc32c = crc;
      q.shard_index = i;
      q.master_term = c.master_term;
      GrpcResult r = pool_.call(target(c.ec_shard_sources[i]), "/dfs.ChunkServerService/WriteBlock",
                                encode_with_payload(q, shards[i].data(), shards[i].size()), rid());
      pb::WriteBlockResponse resp;
      return r.transport_ok && r.status == 0 && resp.decode(r.message) && resp.success;
    }));
  bool ok = true;
  for (auto& f : futs) ok = f.get() && ok;
  return ok;
}

// ---------------------------------------------------------------- recovery
std::vector<std::string> CsAgent::block_locations(const std::string& block_id) {
  pb::GetBlockLocationsRequest q;
  q.block_id = block_id;
  const std::string wire = q.str();
  for (const auto& m : masters()) {
    GrpcResult r = pool_.call(target(m), "/dfs.MasterService/GetBlockLocations", wire, rid(), 5000);
    pb::GetBlockLocationsResponse resp;
    if (r.transport_ok && r.status == 0 && resp.decode(r.message) && resp.found) return resp.locations;
  }
  return {};
}

// Reference recover_block (chunkserver.rs:353-460): fetch a healthy replica, check it against
// our own .meta, rewrite it locally (the self-skip uses the advertised address).
std::string CsAgent::recover(const std::string& block_id) {
  TraceRange tr("dfs.cs.recover");
  std::vector<std::string> locs = block_locations(block_id);
  std::string why = locs.empty() ? "No replica locations found for block" : "Failed to recover block from any replica";
  const std::vector<uint32_t> local = store_->meta(block_id);
  for (const auto& loc : locs) {
    if (is_me(loc)) continue;
    pb::ReadBlockRequest q;
    q.block_id = block_id;
    GrpcResult r = pool_.call(target(loc), "/dfs.ChunkServerService/ReadBlock", q.str(), rid());
    pb::ReadBlockResponse resp;
    if (!r.transport_ok || r.status != 0 || !resp.decode(r.message)) continue;
    const auto* p = reinterpret_cast<const uint8_t*>(resp.data.data());
    if (!local.empty()) {
      std::vector<uint32_t> got(num_slices(resp.data.size()));
      crc32_slices(p, resp.data.size(), got.data());
      if (got != local) continue;  // that replica is corrupt too
    }
    if (store_->write(block_id, p, resp.data.size(), 0).ok) {
      std::lock_guard<std::mutex> g(mu_);
      st_.recoveries++;
      return "";
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  st_.recovery_failed++;
  return why;
}

void CsAgent::queue_recovery(const std::string& block_id) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (std::find(recovering_.begin(), recovering_.end(), block_id) != recovering_.end()) return;
    recovering_.push_back(block_id);
  }
  jobs_.submit([this, block_id] {
    RequestScope rs(rid());
    recover(block_id);
    std::lock_guard<std::mutex> g(mu_);
    recovering_.erase(std::find(recovering_.begin(), recovering_.end(), block_id));
  });
}

}  // namespace dfs
