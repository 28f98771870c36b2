// dfs_master — the native metadata-master process (C35; reference
// dfs/metaserver/src/bin/master.rs:97-255 and the background tasks of master.rs:729-2138).
//
// One Raft member of a metadata shard. MasterCore (master_core.cpp) holds the replicated
// namespace and answers the hot MasterService RPCs and the 2PC coordinator/participant
// RPCs; this executable owns everything around it, so no interpreter lives in a master
// process:
//
//   * the native Raft node with a native host (peer RPCs over the peers' HTTP/2 endpoints,
//     HTTP/JSON to peers without one), snapshots backed up with a PUT when configured;
//   * MasterService over native HTTP/2 gRPC and the same-host socket: MasterCore's methods,
//     plus the cold ones here — AddRaftServer / RemoveRaftServer / GetClusterInfo
//     (membership, master.rs:3424-3533), IngestMetadata / InitiateShuffle (:3535-3660), and a
//     Rename that MasterCore declined (stale shard map: refreshed here, then retried);
//   * the HTTP side channel: /health, /metrics, /raft/state, /raft/endpoint, /shard_map,
//     POST /raft/{vote,append,snapshot,timeout_now}, /debug/partition (DFS_DEBUG_ENDPOINTS=1);
//   * the background tasks, one thread each: liveness (chunkserver eviction + heal),
//     heartbeat reports, the healer, balancer, data shuffler, 2PC cleanup and recovery,
//     metrics decay, shard-map refresh, split/merge detector, tiering + EC conversion.
//
// Flags and environment knobs are those of master/server.py (the reference's spelling), so
// the launcher, helm chart and tests start either process with the same command line.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <fstream>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "dfs_pb.h"
#include "grpc_client.h"
#include "grpc_server.h"
#include "json.h"
#include "localrpc.h"
#include "master_core.h"
#include "node_shell.h"
#include "raft.h"
#include "shard_map.h"
#include "tls.h"
#include "trace.h"

using namespace dfs;
using namespace dfs::shell;

namespace {

constexpr const char* kLog = "dfs.master";
constexpr uint64_t kBalanceGap = 100ull << 20;
constexpr int64_t kEcJobTimeoutMs = 120000;
constexpr int kMaxInquiryRetries = 60;
constexpr int64_t kTxStaleMs = 3600000;
enum Status { OK = 0, INVALID_ARGUMENT = 3, FAILED_PRECONDITION = 9, OUT_OF_RANGE = 11, UNIMPLEMENTED = 12,
              INTERNAL = 13, UNAVAILABLE = 14 };

struct Intervals {
  double liveness = 5, healer_first = 60, healer = 300, balancer = 30, tx_cleanup = 5, tx_recovery = 30,
         shuffler = 10, decay = 5, shard_refresh = 1, split = 5, tiering = 60;
  static Intervals fast() {
    Intervals i;
    i.liveness = 1, i.healer_first = 2, i.healer = 5, i.balancer = 2, i.tx_cleanup = 1, i.tx_recovery = 2,
    i.shuffler = 1, i.decay = 1, i.shard_refresh = 0.5, i.split = 1, i.tiering = 2;
    return i;
  }
};

// Per-prefix request-rate monitor for dynamic sharding (reference master.rs:610-675):
// requests counted by first path component, folded into an EMA (0.3 old, 0.7 new) per window.
class ThroughputMonitor {
 public:
  ThroughputMonitor(double split_rps, double merge_rps, int cooldown_s)
      : split_rps_(split_rps), merge_rps_(merge_rps), cooldown_s_(cooldown_s),
        last_split_(steady_s() - cooldown_s) {}
  void decay(const std::map<std::string, uint64_t>& counts, double window_s) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : counts) m_[kv.first].count += kv.second;
    for (auto& kv : m_) {
      kv.second.rps = kv.second.rps * 0.3 + (static_cast<double>(kv.second.count) / window_s) * 0.7;
      kv.second.count = 0;
    }
  }
  std::map<std::string, double> rps() const {
    std::lock_guard<std::mutex> g(mu_);
    std::map<std::string, double> out;
    for (auto& kv : m_) out[kv.first] = kv.second.rps;
    return out;
  }
  bool hot(std::string* prefix, double* rps) const {
    if (steady_s() - last_split_.load() < cooldown_s_) return false;
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : m_)
      if (kv.second.rps > split_rps_) {
        *prefix = kv.first;
        *rps = kv.second.rps;
        return true;
      }
    return false;
  }
  double total() const {
    std::lock_guard<std::mutex> g(mu_);
    double t = 0;
    for (auto& kv : m_) t += kv.second.rps;
    return t;
  }
  void mark_split() { last_split_ = steady_s(); }
  double merge_rps() const { return merge_rps_; }
  static double steady_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

 private:
  struct M {
    double rps = 0;
    uint64_t count = 0;
  };
  mutable std::mutex mu_;
  std::map<std::string, M> m_;
  double split_rps_, merge_rps_;
  int cooldown_s_;
  std::atomic<double> last_split_;
};

// Range map from the shard config file / a FetchShardMap reply: sorted ids added to a Range
// map, optionally with explicit boundaries (parallel/sharding.py ShardMap.from_config).
ShardMap map_from_config(const std::map<std::string, std::vector<std::string>>& shards,
                         const std::map<std::string, std::string>& ranges) {
  ShardMap m = ShardMap::new_range();
  for (auto& kv : shards) m.add_shard(kv.first, kv.second);
  if (ranges.empty()) return m;
  Json j = m.to_json();
  Json r = Json::object();
  for (auto& kv : ranges)
    if (shards.count(kv.second)) r.set(kv.first, kv.second);
  j.set("strategy", Json(Json::Object{{"Range", Json(Json::Object{{"ranges", r}})}}));
  return ShardMap::from_json(j);
}

ShardMap load_shard_config(const std::string& path) {
  if (!path.empty()) {
    try {
      std::FILE* f = std::fopen(path.c_str(), "rb");
      if (f) {
        std::string text;
        char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, n);
        std::fclose(f);
        Json cfg = Json::parse(text);
        std::map<std::string, std::vector<std::string>> shards;
        for (auto& kv : cfg["shards"].fields()) {
          auto& v = shards[kv.first];
          for (auto& p : kv.second.items()) v.push_back(p.str());
        }
        std::map<std::string, std::string> ranges;
        if (cfg.has("ranges") && cfg["ranges"].is_object())
          for (auto& kv : cfg["ranges"].fields()) ranges[kv.first] = kv.second.str();
        if (!shards.empty()) return map_from_config(shards, ranges);
      }
    } catch (...) {
    }
  }
  return ShardMap::new_consistent_hash(100);
}

std::string uuid4() {
  static thread_local std::mt19937_64 rng(std::random_device{}());
  uint64_t a = rng(), b = rng();
  a = (a & 0xffffffffffff0fffull) | 0x4000ull;
  b = (b & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  char s[40];
  std::snprintf(s, sizeof(s), "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                static_cast<unsigned>((a >> 16) & 0xffff), static_cast<unsigned>(a & 0xffff),
                static_cast<unsigned>(b >> 48), static_cast<unsigned long long>(b & 0xffffffffffffull));
  return s;
}

class Master {
 public:
  explicit Master(const Args& a) : a_(a) {}
  int run();

 private:
  struct Proposal {
    int code = 2;  // 0 applied (payload = result JSON), 1 not leader (hint), 2 failed
    std::string payload;
  };

  // ---- Raft helpers
  Proposal propose(const Json& cmd, int timeout_ms = 30000) {
    auto pr = std::make_shared<std::promise<Proposal>>();
    auto fut = pr->get_future();
    node_->propose(cmd.dump(), [pr](int code, const std::string& p) {
      try {
        pr->set_value(Proposal{code, p});
      } catch (...) {
      }
    });
    if (fut.wait_for(std::chrono::milliseconds(timeout_ms)) != std::future_status::ready)
      return Proposal{2, "proposal timed out"};
    return fut.get();
  }
  static Json master_cmd(const std::string& name, Json args) {
    return Json(Json::Object{{"Master", Json(Json::Object{{name, std::move(args)}})}});
  }
  bool propose_master(const std::string& name, Json args) { return propose(master_cmd(name, std::move(args))).code == 0; }
  bool is_leader() const { return node_->is_leader(); }

  // ---- routing
  ShardMap map_copy() {
    std::lock_guard<std::mutex> g(map_mu_);
    return map_;
  }
  std::string shard_id() {
    std::lock_guard<std::mutex> g(map_mu_);
    return shard_id_;
  }
  void set_routing(const ShardMap* m, const std::string* sid) {
    std::lock_guard<std::mutex> g(map_mu_);
    if (m) map_ = *m;
    if (sid) shard_id_ = *sid;
    core_->set_shard_map(map_.to_json().dump(), shard_id_);
  }
  std::vector<std::string> peers_of(const ShardMap& m, const std::string& sid) {
    const auto* p = m.peers(sid);
    return p ? *p : std::vector<std::string>{};
  }

  // ---- RPC clients
  GrpcResult call(const std::string& target, const std::string& service, const std::string& method,
                  const std::string& req, int timeout_ms = 5000) {
    return pool_->call(target, "/dfs." + service + "/" + method, req, t_request_id, timeout_ms);
  }
  template <class Resp>
  bool config_call(const std::string& method, const std::string& req, Resp* out) {
    for (auto& c : config_servers_) {
      GrpcResult r = call(c, "ConfigService", method, req);
      if (r.transport_ok && r.status == 0 && out->decode(r.message)) return true;
    }
    return false;
  }
  // Each peer of a shard in turn, following leader hints (service.py _call_peers).
  template <class Resp>
  bool call_peers(const std::vector<std::string>& peers, const std::string& method, const std::string& req) {
    std::set<std::string> tried;
    std::deque<std::string> q(peers.begin(), peers.end());
    while (!q.empty()) {
      std::string addr = q.front();
      q.pop_front();
      if (addr.empty() || tried.count(addr)) continue;
      tried.insert(addr);
      GrpcResult r = call(addr, "MasterService", method, req);
      Resp resp;
      if (!r.transport_ok || r.status != 0 || !resp.decode(r.message)) continue;
      if (resp.success) return true;
      if (!resp.leader_hint.empty() && !tried.count(resp.leader_hint)) q.push_front(resp.leader_hint);
      else if (!resp.error_message.empty() && resp.error_message != "Not Leader") return false;
    }
    return false;
  }

  // ---- cold MasterService RPCs
  int handle(const std::string& path, const std::string& rid, const std::string& payload, std::string* out,
             bool* native);
  int cold(const std::string& method, const std::string& payload, std::string* out);
  int rename_declined(const std::string& payload, std::string* out);

  // ---- background
  void every(double first, double period, const char* name, std::function<void()> fn);
  void liveness_check();
  void heartbeat_reports();
  size_t heal();
  void balance();
  void shuffle();
  std::string inquire(const Json& rec);
  void tx_cleanup();
  void tx_recovery();
  void decay();
  bool refresh_shard_map();
  void do_register();
  void split_detector();
  void split(const std::string& prefix, double rps);
  void merge_into(const std::string& neighbor);
  void tiering();
  void ec_convert(int64_t now);
  void queue(const std::string& addr, const pb::ChunkServerCommand& c) { core_->queue_command(addr, c.str()); }

  HttpResponse http(const HttpRequest& req);

  const Args& a_;
  std::shared_ptr<MasterCore> core_;
  std::shared_ptr<NativeRaftHost> raft_host_;
  std::unique_ptr<raft::Node> node_;
  std::unique_ptr<GrpcChannelPool> pool_;
  std::unique_ptr<GrpcServer> grpc_;
  std::unique_ptr<LocalRpcServer> local_;
  std::unique_ptr<HttpLiteServer> http_;
  std::unique_ptr<ThroughputMonitor> monitor_;
  Intervals iv_;
  std::vector<std::string> config_servers_;
  std::string client_addr_, self_http_;
  int64_t cs_dead_ms_ = 15000, tx_timeout_ms_ = 10000;
  int64_t cold_ms_ = 0, ec_ms_ = 0;
  bool ec_conversion_ = false;
  int ec_k_ = 6, ec_m_ = 3;

  std::mutex map_mu_;
  ShardMap map_ = ShardMap::new_range();
  std::string shard_id_;
  std::atomic<int64_t> map_fetched_ms_{0};
  std::mutex refresh_mu_;
  std::atomic<bool> registered_{false};

  struct EcJob {
    std::string path, new_id;
    std::vector<std::string> targets;
    int k = 0, m = 0;
    int64_t started_ms = 0;
    bool done = false;
  };
  std::mutex ec_mu_;
  std::map<std::string, EcJob> ec_jobs_;

  std::atomic<uint64_t> native_calls_{0}, cold_calls_{0}, raft_calls_{0};
  std::atomic<bool> stop_{false};
  std::mutex stop_mu_;
  std::condition_variable stop_cv_;
  std::vector<std::thread> threads_;
};

// ---------------------------------------------------------------- request routing
int Master::handle(const std::string& path, const std::string& rid, const std::string& payload, std::string* out,
                   bool* native) {
  static const std::string kPrefix = "/dfs.MasterService/";
  RequestScope scope(rid);
  *native = false;
  if (path.compare(0, kPrefix.size(), kPrefix) != 0) return (*out = "unknown service: " + path, UNIMPLEMENTED);
  const std::string method = path.substr(kPrefix.size());
  if (core_->native_method(method)) {
    int code = core_->handle(method, payload, out);
    if (code != MasterCore::kDecline) {
      *native = true;
      return code;
    }
    out->clear();
    if (method == "Rename") return rename_declined(payload, out);
  }
  return cold(method, payload, out);
}

// MasterCore declines a Rename while its shard map is older than the max age (a split or
// merge may have moved the destination) or while its 2PC coordinator slots are all busy:
// refresh the map and retry, waiting out the slots (service.py rename's fresh_shard_map).
int Master::rename_declined(const std::string& payload, std::string* out) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
  for (int attempt = 0;; ++attempt) {
    if (!config_servers_.empty()) refresh_shard_map();
    out->clear();
    int code = core_->handle("Rename", payload, out);
    if (code != MasterCore::kDecline) return code;
    if (std::chrono::steady_clock::now() > deadline) {
      *out = "Rename: shard map stays stale or too many cross-shard renames in flight";
      return UNAVAILABLE;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(std::min(200, 10 << std::min(attempt, 4))));
  }
}

int Master::cold(const std::string& method, const std::string& payload, std::string* out) {
  out->clear();
  if (method == "AddRaftServer") {
    pb::AddRaftServerRequest r;
    if (!r.decode(payload)) return (*out = "malformed AddRaftServerRequest", INVALID_ARGUMENT);
    pb::AddRaftServerResponse resp;
    Proposal p = propose(Json(Json::Object{{"Membership", Json(Json::Object{{"AddServer", Json(Json::Object{
        {"server_id", Json(static_cast<int64_t>(r.server_id))}, {"server_address", Json(r.server_address)}})}})}}));
    if (p.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = p.payload;
    } else if (p.code != 0) {
      return (*out = p.payload, INTERNAL);
    } else {
      resp.success = true;
    }
    resp.encode(*out);
    return OK;
  }
  if (method == "RemoveRaftServer") {
    pb::RemoveRaftServerRequest r;
    if (!r.decode(payload)) return (*out = "malformed RemoveRaftServerRequest", INVALID_ARGUMENT);
    pb::RemoveRaftServerResponse resp;
    if (!is_leader()) {
      resp.error_message = "Not Leader";
      resp.leader_hint = node_->leader_address();
    } else if (node_->config().all().size() <= 1) {
      resp.error_message = "Cannot remove server: would leave cluster empty";
    } else {
      Proposal p = propose(Json(Json::Object{{"Membership", Json(Json::Object{{"RemoveServer", Json(Json::Object{
          {"server_id", Json(static_cast<int64_t>(r.server_id))}})}})}}));
      if (p.code == 1) {
        resp.error_message = "Not Leader";
        resp.leader_hint = p.payload;
      } else if (p.code != 0) {
        return (*out = p.payload, INTERNAL);
      } else {
        resp.success = true;
      }
    }
    resp.encode(*out);
    return OK;
  }
  if (method == "GetClusterInfo") {
    Json info = Json::parse(node_->info_json());
    pb::GetClusterInfoResponse resp;
    resp.node_id = static_cast<uint32_t>(info["node_id"].as_int());
    resp.role = info["role"].str();
    resp.current_term = info["current_term"].as_u64();
    resp.leader_id = static_cast<uint32_t>(std::max<int64_t>(0, info["leader_id"].as_int(0)));
    resp.leader_address = info["leader_address"].str();
    resp.commit_index = info["commit_index"].as_u64();
    resp.last_applied = info["last_applied"].as_u64();
    for (auto& [id, addr] : node_->config().all()) {
      pb::ClusterMember m;
      m.server_id = static_cast<uint32_t>(id);
      m.address = addr;
      m.is_self = id == node_->id();
      resp.members.push_back(m);
    }
    resp.encode(*out);
    return OK;
  }
  if (method == "IngestMetadata") {
    pb::IngestMetadataRequest r;
    if (!r.decode(payload)) return (*out = "malformed IngestMetadataRequest", INVALID_ARGUMENT);
    std::string prefix;
    if (!r.files.empty()) {
      const std::string& p = r.files[0].path;
      size_t s = p.rfind('/');
      if (s != std::string::npos) prefix = p.substr(0, s + 1);
    }
    Json files = Json::array();
    for (auto& f : r.files) files.push_back(file_meta_json(f));
    pb::IngestMetadataResponse resp;
    Proposal p = propose(master_cmd("IngestBatch", Json(Json::Object{{"files", files}})));
    if (p.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = p.payload;
    } else if (p.code != 0) {
      return (*out = p.payload, INTERNAL);
    } else {
      resp.success = true;
      if (!prefix.empty()) node_->propose_nowait(master_cmd("TriggerShuffle", Json(Json::Object{{"prefix", Json(prefix)}})).dump());
    }
    resp.encode(*out);
    return OK;
  }
  if (method == "InitiateShuffle") {
    pb::InitiateShuffleRequest r;
    if (!r.decode(payload)) return (*out = "malformed InitiateShuffleRequest", INVALID_ARGUMENT);
    ShardMap m = map_copy();
    std::string target = m.get_shard(r.prefix), me = shard_id();
    if (!target.empty() && target != me) {
      auto peers = peers_of(m, target);
      return (*out = "REDIRECT:" + (peers.empty() ? std::string() : peers[0]), OUT_OF_RANGE);
    }
    if (core_->safe_mode_status()["is_safe_mode"].as_bool())
      return (*out = "Cluster is in Safe Mode. Write operations are blocked.", UNAVAILABLE);
    pb::InitiateShuffleResponse resp;
    Proposal p = propose(master_cmd("TriggerShuffle", Json(Json::Object{{"prefix", Json(r.prefix)}})));
    if (p.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = p.payload;
    } else if (p.code != 0) {
      return (*out = p.payload, INTERNAL);
    } else {
      resp.success = true;
    }
    resp.encode(*out);
    return OK;
  }
  return (*out = "Method not found: " + method, UNIMPLEMENTED);
}

// ---------------------------------------------------------------- background tasks
void Master::every(double first, double period, const char* name, std::function<void()> fn) {
  threads_.emplace_back([this, first, period, name, fn] {
    auto wait = [&](double s) {
      std::unique_lock<std::mutex> lk(stop_mu_);
      return !stop_cv_.wait_for(lk, std::chrono::duration<double>(s), [&] { return stop_.load(); });
    };
    if (!wait(first)) return;
    do {
      try {
        fn();
      } catch (const std::exception& e) {
        log(kError, kLog, "background task %s failed: %s", name, e.what());
      }
    } while (wait(period));
  });
}

void Master::liveness_check() {
  const int64_t now = now_ms();
  bool any = false;
  for (auto& s : core_->chunk_servers())
    if (now - s.last_heartbeat > cs_dead_ms_) {
      log(kWarning, kLog, "chunkserver %s missed heartbeats; removing", s.address.c_str());
      core_->remove_chunk_server(s.address);
      core_->take_commands(s.address);
      any = true;
    }
  if (any) heal();
}

void Master::heartbeat_reports() {
  auto [encoded, failed] = core_->take_ec_reports();
  {
    std::lock_guard<std::mutex> g(ec_mu_);
    for (auto& b : encoded) {
      auto it = ec_jobs_.find(b);
      if (it != ec_jobs_.end()) it->second.done = true;
    }
    for (auto& b : failed)
      if (ec_jobs_.erase(b)) log(kWarning, kLog, "EC conversion of block %s failed; will retry", b.c_str());
  }
  if (core_->take_heal_request()) {
    size_t n = heal();
    if (n) log(kInfo, kLog, "healer queued %zu commands after a bad-block report", n);
  }
}

// Healer (reference master.rs:436-602): the namespace scan is MasterCore::heal_scan; (block,
// target) pairs already queued anywhere are counted as copies on their way.
size_t Master::heal() {
  std::vector<std::string> live;
  for (auto& s : core_->chunk_servers()) live.push_back(s.address);
  if (live.empty()) return 0;
  std::sort(live.begin(), live.end());
  std::set<std::pair<std::string, std::string>> queued;
  for (auto& kv : core_->peek_commands())
    for (auto& raw : kv.second) {
      pb::ChunkServerCommand c;
      if (c.decode(raw) && !c.target_chunk_server_address.empty()) queued.emplace(c.block_id, c.target_chunk_server_address);
    }
  auto acts = core_->heal_scan(3, live, core_->bad_blocks(), queued);
  for (auto& a : acts) {
    pb::ChunkServerCommand c;
    c.block_id = a.block_id;
    c.target_chunk_server_address = a.target;
    if (a.reconstruct) {
      c.type = pb::ChunkServerCommand::RECONSTRUCT_EC_SHARD;
      c.shard_index = a.shard_index;
      c.ec_data_shards = a.ec_data;
      c.ec_parity_shards = a.ec_parity;
      c.ec_shard_sources = a.sources;
      c.original_block_size = a.original_size;
    } else {
      c.type = pb::ChunkServerCommand::REPLICATE;
      c.shard_index = -1;
    }
    queue(a.queue_on, c);
  }
  return acts.size();
}

void Master::balance() {
  auto servers = core_->chunk_servers();
  if (servers.size() < 2) return;
  std::sort(servers.begin(), servers.end(), [](const ChunkServerStatus& x, const ChunkServerStatus& y) {
    return x.available_space != y.available_space ? x.available_space < y.available_space : x.address < y.address;
  });
  const auto& lo = servers.front();
  const auto& hi = servers.back();
  if (hi.available_space - lo.available_space <= kBalanceGap) return;
  std::string bid = core_->pick_block(lo.address, hi.address, nullptr);
  if (bid.empty()) return;
  pb::ChunkServerCommand c;
  c.type = pb::ChunkServerCommand::REPLICATE;
  c.block_id = bid;
  c.target_chunk_server_address = hi.address;
  queue(lo.address, c);
  log(kInfo, kLog, "balancer: replicate %s %s -> %s", bid.c_str(), lo.address.c_str(), hi.address.c_str());
}

void Master::shuffle() {
  auto prefixes = core_->shuffling_prefixes();
  auto servers = core_->chunk_servers();
  if (prefixes.empty() || servers.size() < 2) return;
  std::sort(prefixes.begin(), prefixes.end());
  std::stable_sort(servers.begin(), servers.end(), [](const ChunkServerStatus& x, const ChunkServerStatus& y) {
    return x.available_space > y.available_space;
  });
  const std::string coolest = servers.front().address, hottest = servers.back().address;
  for (auto& p : prefixes) {
    std::string bid = core_->pick_block(hottest, coolest, &p);
    if (!bid.empty()) {
      pb::ChunkServerCommand c;
      c.type = pb::ChunkServerCommand::REPLICATE;
      c.block_id = bid;
      c.target_chunk_server_address = coolest;
      queue(hottest, c);
    } else if (is_leader()) {
      propose_master("StopShuffle", Json(Json::Object{{"prefix", Json(p)}}));
    }
  }
}

std::string Master::inquire(const Json& rec) {
  ShardMap m = map_copy();
  auto peers = peers_of(m, rec["coordinator_shard"].str());
  if (peers.empty())
    for (auto& p : rec["coordinator_peers"].items()) peers.push_back(p.str());
  pb::InquireTransactionRequest req;
  req.tx_id = rec["tx_id"].str();
  for (auto& addr : peers) {
    GrpcResult r = call(addr, "MasterService", "InquireTransaction", req.str(), 3000);
    pb::InquireTransactionResponse resp;
    if (r.transport_ok && r.status == 0 && resp.decode(r.message)) return resp.status;
  }
  return "";
}

// 2PC maintenance (reference master.rs:968-1180): abort stale Pending/Prepared records, ask
// the coordinator what became of a participant's Prepared record, drop old finished ones.
void Master::tx_cleanup() {
  if (!is_leader()) return;
  const std::string shard = shard_id();
  Json recs = Json::parse(core_->tx_records());
  const int64_t now = now_ms();
  for (auto& [tx_id, rec] : recs.fields()) {
    const int64_t age = now - rec["timestamp"].as_int();
    const bool timed_out = age > tx_timeout_ms_, stale = age > kTxStaleMs;
    if (!timed_out && !stale) continue;
    const std::string st = rec["state"].str(), coord = rec["coordinator_shard"].str();
    auto set_state = [&](const char* s) {
      propose_master("UpdateTransactionState", Json(Json::Object{{"tx_id", Json(tx_id)}, {"new_state", Json(s)}}));
    };
    if (coord.empty()) {
      if ((st == "Pending" || st == "Prepared") && timed_out) set_state("Aborted");
      else if (stale) propose_master("DeleteTransactionRecord", Json(Json::Object{{"tx_id", Json(tx_id)}}));
      continue;
    }
    const bool is_coord = coord == shard;
    if (st == "Pending") {
      set_state("Aborted");
    } else if (st == "Prepared" && !is_coord) {
      std::string status = inquire(rec);
      if (status == "COMMITTED") {
        if (rec["operations"].size())
          propose_master("ApplyTransactionOperation",
                         Json(Json::Object{{"tx_id", Json(tx_id)}, {"operation", rec["operations"][0]}}));
        set_state("Committed");
      } else if (status == "ABORTED") {
        set_state("Aborted");
      } else if (status == "UNKNOWN") {
        propose_master("IncrementInquiryCount", Json(Json::Object{{"tx_id", Json(tx_id)}}));
        if (rec["inquiry_count"].as_int() + 1 > kMaxInquiryRetries) {
          log(kWarning, kLog, "tx %s: presuming abort after %d inquiries", tx_id.c_str(), kMaxInquiryRetries);
          set_state("Aborted");
        }
      }
    } else if ((st == "Committed" || st == "Aborted") && stale) {
      if (st == "Committed" && is_coord && !rec["participant_acked"].as_bool()) continue;
      propose_master("DeleteTransactionRecord", Json(Json::Object{{"tx_id", Json(tx_id)}}));
    }
  }
}

// Coordinator recovery (reference master.rs:1182-1322): re-send CommitTransaction for
// records whose participant never acknowledged, finishing the source side afterwards.
void Master::tx_recovery() {
  if (!is_leader()) return;
  const std::string shard = shard_id();
  Json recs = Json::parse(core_->tx_records());
  const int64_t now = now_ms();
  ShardMap m = map_copy();
  for (auto& [tx_id, rec] : recs.fields()) {
    if (rec["coordinator_shard"].str() != shard) continue;
    const std::string st = rec["state"].str();
    const bool timed_out = now - rec["timestamp"].as_int() > tx_timeout_ms_;
    if (!((st == "Committed" && !rec["participant_acked"].as_bool()) || (st == "Prepared" && timed_out))) continue;
    std::string dest;
    for (auto& p : rec["participants"].items())
      if (p.str() != shard) {
        dest = p.str();
        break;
      }
    auto peers = peers_of(m, dest);
    if (peers.empty()) continue;
    pb::CommitTransactionRequest req;
    req.tx_id = tx_id;
    if (!call_peers<pb::CommitTransactionResponse>(peers, "CommitTransaction", req.str())) continue;
    if (st == "Prepared") {
      for (auto& op : rec["operations"].items())
        if (op["op_type"].has("Delete")) {
          propose_master("ApplyTransactionOperation", Json(Json::Object{{"tx_id", Json(tx_id)}, {"operation", op}}));
          propose_master("UpdateTransactionState",
                         Json(Json::Object{{"tx_id", Json(tx_id)}, {"new_state", Json("Committed")}}));
          break;
        }
    }
    propose_master("SetParticipantAcked", Json(Json::Object{{"tx_id", Json(tx_id)}}));
    log(kInfo, kLog, "tx %s recovered (participant committed)", tx_id.c_str());
  }
}

void Master::decay() { monitor_->decay(core_->take_request_counts(), iv_.decay); }

bool Master::refresh_shard_map() {
  if (config_servers_.empty()) return false;
  std::lock_guard<std::mutex> serial(refresh_mu_);
  pb::FetchShardMapResponse resp;
  if (!config_call("FetchShardMap", pb::FetchShardMapRequest().str(), &resp) || resp.shards.empty()) return false;
  std::map<std::string, std::vector<std::string>> shards;
  for (auto& kv : resp.shards) shards[kv.first] = kv.second.peers;
  ShardMap m = map_from_config(shards, resp.ranges);
  map_fetched_ms_ = now_ms();
  std::string sid = shard_id();
  if (sid.empty()) {  // standby master: a SplitShard allocated us a shard
    for (auto& s : m.shards()) {
      auto peers = peers_of(m, s);
      if (std::find(peers.begin(), peers.end(), client_addr_) != peers.end()) {
        sid = s;
        log(kInfo, kLog, "standby master %s now serves shard %s", client_addr_.c_str(), s.c_str());
        break;
      }
    }
  }
  set_routing(&m, &sid);
  core_->note_shard_map_fresh();
  return true;
}

void Master::do_register() {
  if (registered_ || config_servers_.empty()) return;
  pb::RegisterMasterRequest req;
  req.address = client_addr_;
  req.shard_id = shard_id();
  pb::RegisterMasterResponse resp;
  registered_ = config_call("RegisterMaster", req.str(), &resp) && resp.success;
}

void Master::split_detector() {
  if (config_servers_.empty()) return;
  do_register();
  pb::ShardHeartbeatRequest hb;
  hb.address = client_addr_;
  hb.rps_per_prefix = monitor_->rps();
  pb::ShardHeartbeatResponse hr;
  config_call("ShardHeartbeat", hb.str(), &hr);
  if (!is_leader()) return;
  const std::string sid = shard_id();
  std::string prefix;
  double rps = 0;
  if (monitor_->hot(&prefix, &rps) && !sid.empty()) {
    split(prefix, rps);
    return;
  }
  if (0 <= monitor_->merge_rps() && monitor_->total() < monitor_->merge_rps() && core_->file_count() && !sid.empty()) {
    ShardMap m = map_copy();
    if (m.strategy() != ShardMap::Strategy::Range) return;
    std::vector<std::string> order;
    for (auto& kv : m.ranges()) order.push_back(kv.second);
    for (size_t i = 0; i < order.size(); ++i)
      if (order[i] == sid) {
        std::string n = i > 0 ? order[i - 1] : (i + 1 < order.size() ? order[i + 1] : "");
        if (!n.empty()) merge_into(n);
        return;
      }
  }
}

// Split at `prefix` (C31; reference master.rs:1483-1640): the files that move are exactly
// those the post-split map routes to the new shard. Config SplitShard (allocates standby
// masters), IngestMetadata at the new shard, then one Raft entry dropping the moved files.
void Master::split(const std::string& prefix, double rps) {
  const std::string sid = shard_id();
  const std::string new_id = sid + "-split-" + uuid4().substr(0, 8);
  ShardMap after = map_copy();
  monitor_->mark_split();
  if (!after.split_shard(prefix, new_id, {})) return;
  log(kInfo, kLog, "hot prefix %s (%.1f rps): splitting shard %s -> %s", prefix.c_str(), rps, sid.c_str(),
      new_id.c_str());
  std::vector<std::string> moving;
  for (auto& p : core_->paths("", false))
    if (after.get_shard(p) == new_id) moving.push_back(p);
  pb::SplitShardRequest req;
  req.shard_id = sid;
  req.split_key = prefix;
  req.new_shard_id = new_id;
  pb::SplitShardResponse resp;
  if (!config_call("SplitShard", req.str(), &resp) || !resp.success) {
    log(kWarning, kLog, "config server refused split of %s at %s", sid.c_str(), prefix.c_str());
    return;
  }
  if (!moving.empty()) {
    pb::IngestMetadataRequest ing;
    for (auto& p : moving) {
      std::string raw;
      pb::FileMetadata f;
      if (core_->get_file(p, false, &raw) && f.decode(raw)) ing.files.push_back(std::move(f));
    }
    call_peers<pb::IngestMetadataResponse>(resp.new_shard_peers, "IngestMetadata", ing.str());
  }
  Json paths = Json::array(), peers = Json::array();
  for (auto& p : moving) paths.push_back(p);
  for (auto& p : resp.new_shard_peers) peers.push_back(p);
  propose_master("SplitShard", Json(Json::Object{{"split_key", Json(prefix)}, {"new_shard_id", Json(new_id)},
                                                 {"new_shard_peers", peers}, {"paths", paths}}));
  refresh_shard_map();
}

// Hand this idle shard's range and files to `neighbor` (C31 merge, reference
// master.rs:1642-1837): the config server's MergeShard arbitrates first, then the files go
// over with IngestMetadata (retried until the retained shard takes them), then one Raft entry
// drops the namespace here and the master re-registers as a standby.
void Master::merge_into(const std::string& neighbor) {
  const std::string victim = shard_id();
  pb::MergeShardRequest req;
  req.victim_shard_id = victim;
  req.retained_shard_id = neighbor;
  pb::MergeShardResponse resp;
  if (!config_call("MergeShard", req.str(), &resp) || !resp.success) return;
  auto peers = peers_of(map_copy(), neighbor);
  const std::string none;
  set_routing(nullptr, &none);  // stop accepting our old range (requests now redirect)
  std::vector<std::string> paths = core_->paths("", false);
  bool ok = false;
  for (int attempt = 0; attempt < 30 && !stop_; ++attempt) {
    pb::IngestMetadataRequest ing;
    for (auto& p : paths) {
      std::string raw;
      pb::FileMetadata f;
      if (core_->get_file(p, false, &raw) && f.decode(raw)) ing.files.push_back(std::move(f));
    }
    if (ing.files.empty() || call_peers<pb::IngestMetadataResponse>(peers, "IngestMetadata", ing.str())) {
      ok = true;
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(std::min(100 * (attempt + 1), 1000)));
  }
  if (!ok) {
    log(kError, kLog, "merge of %s into %s: ingest kept failing; files stay here", victim.c_str(), neighbor.c_str());
    return;
  }
  Json jp = Json::array();
  for (auto& p : paths) jp.push_back(p);
  propose_master("SplitShard", Json(Json::Object{{"split_key", Json("")}, {"new_shard_id", Json(neighbor)},
                                                 {"new_shard_peers", Json::array()}, {"paths", jp}}));
  log(kInfo, kLog, "merged shard %s into %s; now standby", victim.c_str(), neighbor.c_str());
  registered_ = false;
  refresh_shard_map();
}

// Tiering (C32; reference master.rs:1990-2060 + bin/master.rs:229-238): idle files move to
// the cold tier (MOVE_TO_COLD on every holder, then one MoveToCold entry); with
// EC_CONVERSION_ENABLED cold files older than EC_THRESHOLD_SECS are re-encoded to RS(k,m).
void Master::tiering() {
  if (!is_leader()) return;
  const int64_t now = now_ms();
  for (auto& f : core_->tiering_scan(static_cast<uint64_t>(now), static_cast<uint64_t>(cold_ms_))) {
    for (auto& [bid, locs] : f.blocks)
      for (auto& loc : locs) {
        pb::ChunkServerCommand c;
        c.type = pb::ChunkServerCommand::MOVE_TO_COLD;
        c.block_id = bid;
        queue(loc, c);
      }
    propose_master("MoveToCold", Json(Json::Object{{"path", Json(f.path)}, {"moved_at_ms", Json(now)}}));
  }
  if (ec_conversion_) ec_convert(now);
}

// Each block of a file is re-encoded by a chunkserver holding a replica (ENCODE_EC, GPU RS
// kernel) under a new block id; once every block reported success one ConvertToEc entry swaps
// the metadata and the old replicas get DELETE. Jobs are leader-local; a failed or lost job is
// retried on a later pass.
void Master::ec_convert(int64_t now) {
  const int k = ec_k_, m = ec_m_;
  std::lock_guard<std::mutex> g(ec_mu_);
  for (auto it = ec_jobs_.begin(); it != ec_jobs_.end();) {
    if (!it->second.done && now - it->second.started_ms > kEcJobTimeoutMs) {
      log(kWarning, kLog, "EC job for %s timed out; will retry", it->first.c_str());
      it = ec_jobs_.erase(it);
    } else {
      ++it;
    }
  }
  std::vector<std::string> live;
  for (auto& s : core_->chunk_servers())
    if (s.available_space > 0) live.push_back(s.address);
  std::sort(live.begin(), live.end());
  for (auto& raw : core_->ec_candidates(static_cast<uint64_t>(now), static_cast<uint64_t>(ec_ms_))) {
    pb::FileMetadata f;
    if (!f.decode(raw) || f.blocks.empty()) continue;
    bool all_done = true;
    for (auto& b : f.blocks) {
      auto it = ec_jobs_.find(b.block_id);
      if (it == ec_jobs_.end() || !it->second.done) all_done = false;
    }
    if (all_done) {
      Json blocks = Json::array();
      std::vector<std::pair<std::string, std::vector<std::string>>> old;
      for (auto& b : f.blocks) {
        const EcJob& job = ec_jobs_[b.block_id];
        pb::BlockInfo nb = b;
        nb.block_id = job.new_id;
        nb.locations = job.targets;
        nb.ec_data_shards = job.k;
        nb.ec_parity_shards = job.m;
        nb.original_size = b.original_size ? b.original_size : b.size;
        blocks.push_back(block_info_json(nb));
        old.emplace_back(b.block_id, b.locations);
      }
      const EcJob& j0 = ec_jobs_[f.blocks[0].block_id];
      const int jk = j0.k, jm = j0.m;
      bool ok = propose_master("ConvertToEc", Json(Json::Object{{"path", Json(f.path)}, {"ec_data_shards", Json(jk)},
                                                              {"ec_parity_shards", Json(jm)}, {"new_blocks", blocks}}));
      for (auto& [bid, locs] : old) {
        ec_jobs_.erase(bid);
        if (ok)
          for (auto& loc : locs) {
            pb::ChunkServerCommand c;
            c.type = pb::ChunkServerCommand::DELETE;
            c.block_id = bid;
            queue(loc, c);
          }
      }
      if (ok) log(kInfo, kLog, "converted %s to RS(%d,%d)", f.path.c_str(), jk, jm);
      continue;
    }
    if (live.size() < static_cast<size_t>(k + m)) continue;
    std::vector<std::string> servers(live.begin(), live.begin() + k + m);
    for (auto& b : f.blocks) {
      if (ec_jobs_.count(b.block_id)) continue;
      std::string src;
      for (auto& loc : b.locations)
        if (std::binary_search(live.begin(), live.end(), loc)) {
          src = loc;
          break;
        }
      if (src.empty()) continue;
      EcJob job;
      job.path = f.path;
      job.new_id = b.block_id + "-rs" + std::to_string(k) + "." + std::to_string(m);
      job.targets = servers;
      job.k = k;
      job.m = m;
      job.started_ms = now;
      pb::ChunkServerCommand c;
      c.type = pb::ChunkServerCommand::ENCODE_EC;
      c.block_id = b.block_id;
      c.new_block_id = job.new_id;
      c.ec_data_shards = k;
      c.ec_parity_shards = m;
      c.ec_shard_sources = servers;
      c.original_block_size = b.size;
      c.master_term = node_->term();
      ec_jobs_[b.block_id] = std::move(job);
      queue(src, c);
    }
  }
}

// ---------------------------------------------------------------- HTTP side channel
HttpResponse Master::http(const HttpRequest& req) {
  if (req.path.rfind("/raft/", 0) == 0 && req.method == "POST") return raft_http(*node_, req);
  if (req.path == "/health") return HttpResponse{200, "text/plain", "OK"};
  if (req.path == "/raft/state") return json_response(node_->info_json());
  if (req.path == "/raft/endpoint") return json_response(Json(Json::Object{{"grpc", Json(client_addr_)}}).dump());
  if (req.path == "/shard_map") {
    std::lock_guard<std::mutex> g(map_mu_);
    return json_response(Json(Json::Object{{"shard_id", Json(shard_id_)}, {"map", map_.to_json()}}).dump());
  }
  if (req.path == "/debug/partition" && req.method == "POST" && env("DFS_DEBUG_ENDPOINTS") == "1") {
    std::set<std::string> blocked;
    try {
      const Json body = Json::parse(req.body);  // (the loop below must not range over a temporary's member)
      for (auto& b : body["block"].items()) {
        std::string x = b.str();
        while (!x.empty() && x.back() == '/') x.pop_back();
        blocked.insert(with_scheme(x));
      }
    } catch (...) {
      return HttpResponse{400, "text/plain", "bad request"};
    }
    raft_host_->set_blocked({blocked.begin(), blocked.end()});
    Json arr = Json::array();
    for (auto& b : blocked) arr.push_back(b);
    return json_response(Json(Json::Object{{"blocked", arr}}).dump());
  }
  return HttpResponse{404, "text/plain", "Not Found"};
}

int Master::run() {
  const std::string addr = a_.get("addr", "127.0.0.1:50051");
  const int id = static_cast<int>(a_.get_int("id", 1));
  const int http_port = static_cast<int>(a_.get_int("http-port", 8080));
  const std::string host = addr.find(':') != std::string::npos ? addr.substr(0, addr.find(':')) : "127.0.0.1";
  const std::string http_host = a_.get("http-host", host);
  self_http_ = "http://" + http_host + ":" + std::to_string(http_port);
  client_addr_ = with_scheme(a_.get("advertise-addr", addr));
  const std::string tls_cert = a_.get("tls-cert"), tls_key = a_.get("tls-key"), ca = a_.get("ca-cert"),
                    domain = a_.get("domain-name");
  const bool tls = !tls_cert.empty() && !tls_key.empty();
  cs_dead_ms_ = std::atoll(env("DFS_CS_DEAD_MS", "15000").c_str());
  tx_timeout_ms_ = std::atoll(env("DFS_TX_TIMEOUT_MS", "10000").c_str());
  cold_ms_ = std::atoll(env("COLD_THRESHOLD_SECS", "604800").c_str()) * 1000;
  ec_ms_ = std::atoll(env("EC_THRESHOLD_SECS", "2592000").c_str()) * 1000;
  ec_conversion_ = env("EC_CONVERSION_ENABLED", "0") == "1";
  ec_k_ = std::atoi(env("EC_CONVERSION_DATA_SHARDS", "6").c_str());
  ec_m_ = std::atoi(env("EC_CONVERSION_PARITY_SHARDS", "3").c_str());
  iv_ = a_.flag("fast-intervals") ? Intervals::fast() : Intervals();
  monitor_ = std::make_unique<ThroughputMonitor>(a_.get_double("split-threshold-rps", 100.0),
                                                 a_.get_double("merge-threshold-rps", 1.0),
                                                 static_cast<int>(a_.get_int("split-cooldown-secs", 30)));
  std::string err;
  std::shared_ptr<TlsContext> client_tls;
  if (!ca.empty()) {
    client_tls = TlsContext::client(ca, domain, &err);
    if (!client_tls) {
      std::fprintf(stderr, "dfs_master: client TLS: %s\n", err.c_str());
      return 1;
    }
  }
  pool_ = std::make_unique<GrpcChannelPool>(5000, client_tls);

  core_ = std::make_shared<MasterCore>();
  raft::Options o;
  o.id = id;
  o.members = initial_members(id, self_http_, split_csv(a_.get("peers")));
  o.client_address = client_addr_;
  o.dir = a_.get("storage-dir", "/tmp/raft-logs") + "/raft_node_" + std::to_string(id);
  o.sync = !a_.flag("no-fsync");
  o.snapshot_threshold = static_cast<uint64_t>(a_.get_int("snapshot-threshold", 10000));
  o.backup_endpoint = a_.get("backup-s3-endpoint");
  o.backup_bucket = a_.get("backup-bucket", "dfs-backups");
  if (!a_.get("restore-snapshot").empty()) {
    // seed an empty storage dir from an off-box snapshot backup (a file, or the object's
    // http(s) URL), then start as usual with this command line's members
    const std::string src = a_.get("restore-snapshot");
    std::string payload;
    if (src.rfind("http://", 0) == 0 || src.rfind("https://", 0) == 0) {
      const int st = http_request("GET", src, "", "", 60000, &payload, &err);
      if (st != 200) {
        std::fprintf(stderr, "dfs_master: restore: GET %s: %s\n", src.c_str(),
                     err.empty() ? std::to_string(st).c_str() : err.c_str());
        return 2;
      }
    } else {
      std::ifstream f(src, std::ios::binary);
      if (!f) {
        std::fprintf(stderr, "dfs_master: restore: cannot read %s\n", src.c_str());
        return 2;
      }
      std::stringstream ss;
      ss << f.rdbuf();
      payload = ss.str();
    }
    if (!raft::restore_snapshot_dir(o.dir, payload, &err)) {
      std::fprintf(stderr, "dfs_master: restore: %s\n", err.c_str());
      return 2;
    }
    log(kWarning, "dfs.master", "restored %s into %s", src.c_str(), o.dir.c_str());
  }
  raft_host_ = std::make_shared<NativeRaftHost>(core_, tls ? client_tls : nullptr);
  node_ = std::make_unique<raft::Node>(o, raft_host_);
  core_->attach(node_.get());
  {
    auto p2pc = std::make_shared<GrpcChannelPool>(5000, client_tls);  // 2PC peer calls (native coordinator)
    core_->enable_native_2pc([p2pc](const std::string& target, const std::string& path, const std::string& req,
                                    int timeout_ms) { return p2pc->call(target, path, req, t_request_id, timeout_ms); });
  }
  core_->enter_safe_mode(false);
  core_->set_access_stats(true, 1000);
  config_servers_.clear();
  for (auto& c : split_csv(a_.get("config-servers"))) config_servers_.push_back(with_scheme(c));
  ShardMap initial = config_servers_.empty() ? load_shard_config(a_.get("shard-config")) : ShardMap::new_range();
  const std::string sid = a_.flag("standby") ? "" : a_.get("shard-id", "shard-0");
  set_routing(&initial, &sid);
  if (!config_servers_.empty()) core_->set_shard_map_max_age(1000);

  // MasterService + Raft peer RPCs over HTTP/2
  static const std::string kRaft = "/dfs.RaftPeer/";
  const std::string bind = addr.find(':') != std::string::npos ? addr : "0.0.0.0:" + addr;
  const int gport = std::atoi(bind.substr(bind.rfind(':') + 1).c_str());
  grpc_ = std::make_unique<GrpcServer>(bind.substr(0, bind.rfind(':')), gport, [this](const GrpcCall& c) -> GrpcReply {
    GrpcReply r;
    if (c.path.compare(0, kRaft.size(), kRaft) == 0) {
      r.status = core_->raft_rpc(c.path.substr(kRaft.size()), c.message, &r.message);
      raft_calls_++;
      return r;
    }
    bool native = false;
    r.status = handle(c.path, c.request_id, c.message, &r.message, &native);
    (native ? native_calls_ : cold_calls_)++;
    return r;
  }, 32);
  if (tls) {
    auto t = TlsContext::server(tls_cert, tls_key, &err);
    if (!t) {
      std::fprintf(stderr, "dfs_master: TLS: %s\n", err.c_str());
      return 1;
    }
    grpc_->set_tls(std::move(t));
  }
  if (!grpc_->start(&err)) {
    std::fprintf(stderr, "dfs_master: gRPC server: %s\n", err.c_str());
    return 1;
  }
  if (env("DFS_NO_LOCALRPC") != "1") {
    local_ = std::make_unique<LocalRpcServer>(
        "dfs_rpc_" + std::to_string(gport),
        [this](const std::string& path, const std::string& rid, const std::string& payload, std::string* out) {
          bool native = false;
          return handle(path, rid, payload, out, &native);
        });
    if (!local_->start(&err)) {
      log(kWarning, kLog, "local RPC listener unavailable: %s", err.c_str());
      local_.reset();
    }
  }

  Gauges g;
  g.add("raft_role", "0=follower 1=candidate 2=leader", [&] { return static_cast<double>(static_cast<int>(node_->role())); });
  g.add("raft_current_term", "current term", [&] { return static_cast<double>(node_->term()); });
  g.add("raft_commit_index", "commit index", [&] { return static_cast<double>(node_->commit_index()); });
  g.add("raft_last_applied", "last applied", [&] { return static_cast<double>(node_->last_applied()); });
  g.add("raft_log_len", "log length", [&] { return static_cast<double>(node_->last_index()); });
  g.add("raft_votes_received", "votes", [&] { return static_cast<double>(node_->votes()); });
  g.add("raft_wal_fsyncs", "WAL group-commit fsyncs", [&] { return static_cast<double>(node_->wal_syncs()); });
  g.add("dfs_master_safe_mode_status", "1 if in safe mode",
        [&] { return core_->safe_mode_status()["is_safe_mode"].as_bool() ? 1.0 : 0.0; });
  g.add("dfs_master_files", "files in this shard", [&] { return static_cast<double>(core_->file_count()); });
  g.add("dfs_master_chunkservers", "live chunkservers", [&] { return static_cast<double>(core_->chunk_servers().size()); });
  g.add("dfs_master_native_requests", "requests served by the native handlers",
        [&] { return static_cast<double>(core_->requests()); });
  g.add("dfs_master_native_heartbeats", "chunkserver heartbeats served by the native handler",
        [&] { return static_cast<double>(core_->heartbeats()); });
  for (const char* k : {"native_started", "native_committed", "native_aborted", "native_pending", "declined"})
    g.add(std::string("dfs_master_tx_") + k, "cross-shard rename (native 2PC) counter",
          [&, k] { return core_->txn_stats()[k].as_double(); });
  g.add("dfs_master_native_grpc_calls", "gRPC calls served by the native HTTP/2 server",
        [&] { return static_cast<double>(grpc_->calls()); });
  g.add("dfs_master_native_grpc_fallback", "gRPC calls answered outside MasterCore (cold RPCs, in this process)",
        [&] { return static_cast<double>(cold_calls_.load()); });
  g.add("dfs_master_native_raft_rpcs", "Raft peer RPCs received over the native server",
        [&] { return static_cast<double>(raft_calls_.load()); });
  g.add("dfs_master_native_process", "1: this master is the native dfs_master executable (no Python)",
        [] { return 1.0; });
  http_ = std::make_unique<HttpLiteServer>(http_host == "localhost" ? "127.0.0.1" : http_host, http_port,
                                           [this, &g](const HttpRequest& req) {
                                             if (req.path == "/metrics") return HttpResponse{200, "text/plain", g.render()};
                                             return http(req);
                                           });
  if (!http_->start(&err)) {
    std::fprintf(stderr, "dfs_master: %s\n", err.c_str());
    return 1;
  }
  node_->start();
  threads_.emplace_back([this] { resolve_peers_loop(*node_, *raft_host_, stop_); });
  if (!config_servers_.empty()) {
    do_register();
    refresh_shard_map();
  }
  every(iv_.liveness, iv_.liveness, "liveness_check", [this] { liveness_check(); });
  every(iv_.healer_first, iv_.healer, "periodic_heal", [this] {
    size_t n = heal();
    if (n) log(kInfo, kLog, "healer queued %zu commands", n);
  });
  every(iv_.balancer, iv_.balancer, "balance", [this] { balance(); });
  every(iv_.tx_cleanup, iv_.tx_cleanup, "tx_cleanup", [this] { tx_cleanup(); });
  every(iv_.tx_recovery, iv_.tx_recovery, "tx_recovery", [this] { tx_recovery(); });
  every(iv_.shuffler, iv_.shuffler, "shuffle", [this] { shuffle(); });
  every(iv_.decay, iv_.decay, "decay", [this] { decay(); });
  every(iv_.shard_refresh, iv_.shard_refresh, "refresh_shard_map", [this] { refresh_shard_map(); });
  every(iv_.split, iv_.split, "split_detector", [this] { split_detector(); });
  every(iv_.tiering, iv_.tiering, "tiering", [this] { tiering(); });
  every(0.25, 0.25, "heartbeat_reports", [this] { heartbeat_reports(); });
  write_ready_file(Json(Json::Object{{"addr", Json(addr)}, {"http", Json(self_http_)}, {"native", Json(true)}}).dump());
  log(kInfo, kLog, "master %d of %s serving %s (http %d)", id, sid.empty() ? "(standby)" : sid.c_str(), addr.c_str(),
      http_port);

  wait_for_stop();
  {
    std::lock_guard<std::mutex> lk(stop_mu_);
    stop_ = true;
  }
  stop_cv_.notify_all();
  for (auto& t : threads_) t.join();
  if (local_) local_->stop();
  grpc_->stop();
  http_->stop();
  node_->stop();
  core_->detach();
  return 0;
}

}  // namespace

const char* kUsage =
    "usage: dfs_master [-a ADDR | --addr ADDR] [--id ID] [--peers PEERS] [--http-port HTTP_PORT]\n"
    "                  [--advertise-addr ADVERTISE_ADDR] [--storage-dir STORAGE_DIR] [--shard-id SHARD_ID]\n"
    "                  [--standby] [--shard-config SHARD_CONFIG] [--config-servers CONFIG_SERVERS]\n"
    "                  [--split-threshold-rps SPLIT_THRESHOLD_RPS] [--split-cooldown-secs SPLIT_COOLDOWN_SECS]\n"
    "                  [--merge-threshold-rps MERGE_THRESHOLD_RPS] [--tls-cert TLS_CERT] [--tls-key TLS_KEY]\n"
    "                  [--ca-cert CA_CERT] [--domain-name DOMAIN_NAME] [--backup-s3-endpoint BACKUP_S3_ENDPOINT]\n"
    "                  [--backup-bucket BACKUP_BUCKET] [--snapshot-threshold SNAPSHOT_THRESHOLD] [--no-fsync]\n"
    "                  [--fast-intervals] [--http-host HTTP_HOST] [--restore-snapshot FILE_OR_URL]\n";

// The reference's defaults (bin/master.rs:21-80), printed by --help.
const std::map<std::string, std::string> kDefaults = {
    {"addr", "127.0.0.1:50051"},   {"id", "1"},
    {"http-port", "8080"},         {"storage-dir", "/tmp/raft-logs"},
    {"shard-id", "shard-0"},       {"split-threshold-rps", "100.0"},
    {"split-cooldown-secs", "30"}, {"merge-threshold-rps", "1.0"},
    {"backup-bucket", "dfs-backups"}, {"snapshot-threshold", "10000"}};

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--help" || std::string(argv[i]) == "-h") {
      std::fputs(kUsage, stdout);
      std::fputs(defaults_help(kDefaults).c_str(), stdout);
      return 0;
    }
  block_stop_signals();
  Args a(argc, argv, {"standby", "no-fsync", "fast-intervals"}, {{"a", "addr"}}, kDefaults);
  if (!a.error().empty()) {
    std::fprintf(stderr, "dfs_master: %s\n", a.error().c_str());
    return 2;
  }
  Master m(a);
  return m.run();
}
