#include "config_core.h"

#include <algorithm>
#include <chrono>
#include <future>
#include <memory>

#include "dfs_pb.h"

namespace dfs {

namespace {
int64_t now_s() {
  return std::chrono::duration_cast<std::chrono::seconds>(std::chrono::system_clock::now().time_since_epoch()).count();
}
std::vector<std::string> strings(const Json& a) {
  std::vector<std::string> v;
  for (size_t i = 0; i < a.size(); ++i) v.push_back(a[i].str());
  return v;
}
}  // namespace

ConfigCore::ConfigCore() : map_(ShardMap::new_range()) {}

std::vector<std::string> ConfigCore::apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) {
  std::vector<std::string> out;
  out.reserve(cmds.size());
  std::lock_guard<std::mutex> g(mu_);
  for (auto& c : cmds) {
    Json r;
    try {
      r = apply_one(Json::parse(c.second));
    } catch (const std::exception& e) {
      out.push_back(std::string("!") + e.what());
      continue;
    }
    ++version_;
    out.push_back(r.dump());
  }
  return out;
}

Json ConfigCore::apply_one(const Json& cmd) {
  const Json* cfg = cmd.is_object() ? cmd.find("Config") : nullptr;
  if (!cfg || !cfg->is_object() || cfg->fields().empty()) return Json();  // NoOp / foreign command
  const std::string& name = cfg->fields().front().first;
  const Json& a = cfg->fields().front().second;
  if (name == "AddShard") {
    map_.add_shard(a["shard_id"].str(), strings(a["peers"]));
  } else if (name == "RemoveShard") {
    map_.remove_shard(a["shard_id"].str());
  } else if (name == "SplitShard") {
    auto peers = strings(a["new_shard_peers"]);
    bool ok = map_.split_shard(a["split_key"].str(), a["new_shard_id"].str(), peers);
    if (ok)
      for (auto& p : peers) {
        auto it = masters_.find(p);
        if (it != masters_.end()) it->second.shard_id = a["new_shard_id"].str();
      }
    return Json(ok);
  } else if (name == "MergeShard") {
    return Json(map_.merge_shards(a["victim_shard_id"].str(), a["retained_shard_id"].str()));
  } else if (name == "RebalanceShard") {
    return Json(map_.rebalance_boundary(a["old_key"].str(), a["new_key"].str()));
  } else if (name == "RegisterMaster") {
    std::string addr = a["address"].str(), sid = a["shard_id"].str();
    MasterInfo info;
    info.last_heartbeat = now_s();
    if (sid.empty()) {
      // standby: waits for a SplitShard allocation; one a split already placed keeps it
      for (auto& s : map_.shards()) {
        const auto* p = map_.peers(s);
        if (p && std::find(p->begin(), p->end(), addr) != p->end()) {
          info.shard_id = s;
          break;
        }
      }
    } else {
      if (!map_.has_shard(sid)) {
        map_.add_shard(sid, {addr});
      } else {
        std::vector<std::string> peers = map_.peers(sid) ? *map_.peers(sid) : std::vector<std::string>{};
        if (std::find(peers.begin(), peers.end(), addr) == peers.end()) {
          peers.push_back(addr);
          map_.add_shard(sid, peers);
        }
      }
      info.shard_id = sid;
    }
    masters_[addr] = std::move(info);
  } else if (name == "ShardHeartbeat") {
    auto it = masters_.find(a["address"].str());
    if (it != masters_.end()) {
      it->second.last_heartbeat = now_s();
      it->second.rps = a["rps_per_prefix"].is_object() ? a["rps_per_prefix"] : Json::object();
    }
  } else {
    throw std::runtime_error("unknown config command " + name);
  }
  return Json();
}

Json ConfigCore::snapshot_locked() const {
  Json masters = Json::object();
  for (auto& kv : masters_) {
    Json m = Json::object();
    m.set("address", kv.first);
    m.set("shard_id", kv.second.shard_id);
    m.set("last_heartbeat", kv.second.last_heartbeat);
    m.set("rps_per_prefix", kv.second.rps);
    masters.set(kv.first, m);
  }
  Json inner = Json::object();
  inner.set("shard_map", map_.to_json());
  inner.set("masters", masters);
  Json out = Json::object();
  out.set("Config", inner);
  return out;
}

std::string ConfigCore::snapshot() {
  std::lock_guard<std::mutex> g(mu_);
  return snapshot_locked().dump();
}

void ConfigCore::restore(const std::string& state) {
  Json j = Json::parse(state);
  const Json& c = j.has("Config") ? j["Config"] : j;
  std::lock_guard<std::mutex> g(mu_);
  map_ = c.has("shard_map") ? ShardMap::from_json(c["shard_map"]) : ShardMap::new_range();
  masters_.clear();
  const Json& ms = c["masters"];
  if (ms.is_object())
    for (auto& kv : ms.fields()) {
      MasterInfo m;
      m.shard_id = kv.second["shard_id"].str();
      m.last_heartbeat = kv.second["last_heartbeat"].as_int();
      m.rps = kv.second["rps_per_prefix"].is_object() ? kv.second["rps_per_prefix"] : Json::object();
      masters_[kv.first] = std::move(m);
    }
  ++version_;
}

std::string ConfigCore::shard_map_json() const {
  std::lock_guard<std::mutex> g(mu_);
  return map_.to_json().dump();
}

std::string ConfigCore::masters_json() const {
  std::lock_guard<std::mutex> g(mu_);
  return snapshot_locked()["Config"]["masters"].dump();
}

uint64_t ConfigCore::version() const {
  std::lock_guard<std::mutex> g(mu_);
  return version_;
}

std::vector<std::string> ConfigCore::split_candidates(size_t n) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::pair<int64_t, std::string>> all, standby;
  for (auto& kv : masters_) {
    all.push_back({-kv.second.last_heartbeat, kv.first});
    if (kv.second.shard_id.empty()) standby.push_back({-kv.second.last_heartbeat, kv.first});
  }
  std::stable_sort(all.begin(), all.end());
  std::stable_sort(standby.begin(), standby.end());
  auto& pick = standby.empty() ? all : standby;
  std::vector<std::string> out;
  for (size_t i = 0; i < pick.size() && i < n; ++i) out.push_back(pick[i].second);
  return out;
}

// ---------------------------------------------------------------- ConfigService
// Semantics of the reference's config_server.rs handlers (and of the Python service this
// replaces): mutations commit through Raft and answer success=false + "Not Leader" +
// leader_hint on a follower; FetchShardMap is a ReadIndex read (FAILED_PRECONDITION
// "Not Leader|<hint>" on a follower) returning shard -> peers plus the `ranges` extension;
// ShardHeartbeat is fire-and-forget on the leader.
namespace {
constexpr int kOk = 0, kFailedPrecondition = 9, kInternal = 13, kUnavailable = 14, kUnimplemented = 12;
Json jstrings(const std::vector<std::string>& v) {
  Json a = Json::array();
  for (auto& x : v) a.push_back(Json(x));
  return a;
}
}  // namespace

bool ConfigCore::native_method(const std::string& m) {
  return m == "FetchShardMap" || m == "AddShard" || m == "RemoveShard" || m == "SplitShard" || m == "MergeShard" ||
         m == "RebalanceShard" || m == "RegisterMaster" || m == "ShardHeartbeat";
}

ConfigCore::Result ConfigCore::propose(const std::string& name, const Json& args) {
  raft::Node* node = node_.load();
  if (!node) return {1, ""};
  Json inner = Json::object();
  inner.set(name, args);
  Json cmd = Json::object();
  cmd.set("Config", inner);
  auto prom = std::make_shared<std::promise<Result>>();
  auto fut = prom->get_future();
  node->propose(cmd.dump(), [prom](int code, const std::string& payload) { prom->set_value(Result{code, payload}); });
  if (fut.wait_for(std::chrono::seconds(30)) != std::future_status::ready) return {2, "proposal timed out"};
  return fut.get();
}

int ConfigCore::raft_rpc(const std::string& kind, const std::string& body, std::string* out) {
  raft::Node* node = node_.load();
  if (!node) return (*out = "raft node not attached", kUnavailable);
  try {
    *out = node->handle(kind, body);
    return kOk;
  } catch (const std::exception& e) {
    *out = e.what();
    return kInternal;
  }
}

int ConfigCore::handle(const std::string& method, const std::string& req, std::string* out) {
  requests_++;
  // a mutation's reply: success, or the follower's "Not Leader" + hint, or an INTERNAL status
  auto simple = [&](auto resp, const Result& r) -> int {
    if (r.code == 2) return (*out = r.payload, kInternal);
    resp.success = r.code == 0;
    if (r.code == 1) {
      resp.error_message = "Not Leader";
      resp.leader_hint = r.payload;
    }
    *out = resp.str();
    return kOk;
  };
  if (method == "FetchShardMap") {
    raft::Node* node = node_.load();
    Result r{1, ""};
    if (node) {
      auto prom = std::make_shared<std::promise<Result>>();
      auto fut = prom->get_future();
      node->read_index([prom](int code, const std::string& payload) { prom->set_value(Result{code, payload}); });
      if (fut.wait_for(std::chrono::seconds(10)) != std::future_status::ready) return (*out = "ReadIndex timed out", kUnavailable);
      r = fut.get();
    }
    if (r.code == 1) return (*out = "Not Leader|" + r.payload, kFailedPrecondition);
    if (r.code != 0) return (*out = r.payload, kInternal);
    pb::FetchShardMapResponse resp;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& sid : map_.shards()) {
        const auto* p = map_.peers(sid);
        if (p) resp.shards[sid].peers = *p;
        else resp.shards[sid];
      }
      if (map_.strategy() == ShardMap::Strategy::Range) resp.ranges = map_.ranges();
    }
    *out = resp.str();
    return kOk;
  }
  if (method == "AddShard") {
    pb::AddShardRequest q;
    if (!q.decode(req)) return (*out = "malformed AddShardRequest", kInternal);
    Json a = Json::object();
    a.set("shard_id", q.shard_id);
    a.set("peers", jstrings(q.peers));
    return simple(pb::AddShardResponse{}, propose("AddShard", a));
  }
  if (method == "RemoveShard") {
    pb::RemoveShardRequest q;
    if (!q.decode(req)) return (*out = "malformed RemoveShardRequest", kInternal);
    Json a = Json::object();
    a.set("shard_id", q.shard_id);
    return simple(pb::RemoveShardResponse{}, propose("RemoveShard", a));
  }
  if (method == "RebalanceShard") {
    pb::RebalanceShardRequest q;
    if (!q.decode(req)) return (*out = "malformed RebalanceShardRequest", kInternal);
    Json a = Json::object();
    a.set("old_key", q.old_key);
    a.set("new_key", q.new_key);
    return simple(pb::RebalanceShardResponse{}, propose("RebalanceShard", a));
  }
  if (method == "SplitShard") {
    pb::SplitShardRequest q;
    if (!q.decode(req)) return (*out = "malformed SplitShardRequest", kInternal);
    pb::SplitShardResponse resp;
    // without explicit peers: standby masters first, else the three most recently
    // heartbeated masters (the reference's choice)
    std::vector<std::string> peers = q.new_shard_peers.empty() ? split_candidates(3) : q.new_shard_peers;
    if (peers.empty()) {
      resp.error_message = "No available master nodes for new shard";
      *out = resp.str();
      return kOk;
    }
    Json a = Json::object();
    a.set("shard_id", q.shard_id);
    a.set("split_key", q.split_key);
    a.set("new_shard_id", q.new_shard_id);
    a.set("new_shard_peers", jstrings(peers));
    Result r = propose("SplitShard", a);
    if (r.code == 0 && r.payload != "true") {
      resp.error_message = "split rejected by the shard map";
      *out = resp.str();
      return kOk;
    }
    if (r.code == 0) resp.new_shard_peers = peers;
    return simple(resp, r);
  }
  if (method == "MergeShard") {
    // the apply result decides: two idle neighbours may try to merge into each other
    pb::MergeShardRequest q;
    if (!q.decode(req)) return (*out = "malformed MergeShardRequest", kInternal);
    Json a = Json::object();
    a.set("victim_shard_id", q.victim_shard_id);
    a.set("retained_shard_id", q.retained_shard_id);
    Result r = propose("MergeShard", a);
    if (r.code == 0 && r.payload != "true") {
      pb::MergeShardResponse resp;
      resp.error_message = "merge rejected: unknown shard";
      *out = resp.str();
      return kOk;
    }
    return simple(pb::MergeShardResponse{}, r);
  }
  if (method == "RegisterMaster") {
    pb::RegisterMasterRequest q;
    if (!q.decode(req)) return (*out = "malformed RegisterMasterRequest", kInternal);
    Json a = Json::object();
    a.set("address", q.address);
    a.set("shard_id", q.shard_id);
    Result r = propose("RegisterMaster", a);
    if (r.code == 2) return (*out = r.payload, kInternal);
    pb::RegisterMasterResponse resp;
    resp.success = r.code == 0;
    *out = resp.str();
    return kOk;
  }
  if (method == "ShardHeartbeat") {
    pb::ShardHeartbeatRequest q;
    if (!q.decode(req)) return (*out = "malformed ShardHeartbeatRequest", kInternal);
    pb::ShardHeartbeatResponse resp;
    raft::Node* node = node_.load();
    if (node && node->is_leader()) {
      Json rps = Json::object();
      for (const auto& kv : q.rps_per_prefix) rps.set(kv.first, Json(kv.second));
      Json a = Json::object();
      a.set("address", q.address);
      a.set("rps_per_prefix", rps);
      Json inner = Json::object();
      inner.set("ShardHeartbeat", a);
      Json cmd = Json::object();
      cmd.set("Config", inner);
      node->propose_nowait(cmd.dump());
      resp.success = true;
    }
    *out = resp.str();
    return kOk;
  }
  *out = "method not implemented: " + method;
  return kUnimplemented;
}

}  // namespace dfs
