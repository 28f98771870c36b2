#include "config_core.h"

#include <algorithm>
#include <chrono>

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

}  // namespace dfs
