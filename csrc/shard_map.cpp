#include "shard_map.h"

#include "crc32.h"

namespace dfs {

namespace {
const std::string kMaxKey = "\xF4\x8F\xBF\xBF";  // U+10FFFF in UTF-8

uint32_t hash_key(const std::string& s) { return crc32(reinterpret_cast<const uint8_t*>(s.data()), s.size()); }
}  // namespace

ShardMap ShardMap::new_range() {
  ShardMap m;
  m.strategy_ = Strategy::Range;
  return m;
}

ShardMap ShardMap::new_consistent_hash(int virtual_nodes) {
  ShardMap m;
  m.strategy_ = Strategy::ConsistentHash;
  m.virtual_nodes_ = virtual_nodes;
  return m;
}

ShardMap ShardMap::from_json(const Json& j) {
  const Json& strat = j["strategy"];
  ShardMap m;
  if (const Json* r = strat.find("Range")) {
    m.strategy_ = Strategy::Range;
    for (auto& kv : (*r)["ranges"].fields()) m.ranges_[kv.first] = kv.second.str();
  } else {
    const Json& ch = strat["ConsistentHash"];
    m.strategy_ = Strategy::ConsistentHash;
    m.virtual_nodes_ = static_cast<int>(ch["virtual_nodes"].as_int(100));
    for (auto& kv : ch["ring"].fields()) m.ring_[static_cast<uint32_t>(std::stoul(kv.first))] = kv.second.str();
  }
  for (auto& s : j["shards"].items()) m.shards_.insert(s.str());
  for (auto& kv : j["shard_peers"].fields()) {
    std::vector<std::string> p;
    for (auto& a : kv.second.items()) p.push_back(a.str());
    m.peers_[kv.first] = p;
  }
  return m;
}

Json ShardMap::to_json() const {
  Json strat = Json::object(), inner = Json::object();
  if (strategy_ == Strategy::Range) {
    Json r = Json::object();
    for (auto& kv : ranges_) r.set(kv.first, kv.second);
    inner.set("ranges", r);
    strat.set("Range", inner);
  } else {
    Json r = Json::object();
    for (auto& kv : ring_) r.set(std::to_string(kv.first), kv.second);
    inner.set("ring", r);
    inner.set("virtual_nodes", virtual_nodes_);
    strat.set("ConsistentHash", inner);
  }
  Json out = Json::object(), shards = Json::array(), peers = Json::object();
  for (auto& s : shards_) shards.push_back(s);
  for (auto& kv : peers_) {
    Json a = Json::array();
    for (auto& p : kv.second) a.push_back(p);
    peers.set(kv.first, a);
  }
  out.set("strategy", strat);
  out.set("shards", shards);
  out.set("shard_peers", peers);
  return out;
}

void ShardMap::add_shard(const std::string& id, const std::vector<std::string>& peers) {
  peers_[id] = peers;
  if (!shards_.insert(id).second) return;
  if (strategy_ == Strategy::ConsistentHash) {
    for (int i = 0; i < virtual_nodes_; ++i) ring_[hash_key(id + ":" + std::to_string(i))] = id;
  } else if (ranges_.empty()) {
    ranges_[kMaxKey] = id;
  } else if (ranges_.size() == 1) {
    // order-dependent bootstrap (reference sharding.rs:99-106): the SECOND shard takes <= "/m"
    std::string old = ranges_.begin()->second;
    ranges_.clear();
    ranges_["/m"] = id;
    ranges_[kMaxKey] = old;
  } else {
    ranges_["z-" + id] = id;
  }
}

void ShardMap::remove_shard(const std::string& id) {
  if (!shards_.erase(id)) return;
  peers_.erase(id);
  for (auto it = ring_.begin(); it != ring_.end();) it = it->second == id ? ring_.erase(it) : std::next(it);
  for (auto it = ranges_.begin(); it != ranges_.end();) it = it->second == id ? ranges_.erase(it) : std::next(it);
}

bool ShardMap::split_shard(const std::string& split_key, const std::string& new_id,
                           const std::vector<std::string>& peers) {
  if (strategy_ != Strategy::Range || shards_.count(new_id) || ranges_.count(split_key)) return false;
  if (ranges_.lower_bound(split_key) == ranges_.end()) return false;
  ranges_[split_key] = new_id;
  shards_.insert(new_id);
  peers_[new_id] = peers;
  return true;
}

bool ShardMap::merge_shards(const std::string& victim, const std::string& retained) {
  if (strategy_ != Strategy::Range || !shards_.count(victim) || !shards_.count(retained)) return false;
  auto vk = ranges_.end();
  for (auto it = ranges_.begin(); it != ranges_.end(); ++it)
    if (it->second == victim) {
      vk = it;
      break;
    }
  if (vk == ranges_.end()) return false;
  bool was_max = vk->first == kMaxKey;
  ranges_.erase(vk);
  if (was_max) {
    for (auto it = ranges_.begin(); it != ranges_.end(); ++it)
      if (it->second == retained) {
        ranges_.erase(it);
        break;
      }
    ranges_[kMaxKey] = retained;
  }
  shards_.erase(victim);
  peers_.erase(victim);
  return true;
}

bool ShardMap::rebalance_boundary(const std::string& old_key, const std::string& new_key) {
  auto it = ranges_.find(old_key);
  if (strategy_ != Strategy::Range || it == ranges_.end()) return false;
  std::string shard = it->second;
  ranges_.erase(it);
  ranges_[new_key] = shard;
  return true;
}

std::string ShardMap::get_shard(const std::string& key) const {
  if (strategy_ == Strategy::ConsistentHash) {
    if (ring_.empty()) return "";
    auto it = ring_.lower_bound(hash_key(key));
    return it == ring_.end() ? ring_.begin()->second : it->second;
  }
  auto it = ranges_.lower_bound(key);
  return it == ranges_.end() ? std::string() : it->second;
}

const std::vector<std::string>* ShardMap::peers(const std::string& shard) const {
  auto it = peers_.find(shard);
  return it == peers_.end() ? nullptr : &it->second;
}

}  // namespace dfs
