// Namespace sharding map (C04, P1/P2), native twin of parallel/sharding.py. Routing must
// agree bit for bit with the reference because clients and servers compute it
// independently (reference: dfs/common/src/sharding.rs:17-341):
//   * ConsistentHash: CRC32("{shard}:{i}") for `virtual_nodes` vnodes on a ring; a key maps
//     to the first vnode >= CRC32(key), wrapping around;
//   * Range: inclusive range END key -> shard; a key maps to the first end >= key
//     (BTreeMap::range(key..)). UTF-8 byte order equals code-point order, so std::string
//     comparison matches Python's str ordering.
// The JSON form is the reference's serde layout.
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "json.h"

namespace dfs {

class ShardMap {
 public:
  enum class Strategy { ConsistentHash, Range };

  static ShardMap new_range();
  static ShardMap new_consistent_hash(int virtual_nodes = 100);
  static ShardMap from_json(const Json& j);
  Json to_json() const;

  void add_shard(const std::string& id, const std::vector<std::string>& peers);
  void remove_shard(const std::string& id);
  bool split_shard(const std::string& split_key, const std::string& new_id, const std::vector<std::string>& peers);
  bool merge_shards(const std::string& victim, const std::string& retained);
  bool rebalance_boundary(const std::string& old_key, const std::string& new_key);

  // Owning shard of `key`; empty when the map has no shards.
  std::string get_shard(const std::string& key) const;
  const std::vector<std::string>* peers(const std::string& shard) const;
  bool has_shard(const std::string& id) const { return shards_.count(id) != 0; }
  std::vector<std::string> shards() const { return {shards_.begin(), shards_.end()}; }
  Strategy strategy() const { return strategy_; }
  const std::map<std::string, std::string>& ranges() const { return ranges_; }

 private:
  Strategy strategy_ = Strategy::Range;
  int virtual_nodes_ = 100;
  std::map<uint32_t, std::string> ring_;
  std::map<std::string, std::string> ranges_;  // end key -> shard
  std::set<std::string> shards_;
  std::map<std::string, std::vector<std::string>> peers_;
};

}  // namespace dfs
