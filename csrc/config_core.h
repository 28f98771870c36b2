// Native config-server state machine (C36): the Raft-replicated shard map and master
// registry of the reference's ConfigService (dfs/metaserver/src/config_server.rs,
// simple_raft.rs ConfigCommand apply). Applied on the native Raft applier thread like
// MasterCore. The ConfigService RPCs are answered here too (handle(): every method of the
// reference's config_server.rs, served by the native HTTP/2 server and the local socket),
// so a config server runs no Python on any request; Python keeps process setup and the
// /metrics and /shards HTTP views.
//
// Commands (externally tagged JSON, {"Config": {"<Name>": {...}}}):
//   AddShard{shard_id, peers}  RemoveShard{shard_id}
//   SplitShard{shard_id, split_key, new_shard_id, new_shard_peers} -> true/false
//   MergeShard{victim_shard_id, retained_shard_id} -> true/false
//   RebalanceShard{old_key, new_key} -> true/false
//   RegisterMaster{address, shard_id}   (empty shard_id = standby master)
//   ShardHeartbeat{address, rps_per_prefix}
// Snapshot: {"Config": {"shard_map": <ShardMap serde>, "masters": {addr: MasterInfo}}}.
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "json.h"
#include "raft.h"
#include "shard_map.h"

namespace dfs {

class ConfigCore : public raft::StateMachine {
 public:
  ConfigCore();

  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) override;
  std::string snapshot() override;
  void restore(const std::string& state) override;

  // Views for the service layer (thread-safe copies).
  std::string shard_map_json() const;
  std::string masters_json() const;
  uint64_t version() const;
  // Peers for a split without explicit ones: standby masters (registered without a shard)
  // by most recent heartbeat, else the three most recently heartbeated masters.
  std::vector<std::string> split_candidates(size_t n = 3) const;

  // ConfigService: `method` is the bare method name; returns a gRPC status code with the
  // serialized response (OK) or the status message in *out.
  void attach(raft::Node* node) { node_ = node; }
  void detach() { node_ = nullptr; }
  static bool native_method(const std::string& method);
  int handle(const std::string& method, const std::string& req, std::string* out);
  // Raft peer RPC (vote / append / snapshot / timeout_now, JSON) for /dfs.RaftPeer/<kind>.
  int raft_rpc(const std::string& kind, const std::string& body, std::string* out);
  uint64_t requests() const { return requests_.load(); }

 private:
  struct Result {  // of a proposal: 0 applied (payload = apply result), 1 not leader (hint), 2 error
    int code;
    std::string payload;
  };
  Result propose(const std::string& name, const Json& args);
  struct MasterInfo {
    std::string shard_id;
    int64_t last_heartbeat = 0;  // unix seconds
    Json rps = Json::object();
  };
  Json apply_one(const Json& cmd);
  Json snapshot_locked() const;

  mutable std::mutex mu_;
  ShardMap map_;
  std::map<std::string, MasterInfo> masters_;
  uint64_t version_ = 0;
  std::atomic<raft::Node*> node_{nullptr};
  std::atomic<uint64_t> requests_{0};
};

}  // namespace dfs
