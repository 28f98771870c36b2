// Native metadata master of one namespace shard: the replicated state machine (C24, C26)
// and the hot MasterService handlers (C33) — GetFileInfo, CreateFile, AllocateBlock,
// CompleteFile, ListFiles, DeleteFile, GetBlockLocations — served straight from C++,
// with rack/GPU-aware placement (C28) and the Raft node (raft.h) underneath.
//
// Reference: dfs/metaserver/src/master.rs:195-367 (state, safe mode), :378-432
// (placement), :2141-2560 (handlers), :2684-2723 (GetBlockLocations), and the command
// semantics of simple_raft.rs:2995-3398. Behaviour differences, all client-compatible:
//   * a block_id -> path index makes GetBlockLocations O(1) (reference: linear scan);
//   * files are invisible until CompleteFile, and CreateFile/Rename decide existence at
//     apply time, so racing writers cannot both succeed (linearizability);
//   * paths pinned by an unresolved cross-shard rename make readers and writers wait;
//   * access statistics (the reference's Raft write per GetFileInfo) are batched into one
//     UpdateAccessStatsBatch entry per second;
//   * a deferred create places the block without a Raft entry and creates the file in
//     CompleteFile{create=true}: one Raft entry (one WAL fdatasync) per write.
// Status codes and message strings match the reference (REDIRECT:, Not Leader|, safe mode).
//
// Threading: the state lives under one mutex. Raft applies on its applier thread; RPCs
// run on the callers' threads (native local-RPC connections, or gRPC workers through the
// Python binding) and block only on Raft completions, never while holding the mutex.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dfs_pb.h"
#include "grpc_client.h"
#include "json.h"
#include "raft.h"
#include "shard_map.h"

namespace dfs {

struct ChunkServerStatus {
  std::string address;
  int64_t last_heartbeat = 0;
  uint64_t used_space = 0, available_space = 0, chunk_count = 0;
  std::string rack_id;
  int32_t gpu_rank = -1;
  uint64_t hbm_capacity = 0, hbm_used = 0;
  uint64_t scheduled = 0;  // bytes placed here since the last heartbeat (local only)
};

// Rack-aware round robin by free space (reference master.rs:378-432); `preferred` (the
// writer-local chunkserver) is pinned first when live.
std::vector<std::string> select_servers_rack_aware(const std::vector<ChunkServerStatus>& servers, size_t n,
                                                   const std::string& preferred);

// The serde layout of FileMetadata / BlockInfo that Raft commands carry (IngestBatch,
// ConvertToEc, transaction records; models/meta.py file_to_dict / block_to_dict).
Json file_meta_json(const pb::FileMetadata& m);
Json block_info_json(const pb::BlockInfo& b);

class MasterCore : public raft::StateMachine {
 public:
  enum Code { OK = 0, NOT_FOUND = 5, FAILED_PRECONDITION = 9, INTERNAL = 13, UNAVAILABLE = 14, OUT_OF_RANGE = 11,
              UNIMPLEMENTED = 12 };

  MasterCore();
  ~MasterCore() override;

  void attach(raft::Node* node);  // the Raft node proposals go to
  void detach();

  // raft::StateMachine
  std::vector<std::string> apply(const std::vector<std::pair<uint64_t, std::string>>& cmds) override;
  std::string snapshot() override;
  void restore(const std::string& state) override;

  // Hot RPCs: `method` is the bare MasterService method name. Returns a gRPC status code;
  // *out holds the serialized response (OK) or the status message, or kDecline: the request
  // is one this core does not serve (a cross-shard Rename, which is the Python
  // coordinator's 2PC) and goes to the fallback handler unchanged.
  static constexpr int kDecline = -100;
  bool native_method(const std::string& method) const;
  int handle(const std::string& method, const std::string& req, std::string* out);

  // Routing: the shard map (JSON, ShardMap serde layout) and this master's shard id.
  void set_shard_map(const std::string& json, const std::string& shard_id);
  // The map was just fetched from the config servers. With a max age set (> 0), a Rename
  // decides same-shard vs 2PC natively only while the map is younger than that; otherwise it
  // is declined to the Python handler, which refreshes the map first (master/service.py).
  void note_shard_map_fresh();
  void set_shard_map_max_age(int64_t ms);

  // Chunkserver registry (local, rebuilt from heartbeats).
  void upsert_chunk_server(const ChunkServerStatus& st);
  bool remove_chunk_server(const std::string& addr);
  std::vector<ChunkServerStatus> chunk_servers() const;

  // Safe mode (reference master.rs:258-367).
  void enter_safe_mode(bool manual);
  void exit_safe_mode();
  bool should_exit_safe_mode() const;
  void report_blocks(uint64_t n);  // + reported blocks, auto-exit when due
  Json safe_mode_status() const;

  // Chunkserver commands (local, not replicated): queued by the healer / balancer / tiering
  // (Python, serialized ChunkServerCommand) and by GC, handed out by the native Heartbeat.
  void queue_command(const std::string& addr, const std::string& cmd);
  std::vector<std::string> take_commands(const std::string& addr);
  std::map<std::string, std::vector<std::string>> peek_commands() const;
  // What heartbeats reported for the Python background tasks: blocks that failed
  // verification (block -> servers), EC conversions done / failed, and whether a heal pass
  // is due (a bad block arrived since the last call).
  std::map<std::string, std::vector<std::string>> bad_blocks() const;
  void add_bad_block(const std::string& block_id, const std::string& addr);
  std::pair<std::vector<std::string>, std::vector<std::string>> take_ec_reports();
  bool take_heal_request();

  // Queries for the Python services (serialized FileMetadata / JSON).
  bool get_file(const std::string& path, bool visible_only, std::string* pb) const;
  bool contains(const std::string& path) const;
  bool under_construction(const std::string& path) const;
  size_t file_count() const;
  std::vector<std::string> paths(const std::string& prefix, bool visible_only) const;
  std::vector<std::string> files_pb(const std::string& prefix) const;
  bool find_block(const std::string& block_id, std::string* file_pb) const;
  bool has_block(const std::string& block_id) const;
  uint64_t total_blocks() const;
  std::string tx_record(const std::string& tx_id) const;  // "" if absent
  std::string tx_records() const;                          // JSON object
  std::string tx_lock(const std::string& path) const;      // tx id or ""
  std::vector<std::string> shuffling_prefixes() const;

  // Drained by the Python side: per-prefix request counts (dynamic sharding monitor) and
  // blocks no file references any more (DELETE commands for their holders).
  std::map<std::string, uint64_t> take_request_counts();
  std::vector<std::pair<std::string, std::vector<std::string>>> take_gc();

  // Healer scan (C29, reference master.rs:436-602) over the whole namespace in one pass under
  // the lock: REPLICATE for replicated blocks short of min(rf, live) healthy copies (queued on
  // the first healthy holder), RECONSTRUCT_EC_SHARD for EC shards on dead servers (queued on
  // the target) while >= k shards survive. `live` sorted; `bad` = block -> servers whose copy
  // failed verification; `queued` = (block, target) already pending anywhere (counted as
  // copies on their way, and never queued twice).
  struct HealAction {
    bool reconstruct = false;
    std::string queue_on, block_id, target;
    int shard_index = -1, ec_data = 0, ec_parity = 0;
    std::vector<std::string> sources;  // reconstruct: per shard index, "" where dead
    uint64_t original_size = 0;
  };
  std::vector<HealAction> heal_scan(int rf, const std::vector<std::string>& live,
                                    const std::map<std::string, std::vector<std::string>>& bad,
                                    const std::set<std::pair<std::string, std::string>>& queued) const;

  // Balancer / shuffler pick (reference master.rs:1033-1120): a replicated block held by `src`
  // and not by `dst`, under `prefix` when given; "" if none. One pass under the lock.
  std::string pick_block(const std::string& src, const std::string& dst, const std::string* prefix) const;
  // Tiering scan (C32, reference master.rs:1990-2060): files idle for longer than cold_ms that
  // are neither cold nor EC yet, with each block's holders (MOVE_TO_COLD targets).
  struct ColdFile {
    std::string path;
    std::vector<std::pair<std::string, std::vector<std::string>>> blocks;  // block id, locations
  };
  std::vector<ColdFile> tiering_scan(uint64_t now_ms, uint64_t cold_ms) const;
  // EC conversion candidates: cold, replicated, non-empty files cold for longer than ec_ms
  // (encoded FileMetadata, only those — the caller decodes a handful, not the namespace).
  std::vector<std::string> ec_candidates(uint64_t now_ms, uint64_t ec_ms) const;

  // Cross-shard Rename as a native 2PC coordinator (reference master.rs:2562-2683 rename,
  // :2724-2900 participant handlers). `call` is a unary gRPC call to a peer master (the
  // bindings pass a GrpcChannelPool, tests wire two cores together); without it a
  // cross-shard Rename is declined to the Python coordinator.
  using PeerCall = std::function<GrpcResult(const std::string& target, const std::string& path,
                                            const std::string& req, int timeout_ms)>;
  void enable_native_2pc(PeerCall call);
  Json txn_stats() const;

  // Raft peer RPC (vote / append / snapshot / timeout_now, JSON) for the attached node, as
  // served by the native gRPC server on /dfs.RaftPeer/<kind>.
  int raft_rpc(const std::string& kind, const std::string& body, std::string* out);

  void set_access_stats(bool on, int flush_ms);
  uint64_t requests() const { return requests_.load(); }
  uint64_t heartbeats() const { return heartbeats_.load(); }

 private:
  struct Result {  // of a proposal
    int code;      // 0 ok, 1 not leader (payload = hint), 2 error
    std::string payload;
  };
  Result propose(const Json& cmd);
  Result propose_unlocked(const std::string& name, const Json& args);  // waits out tx pins
  std::vector<Result> propose_all(const std::vector<Json>& cmds);       // queued back to back
  int read_index(std::string* err);
  bool wait_unlocked(const std::string& path, int timeout_ms, std::string* err);
  int check_ownership(const std::string& path, std::string* err) const;
  bool place(int ec_d, int ec_p, const std::string& preferred, std::vector<std::string>* out, std::string* err);
  void allocation(const std::string& block_id, const std::vector<std::string>& sel, int ec_d, int ec_p,
                  pb::AllocateBlockResponse* a) const;
  void record_request(const std::string& path);
  void record_access(const std::string& path);
  void access_loop();
  void queue_gc(const Json& blocks);  // [[block_id, [locations]]...]
  std::string new_uuid();

  int get_file_info(const std::string& req, std::string* out);
  int create_file(const std::string& req, std::string* out);
  int allocate_block(const std::string& req, std::string* out);
  int complete_file(const std::string& req, std::string* out);
  int list_files(const std::string& req, std::string* out);
  int delete_file(const std::string& req, std::string* out);
  int rename(const std::string& req, std::string* out);
  int get_block_locations(const std::string& req, std::string* out);
  int heartbeat(const std::string& req, std::string* out);
  int register_chunk_server(const std::string& req, std::string* out);
  int get_safe_mode_status(const std::string& req, std::string* out);
  int set_safe_mode(const std::string& req, std::string* out);
  int rename_2pc(const pb::RenameRequest& r, const std::string& src_shard, const std::string& dst_shard,
                 std::string* out);
  int prepare_transaction(const std::string& req, std::string* out);
  int commit_transaction(const std::string& req, std::string* out);
  int abort_transaction(const std::string& req, std::string* out);
  int inquire_transaction(const std::string& req, std::string* out);
  // Unary call to the leader of a peer shard: each address in turn, following leader hints;
  // true when a reply says success. `decode` parses (success, error_message, leader_hint).
  template <class Resp>
  bool call_peers(const std::vector<std::string>& peers, const std::string& method, const std::string& req);

  // state machine helpers (mu_ held)
  Json apply_one(const std::string& name, const Json& a);
  void put(const std::string& path, pb::FileMetadata m);
  bool del(const std::string& path, pb::FileMetadata* out);
  const pb::FileMetadata* visible(const std::string& path) const;
  pb::BlockInfo* find_block_locked(const std::string& block_id, pb::FileMetadata** file);
  void relock(const Json& rec);

  mutable std::mutex mu_;
  std::condition_variable applied_cv_;
  // replicated
  std::unordered_map<std::string, pb::FileMetadata> files_;
  // the same paths in order (kept by put / del / restore): prefix listings walk
  // [lower_bound(prefix), first path without it) instead of scanning every file under mu_
  std::set<std::string> ordered_;
  template <class F>
  void for_prefix(const std::string& prefix, F&& f) const {
    for (auto it = ordered_.lower_bound(prefix); it != ordered_.end() && it->compare(0, prefix.size(), prefix) == 0;
         ++it)
      f(*it);
  }
  std::unordered_map<std::string, std::string> block_index_;
  // path -> writer generation (the create entry's ts) while a classic create is open, and the
  // last progress (create / AllocateBlock) of that writer: the lease runs from the latter.
  std::unordered_map<std::string, int64_t> under_construction_;
  std::unordered_map<std::string, int64_t> uc_progress_;
  std::map<std::string, Json> tx_records_;
  std::unordered_map<std::string, std::string> tx_locks_;
  std::set<std::string> shuffling_prefixes_;
  // local
  std::map<std::string, ChunkServerStatus> chunk_servers_;
  bool safe_mode_ = false, safe_mode_manual_ = false;
  int64_t safe_mode_entered_at_ = 0;
  uint64_t expected_blocks_ = 0, reported_blocks_ = 0;
  double safe_mode_threshold_ = 0.99;
  ShardMap shard_map_;
  std::string shard_id_;
  bool have_map_ = false;
  int64_t map_fresh_ms_ = 0;    // mu_: steady-clock ms of the last note_shard_map_fresh()
  int64_t map_max_age_ms_ = 0;  // mu_: 0 = no freshness requirement (no config servers)
  std::atomic<uint64_t> stale_map_declines_{0};
  std::map<std::string, uint64_t> request_counts_;
  std::map<std::string, std::vector<std::string>> cmd_q_;        // addr -> serialized commands
  std::map<std::string, std::set<std::string>> bad_blocks_;      // block -> reporting servers
  std::vector<std::string> ec_encoded_, ec_failed_;
  bool heal_req_ = false;
  std::vector<std::pair<std::string, std::vector<std::string>>> gc_;
  std::map<std::string, uint64_t> access_buf_;
  bool access_stats_ = true;
  int access_flush_ms_ = 1000;
  std::mt19937_64 rng_;

  // native 2PC coordinator (enable_native_2pc); at most kMaxCoordinators renames hold an
  // RPC worker while they wait on the peer shard (a quarter of the master's 64 native gRPC
  // workers, so participant calls always find one), the rest go to the Python coordinator
  static constexpr int kMaxCoordinators = 16;
  PeerCall peer_call_;  // set once before serving
  std::atomic<int> coordinators_{0};
  std::atomic<uint64_t> tx_started_{0}, tx_committed_{0}, tx_aborted_{0}, tx_pending_{0}, tx_declined_{0};

  std::atomic<raft::Node*> node_{nullptr};
  std::atomic<uint64_t> requests_{0}, heartbeats_{0};
  std::atomic<bool> running_{true};
  std::condition_variable access_cv_;
  std::thread access_thread_;
};

}  // namespace dfs
