// Native ChunkServer control loop (C41/C43; reference dfs/chunkserver/src/bin/chunkserver.rs
// :144-355 for the heartbeat and command dispatch, chunkserver.rs:353-718 for recovery, EC
// reconstruction and the scrubber). It replaces the Python heartbeat/command/recovery code
// of tests/models/chunkserver_shell.py + chunkserver_service.py when the native fast path is up:
//
//   heartbeat thread  every `heartbeat_ms`: FetchShardMap from the config servers (masters =
//                     every shard's peers, else the static list), then HeartbeatRequest
//                     (disk + HBM stats and the pending reports) to every master; adopt
//                     master_term; hand the returned commands to the job pool.
//   scrub thread      every `scrub_ms`: the store's batched scrub (K1b on the GPU); bad blocks
//                     are reported on the next heartbeat and recovered.
//   jobs              REPLICATE   the replication engine for same-node targets (HBM -> HBM,
//                                 FastPathServer::replicate_block), gRPC ReplicateBlock{heal}
//                                 otherwise;
//                     RECONSTRUCT_EC_SHARD  parallel ReadBlock of the survivors, GF(2^8)
//                                 decode on the GPU (CPU codec without one), local write;
//                     ENCODE_EC   RS encode of the verified local replica, k+m shard writes
//                                 in parallel (tiering, C32);
//                     DELETE / MOVE_TO_COLD  store operations;
//                     recovery    of a corrupt block: ReadBlock from another holder, checked
//                                 against OUR .meta (reference: the replica must match what
//                                 we were given), rewritten.
// Reports (bad / new / EC encoded / failed / rebuilt) are queued here; the Python gRPC
// fallback paths that still produce some push them through report_*().
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "chunk_store.h"
#include "dfs_pb.h"
#include "fastpath.h"
#include "grpc_client.h"
#include "io_pool.h"

namespace dfs {

class TlsContext;

struct CsAgentConfig {
  std::string advertise;     // host:port this chunkserver is known by
  std::string rack_id;
  std::string storage_dir;   // for the disk-space figures
  int gpu_rank = -1;
  std::vector<std::string> masters;         // static master list (no config server)
  std::vector<std::string> config_servers;  // FetchShardMap sources
  int heartbeat_ms = 5000;
  int scrub_ms = 60000;
  int rpc_timeout_ms = 60000;
  bool tls = false;          // masters / peers are https:// targets
};

struct CsAgentStats {
  uint64_t heartbeats = 0, heartbeat_failures = 0, commands = 0, map_refreshes = 0;
  uint64_t replicate_engine = 0, replicate_grpc = 0, replicate_failed = 0;
  uint64_t reconstructs = 0, reconstruct_failed = 0, encodes = 0, encode_failed = 0;
  uint64_t reconstruct_device = 0;  // of the reconstructs: gathered into HBM and decoded there
  uint64_t recoveries = 0, recovery_failed = 0, deletes = 0, moves = 0, scrubs = 0, scrub_bad = 0;
  uint64_t ec_gpu = 0, ec_cpu = 0;
};

class CsAgent {
 public:
  CsAgent(CsAgentConfig cfg, ChunkStore* store, FastPathServer* fp, std::shared_ptr<TlsContext> tls);
  ~CsAgent();
  CsAgent(const CsAgent&) = delete;

  void start();
  void stop();

  // One heartbeat round now (tests, and the first round at start).
  void heartbeat_once();
  // One scrub pass now: bad blocks are reported and queued for recovery.
  std::vector<std::string> scrub_once();
  // Synchronous recovery of a corrupt block (the read paths retry after it); "" = recovered.
  std::string recover(const std::string& block_id);
  void queue_recovery(const std::string& block_id);
  // A command as the master sent it (serialized ChunkServerCommand); runs on the job pool.
  void submit_command(const std::string& cmd_pb);

  // Reports from the Python fallback paths.
  void report_new_block(const std::string& id);
  void report_bad_block(const std::string& id);

  std::vector<std::string> masters();
  uint64_t known_term();
  CsAgentStats stats();

 private:
  void heartbeat_loop();
  void scrub_loop();
  bool refresh_masters();
  void dispatch(const pb::ChunkServerCommand& c);
  bool replicate_to(const std::string& block_id, const std::string& target);
  bool reconstruct(const pb::ChunkServerCommand& c);
  bool encode_ec(const pb::ChunkServerCommand& c);
  std::vector<std::string> block_locations(const std::string& block_id);
  bool read_local(const std::string& id, std::vector<uint8_t>* out);
  bool gf_product(const std::vector<std::vector<uint8_t>>& mat, const std::vector<const uint8_t*>& in,
                  const std::vector<uint8_t*>& out, uint64_t len);
  std::string target(const std::string& addr) const;
  bool is_me(const std::string& addr) const;
  void adopt(uint64_t term);

  CsAgentConfig cfg_;
  ChunkStore* store_;
  FastPathServer* fp_;
  GrpcChannelPool pool_;
  std::atomic<uint64_t> term_{0};  // without a fast path

  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::vector<std::string> masters_;  // from the shard map (or cfg_.masters)
  std::vector<std::string> bad_, new_, enc_, fail_, rebuilt_;
  std::vector<std::string> recovering_;  // block ids with a recovery queued or running
  // the masters' DELETE commands, drained by at most kDeleteWorkers jobs (a heartbeat can
  // carry thousands after an overwrite-heavy burst; one job each grew the pool to as many
  // threads)
  std::deque<std::string> del_q_;
  int del_workers_ = 0;
  static constexpr int kDeleteWorkers = 8;
  CsAgentStats st_;
  std::thread hb_, scrub_;
  IoPool jobs_{8, 30000, "cs-jobs"};  // last: destroyed first, after its jobs finished
};

}  // namespace dfs
