// Native local data path of a ChunkServer ("fast path").
//
// HDFS serves co-located readers through UNIX domain sockets + shared memory
// (short-circuit local reads). This is the same idea for both directions, handled
// entirely in C++: a client on the same host puts a block into its /dev/shm arena slot
// and sends a ~100-byte request over an abstract UNIX socket; the server thread stages
// it into HBM (H2D DMA + CDNA4 CRC kernel), persists it and answers — no Python, no GIL,
// no HTTP/2 framing on the ChunkServer side. Reads DMA the verified range from HBM
// straight into the client's slot.
//
// Scope: WriteBlock (locally, and along same-node RCCL chains) and ReadBlock. Anything
// else — cross-node hops, corruption needing recovery, fenced or malformed requests — is
// answered with a status telling the client to use the regular gRPC service, which keeps
// every semantic of the reference (fencing, recovery, replicas_written) in one place.
//
// Wire format (little endian), one request/response pair at a time per connection:
//   request  = u32 body_len | u8 op | body
//     op 1 WRITE: u64 term | u32 crc | u64 shm_off | u64 len | u16 id_len id | u16 path_len path
//               [| u16 n_next | (u16 len addr)*]      -- replicas, fanned out natively
//     op 2 READ : u64 offset | u64 length | u64 shm_off | u64 shm_cap | u16 id_len id | u16 path_len path
//     op 3 REPL : u64 term | u32 crc | i32 src_rank | u64 gen | i64 seq | u64 size | u64 slice
//               | u16 id_len id | u16 n_next | (u16 len addr)*   -- payload over the P2P transport
//     op 4 REPL_SHM: u64 term | u32 crc | u64 shm_off | u64 len | u16 id_len id | u16 path_len path
//               | u16 n_next | (u16 len addr)*      -- same-host hop without a P2P pair: read the client slot
//     op 5 CTRL : u16 len blob                       -- replication control (pair bring-up / rebuild)
//     op 6 EC   : u16 k | u16 rows | u64 len | u64 in_off | u64 out_off | u16 rows*k matrix | u16 path
//               [| u16 rid]  -- GF(2^8) matrix x shards (RS encode / reconstruct) on this GPU;
//               shards sit in the client's slot at 16-byte-aligned strides, outputs land there
//     op 7 EC_WRITE: u64 term | u16 k | u16 m | u64 shard_len | u64 shm_off | u64 shm_stride | u16 id
//               | u16 path | u16 n | (u16 len addr)* (k + m targets) [| u16 rid]
//               -- device-resident RS write: the k stripes go up once, parity is computed in
//               HBM, every shard is checksummed there and scattered HBM -> HBM over the engine
//     op 8 EC_READ: u64 offset | u64 length | u16 k | u16 m | u64 shard_len | u64 orig | u64 shm_off
//               | u64 shm_cap | u16 id | u16 path | u16 n | (u16 len addr)* ("" = lost) [| u16 rid]
//               -- degraded read: surviving shards gathered into this GPU, missing data decoded
//               there, the requested range DMA'd into the client's slot
//     op 9 PUSH: u16 id | u16 as_id | u16 dst_addr [| u16 rid] -- send local block `id` to the
//               same-node peer `dst_addr` over the engine, stored there as ephemeral `as_id`
//   response = u32 body_len | u8 status | u64 total | u64 bytes | u16 msg_len msg
//   (for WRITE/REPL ``bytes`` carries replicas_written; for CTRL ``msg`` is the engine reply)
//
// Replication stays native when every replica is a ChunkServer of this host. The head
// stages the block in HBM (H2D + CRC kernel) and FANS OUT to all replicas at once: over the
// P2P transport (RCCL/xGMI, slices pipelined with the receiver's checksum kernel) where the
// pair is up, else the replica stages straight from the client's shared-memory slot. Each
// path overlaps the local fdatasync. A replica that fails is not counted (replicas_written
// shrinks, like the reference's chain); a replica off this host makes the head answer
// Unsupported and the client redoes the write on the gRPC path.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "chunk_store.h"
#include "io_pool.h"
#include "replication.h"

namespace dfs {

enum class FpStatus : uint8_t {
  Ok = 0,
  NotFound = 1,
  OutOfRange = 2,
  Corrupt = 3,      // use gRPC: the Python service recovers from a replica
  IoError = 4,
  Fenced = 5,       // stale master term
  Unsupported = 6,  // use gRPC
  BadRequest = 7,
  PartialCorrupt = 8,  // data returned; block queued for background recovery
};

struct FpStats {
  uint64_t writes = 0, reads = 0, fenced = 0, punts = 0, connections = 0;
  uint64_t replicas_in = 0, rccl_forwards = 0, shm_forwards = 0, forward_failures = 0;
  uint64_t rejected_peers = 0;  // connections from another uid (SO_PEERCRED)
  uint64_t replica_failures = 0;  // replicas that could not be written (not counted)
  uint64_t p2p_fallbacks = 0;     // replicas moved to shared memory after a P2P failure
  uint64_t ec_ops = 0;            // erasure-coding matrix products run for clients
  uint64_t heals_out = 0, heals_in = 0;  // heal / balancer copies sent / received on the engine
  uint64_t sliced_writes = 0;  // head writes whose replica sends overlapped the staging
  // device-resident erasure coding: EC writes whose shards were encoded and scattered HBM ->
  // HBM, shards forwarded that way, degraded reads / reconstructions gathered into HBM and
  // decoded there, shards pulled for a gather, and requests that had to take the host path
  uint64_t ec_device_writes = 0, ec_shard_forwards = 0, ec_device_reads = 0, ec_device_decodes = 0;
  uint64_t ec_gathered = 0, ec_device_fallbacks = 0;
  // chained head writes (below the sliced size): staging + checksum, then the local persist
  // and replica fan-out together (ns summed); each device forward's descriptor round trip
  // (from its sends being posted to the replica's reply)
  uint64_t chain_writes = 0, chain_stage_ns = 0, chain_forward_ns = 0;
  uint64_t desc_calls = 0, desc_ns = 0;
};

class FastPathServer {
 public:
  FastPathServer(ChunkStore* store, std::string name);
  ~FastPathServer();
  FastPathServer(const FastPathServer&) = delete;
  FastPathServer& operator=(const FastPathServer&) = delete;

  bool start(std::string* err);
  void stop();
  // Abstract-namespace socket name (without the leading NUL), e.g. "dfs_fp_1234_50051".
  const std::string& name() const { return name_; }

  // Epoch fencing shared with the gRPC service: rejects 0 < term < known, adopts higher.
  bool fence(uint64_t term, uint64_t* known);
  void adopt_term(uint64_t term);
  uint64_t term() const { return term_.load(); }

  std::vector<std::string> drain_suspects();  // blocks needing background recovery
  // The request ids of the last few data-path ops served here (newest last): lets tests and
  // operators follow one client request across the head and every replica.
  std::vector<std::string> recent_request_ids();
  FpStats stats();

  // Native replication: this server's engine (RCCL or socket transport) and the fast-path
  // socket of every same-node peer (advertised address -> rank, socket name).
  void set_replication(ReplicationEngine* engine);
  void set_peer(const std::string& addr, int rank, const std::string& fp_name);
  // Control exchange with the fast path of the peer of `rank` (the engine's ControlFn).
  bool control(int rank, const std::string& req, std::string* reply);
  // For the native gRPC service (cs_grpc.cpp): whether every address is a same-host peer
  // this server can replicate to natively; persist a staged block while fanning it out to
  // `next` (the replicas count written downstream); queue a block for background recovery.
  bool all_local(const std::vector<std::string>& next);
  bool p2p_ready(const std::vector<std::string>& next);  // every hop has a P2P pair up
  bool persist_and_replicate(const std::string& id, const uint8_t* host, uint64_t n, uint32_t crc, uint64_t term,
                             const std::vector<std::string>& next, int* downstream, std::string* err);
  void add_suspect(const std::string& id);
  // For the native gRPC chain (dfs_chunkserver): a client's shared-memory slot
  // [off, off+len) (nullptr + *err when it is not mappable here), the replication engine,
  // and one replica pushed to a same-node `addr` over it (replicas written, 0 = failed).
  uint8_t* map_client_shm(const std::string& path, uint64_t off, uint64_t len, std::string* err) {
    return map_shm(path, off, len, err);
  }
  ReplicationEngine* replication() const { return repl_; }
  int replicate_to(const std::string& addr, const std::string& id, uint32_t crc, uint64_t term, const uint8_t* host,
                   uint64_t n, bool heal) {
    return replicate_one(addr, id, crc, term, ShmSrc{}, host, n, heal);
  }
  // Heal / balancer / shuffle copy (master REPLICATE command; reference chunkserver.rs:462-499)
  // of a block held here to same-node `targets`, payload over the replication engine (HBM ->
  // HBM on device transports), descriptor on the peers' fast-path sockets. Returns the
  // replicas written; a target that is not reachable this way counts 0 (the caller falls
  // back to gRPC for it).
  int replicate_block(const std::string& id, const std::vector<std::string>& targets, uint64_t term,
                      std::vector<std::string>* done);
  // Blocks received as heal copies since the last call (reported to the masters as new
  // locations by the heartbeat).
  std::vector<std::string> drain_healed();
  void note_rid(const std::string& rid);  // record a served request id (recent_request_ids)
  // Test hook: the next `n` REPL descriptors are dropped on the way out.
  void debug_drop_descriptors(int n) { drop_descriptors_ += n; }
  void set_self_host(const std::string& host);  // our advertised host: same-host peer detection
  void set_self_addr(const std::string& addr);  // our advertised address (EC targets that are us)

  // Device gather of EC shards into this GPU (degraded reads, RECONSTRUCT_EC_SHARD): each
  // shard held here is pinned in place, each held by a same-node peer is pushed over the
  // replication engine into an ephemeral block here. ptrs[i] = device pointer (nullptr:
  // lost, skipped or unreachable). The destructor unpins and drops what it gathered.
  struct EcGather {
    FastPathServer* fp = nullptr;
    std::vector<const uint8_t*> ptrs;
    std::vector<std::string> pinned, temps;
    int unreachable = 0;  // shards that exist but could not be gathered over the engine
    uint64_t len = 0;     // shard length (given, or the length the gathered shards agree on)
    ~EcGather();
  };
  bool ec_gather(const std::string& id, const std::vector<std::string>& locations, uint64_t shard_len, int skip,
                 int want, EcGather* g, std::string* err);

 private:
  struct Peer {
    int rank = -1;
    std::string name;
    std::mutex mu;
    std::vector<int> idle;  // pooled connections to the peer's fast-path socket
  };
  void accept_loop();
  void serve(int fd);
  // Maps the client arena and checks [off, off+len) lies inside it (overflow-safe).
  uint8_t* map_shm(const std::string& path, uint64_t off, uint64_t len, std::string* err);
  struct ShmSrc {
    std::string path;  // client arena the block came from (empty: HBM-only, e.g. P2P-received)
    uint64_t off = 0, len = 0;
  };
  // Fan block `id` out to every address in `next` (all same-host); *replicas = replicas
  // written downstream. `host` is the block in host memory when there is one (shm slot).
  void replicate(const std::string& id, uint32_t crc, uint64_t term, const std::vector<std::string>& next,
                 const ShmSrc& src, const uint8_t* host, uint64_t n, int* replicas,
                 const StagedSource* staged = nullptr);
  int replicate_one(const std::string& addr, const std::string& id, uint32_t crc, uint64_t term, const ShmSrc& src,
                    const uint8_t* host, uint64_t n, bool heal = false, const StagedSource* staged = nullptr,
                    bool ephemeral = false);
  bool is_self(const std::string& addr) const;
  // op 7 / op 8 / op 9 bodies (answered on fd)
  bool ec_write(int fd, const uint8_t* body, const uint8_t* end);
  bool ec_read(int fd, const uint8_t* body, const uint8_t* end);
  bool push_block(int fd, const uint8_t* body, const uint8_t* end);
  // Pipelined head write of a large replicated block; false = not applicable (the caller
  // takes the stage-then-forward path), true = answered on `fd` (*sent = write result).
  bool write_sliced(int fd, const std::string& id, const uint8_t* host, uint64_t len, uint32_t crc, uint64_t term,
                    const std::vector<std::string>& next, const ShmSrc& src, bool* sent);
  bool exchange_with(struct Peer* p, const std::vector<uint8_t>& req, std::vector<uint8_t>* resp);
  Peer* local_peer(const std::string& addr);

  ChunkStore* store_;
  std::string name_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> term_{0};
  std::thread acceptor_;
  std::mutex mu_;
  int live_workers_ = 0;  // detached per-connection threads still running (guarded by mu_)
  std::condition_variable workers_cv_;
  std::vector<int> conns_;
  struct Mapping {
    uint8_t* p = nullptr;
    uint64_t size = 0;
    bool registered = false;  // hipHostRegister'ed for direct DMA
  };
  std::unordered_map<std::string, Mapping> maps_;
  int pending_regs_ = 0;  // arena registrations in flight (mu_); stop() waits for them
  std::vector<Mapping> retired_;
  std::vector<std::string> suspects_;
  std::vector<std::string> healed_;  // heal copies received (mu_), drained by the heartbeat
  std::vector<std::string> recent_rids_;  // ring of the last kRecentRids request ids (mu_)
  size_t recent_pos_ = 0;
  FpStats st_;
  IoPool pool_{16, 30000, "fp-fanout"};  // replica fan-out helpers: reused threads, none created per write
  ReplicationEngine* repl_ = nullptr;
  std::atomic<int> drop_descriptors_{0};
  std::mutex peers_mu_;
  std::unordered_map<std::string, std::unique_ptr<Peer>> peers_;
  std::string self_host_;
  std::string self_addr_;
  std::atomic<uint64_t> tmp_seq_{0};
};

}  // namespace dfs
