// RCCL-over-xGMI chain replication (reference: synchronous store-and-forward gRPC chain,
// dfs/chunkserver/src/chunkserver.rs:777-819,1039-1077).
//
// One process per GPU = one ChunkServer = one RCCL rank. RCCL p2p needs matched
// send/recv posts, while a DFS picks a fresh (src, dst) pair per block with many blocks
// in flight. Mapping that onto ONE communicator invites ordering deadlocks (A sends to B
// while B sends to A). Instead every ordered pair (a -> b) gets its own 2-rank
// communicator and stream, so traffic on a communicator is unidirectional and strictly
// FIFO: the sender stamps each transfer with a per-pair sequence number and the
// receiver posts ncclRecv in sequence order (the gRPC descriptor carries the seq).
// Communicator bootstrap: unique ids through a shared rendezvous directory, pairs
// initialised in a global lexicographic order (deadlock-free, like ordered locking).
// Every wait is bounded: communicators are nonblocking (init and lazily connected p2p
// channels are polled against a deadline), each pair is proven with a warm-up transfer,
// and RCCL is enabled only if every rank brought up every pair (published through the
// rendezvous directory) — otherwise all ranks fall back together. On a later timeout the
// pair is aborted and the caller falls back to the shared-memory / gRPC data path.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "chunk_store.h"

namespace dfs {

class RcclEngine {
 public:
  RcclEngine(ChunkStore* store, int rank, int world, std::string rendezvous_dir, int timeout_ms);
  ~RcclEngine();
  bool init(std::string* err);
  bool ready() const { return ready_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  bool pair_ok(int src, int dst) const;

  // Sender side: enqueue the block on the (rank -> peer) communicator. Returns seq >= 0.
  int64_t send(int peer, const std::string& id, uint64_t* size, std::string* err);
  bool wait_send(int peer, int64_t seq, std::string* err);
  // Receiver side: post the recv for `seq` in order, then verify + persist + index.
  WriteResult recv(int src, int64_t seq, const std::string& id, uint64_t size, uint32_t expected_crc,
                   bool persist_now = true);
  void abort_pair(int src, int dst);
  uint64_t bytes_sent() const { return bytes_sent_; }
  uint64_t bytes_recv() const { return bytes_recv_; }

 private:
  struct Pair {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    bool broken = false;
    std::mutex mu;
    std::condition_variable cv;
    int64_t next_seq = 0;  // sender: next seq to assign; receiver: next seq to post
    struct Pending {
      hipEvent_t ev;
      std::string id;
    };
    std::map<int64_t, Pending> pending;  // sender: in-flight sends
  };
  Pair* pair(int src, int dst);
  bool init_pairs(std::string* err);
  bool wait_event(hipEvent_t ev, Pair* p);

  ChunkStore* store_;
  int rank_, world_;
  std::string dir_;
  int timeout_ms_;
  bool ready_ = false;
  std::map<std::pair<int, int>, std::unique_ptr<Pair>> pairs_;
  std::atomic<uint64_t> bytes_sent_{0}, bytes_recv_{0};
};

}  // namespace dfs
