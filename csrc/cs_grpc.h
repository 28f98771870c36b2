// ChunkServerService on the native gRPC server (reference handlers:
// dfs/chunkserver/src/chunkserver.rs:721-1088). The data RPCs run in C++ without the GIL:
//   WriteBlock   — fencing, CRC verify, durable write; replicas fanned out over the P2P
//                  transport when every next server is a same-host rank with a pair up;
//   ReadBlock    — verified range read (K3 on HBM) straight into the response buffer;
//   ReplicateBlock (payload inline, end of chain) — fencing, verify, durable write.
// In the native chunkserver (dfs_chunkserver, set_native) the rest is native too: the
// reference's store-and-forward chain for hops without a P2P pair (chunkserver.rs:777-829,
// 1039-1077: local write, then ReplicateBlock{data, next_servers[1..]} to next_servers[0],
// downstream failures counted, not returned), ReplicateBlock descriptors of payloads on the
// replication engine and heal copies, shm-in-gRPC writes and reads, and a corrupt full read
// recovered synchronously from another replica before it is answered (chunkserver.rs:913-949).
// Inside the Python shell those cases are handed to its service instead.
#pragma once
#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "chunk_store.h"
#include "fastpath.h"
#include "grpc_server.h"

namespace dfs {

struct CsGrpcStats {
  uint64_t native_writes = 0, native_reads = 0, native_replicates = 0, fallbacks = 0;
  uint64_t grpc_forwards = 0, grpc_forward_failures = 0, recoveries = 0, shm_writes = 0, shm_reads = 0;
};

class CsAgent;
class GrpcChannelPool;

class NativeChunkService {
 public:
  using Fallback = std::function<GrpcReply(const GrpcCall&)>;
  NativeChunkService(ChunkStore* store, FastPathServer* fp, Fallback fallback);
  // Serve every case natively (no fallback): chain hops leave over `peers`, corrupt blocks
  // are recovered through `agent`.
  void set_native(CsAgent* agent, std::shared_ptr<GrpcChannelPool> peers);
  GrpcReply handle(const GrpcCall& call);
  CsGrpcStats stats() const;
  // GrpcServer body allocator (registered request buffers); nullptr = default body.
  std::shared_ptr<uint8_t> request_buffer(size_t n);
  static constexpr size_t kRequestBufferMin = 64 << 10;

 private:
  GrpcReply write_block(const GrpcCall& call, bool* handled);
  GrpcReply read_block(const GrpcCall& call, bool* handled);
  GrpcReply replicate_block(const GrpcCall& call, bool* handled);
  bool fence(uint64_t term, std::string* msg);
  // the reference chain hop: `id` (from `data`, or read back from the store) to next[0] with
  // next[1..]; returns the replicas written downstream (0 on failure, which is logged)
  int forward(const std::string& id, const uint8_t* data, uint64_t n, const std::vector<std::string>& next,
              uint32_t crc, uint64_t term, bool heal, const std::string& rid);
  // staged (or, on the host store, written) block: persist it while the chain forwards it
  GrpcReply store_and_forward(const std::string& id, const uint8_t* data, uint64_t n,
                              const std::vector<std::string>& next, uint32_t crc, uint64_t term, bool heal,
                              const std::string& rid, int* replicas, std::string* err, bool staged);

  ChunkStore* store_;
  FastPathServer* fp_;
  Fallback fallback_;
  std::shared_ptr<class ReplyPool> replies_, requests_;
  std::atomic<uint64_t> writes_{0}, reads_{0}, replicates_{0}, fallbacks_{0};
  std::atomic<uint64_t> grpc_forwards_{0}, grpc_forward_failures_{0}, recoveries_{0}, shm_writes_{0}, shm_reads_{0};
  CsAgent* agent_ = nullptr;
  std::shared_ptr<GrpcChannelPool> peers_;
  bool native_ = false;
};

}  // namespace dfs
