// ChunkServerService on the native gRPC server (reference handlers:
// dfs/chunkserver/src/chunkserver.rs:721-1088). The data RPCs run in C++ without the GIL:
//   WriteBlock   — fencing, CRC verify, durable write; replicas fanned out over the P2P
//                  transport when every next server is a same-host rank with a pair up;
//   ReadBlock    — verified range read (K3 on HBM) straight into the response buffer;
//   ReplicateBlock (payload inline, end of chain) — fencing, verify, durable write.
// Everything else — chains leaving the host, shm-in-gRPC requests, corruption needing
// recovery from a replica, P2P descriptors — is handed to the Python service (the same
// handlers the grpcio server ran), so no reference semantics are duplicated.
#pragma once
#include <atomic>
#include <functional>
#include <memory>
#include <string>

#include "chunk_store.h"
#include "fastpath.h"
#include "grpc_server.h"

namespace dfs {

struct CsGrpcStats {
  uint64_t native_writes = 0, native_reads = 0, native_replicates = 0, fallbacks = 0;
};

class NativeChunkService {
 public:
  using Fallback = std::function<GrpcReply(const GrpcCall&)>;
  NativeChunkService(ChunkStore* store, FastPathServer* fp, Fallback fallback);
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

  ChunkStore* store_;
  FastPathServer* fp_;
  Fallback fallback_;
  std::shared_ptr<class ReplyPool> replies_, requests_;
  std::atomic<uint64_t> writes_{0}, reads_{0}, replicates_{0}, fallbacks_{0};
};

}  // namespace dfs
