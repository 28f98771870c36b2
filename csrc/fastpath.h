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
// Scope: WriteBlock without downstream replicas (the last hop of any chain, RF=1) and
// ReadBlock. Anything else — chain forwarding, corruption needing recovery, fenced or
// malformed requests — is answered with a status telling the client to use the regular
// gRPC service, which keeps every semantic of the reference (fencing, recovery,
// replicas_written) in one place.
//
// Wire format (little endian), one request/response pair at a time per connection:
//   request  = u32 body_len | u8 op | body
//     op 1 WRITE: u64 term | u32 crc | u64 shm_off | u64 len | u16 id_len id | u16 path_len path
//     op 2 READ : u64 offset | u64 length | u64 shm_off | u64 shm_cap | u16 id_len id | u16 path_len path
//   response = u32 body_len | u8 status | u64 total | u64 bytes | u16 msg_len msg
#pragma once
#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "chunk_store.h"

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
  FpStats stats();

 private:
  void accept_loop();
  void serve(int fd);
  uint8_t* map_shm(const std::string& path, uint64_t need, std::string* err);

  ChunkStore* store_;
  std::string name_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> term_{0};
  std::thread acceptor_;
  std::mutex mu_;
  std::vector<std::thread> workers_;
  std::vector<int> conns_;
  struct Mapping {
    uint8_t* p = nullptr;
    uint64_t size = 0;
  };
  std::unordered_map<std::string, Mapping> maps_;
  std::vector<std::string> suspects_;
  FpStats st_;
};

}  // namespace dfs
